"""Latency of the MMTM FC GEMMs (k_gemm_f32 via gm_gemm_f32) on the C2 site shapes, in
isolation: the forward joint FC [B, 2C] x [2C, C'] (+bias, ReLU), the excite FC pair
[B, C'] x [C', C] (+bias, sigmoid) and the backward weight-gradient problems, for each
site (C = 128, 256, 512 per modality, ratio 4 as in MMTM_MVCNN), B = 64.  Interleaved
rounds of the GEMM forms (gm_gemm_set_form 0-3) in one process; HIP events on
the launch stream, 50 launches per timing.

    python tools/gemm_probe.py                 # event timing (host-launch-bound: Python ctypes)
    python tools/gemm_probe.py report TRACE    # kernel durations per (form, case) from a rocprofv3
                                               # kernel trace of the run above
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def problems(dev, B, C, ratio=4):
    from greedy_multimodal_learning_amd.ops import ONES, Op
    C2 = 2 * C
    Cz = int(2 * C2 / ratio)
    f = dict(device=dev, dtype=torch.float32)
    sq, w_sq, b_sq = torch.randn(B, C2, **f), torch.randn(Cz, C2, **f), torch.randn(Cz, **f)
    z, w_v, b_v = torch.randn(B, Cz, **f), torch.randn(C, Cz, **f), torch.randn(C, **f)
    e_v, e_s = torch.empty(B, C, **f), torch.empty(B, C, **f)
    da, gw, gb, dz = torch.randn(B, C, **f), torch.empty(C, Cz, **f), torch.empty(C, **f), torch.empty(B, Cz, **f)
    zj = torch.empty(B, Cz, **f)
    return {
        "joint": [dict(M=B, N=Cz, segs=[(C2, Op(sq, C2, 1), Op(w_sq, 1, C2))], C=zj, ld_c=Cz, bias=b_sq, act=1)],
        "excite": [dict(M=B, N=C, segs=[(Cz, Op(z, Cz, 1), Op(w_v, 1, Cz))], C=e, ld_c=C, bias=b_v, act=2)
                   for e in (e_v, e_s)],
        "bwd_w": [dict(M=C, N=Cz, segs=[(B, Op(da, 1, C), Op(z, Cz, 1))], C=gw, ld_c=Cz),
                  dict(M=1, N=C, segs=[(B, ONES, Op(da, C, 1))], C=gb, ld_c=C),
                  dict(M=B, N=Cz, segs=[(C, Op(da, C, 1), Op(w_v, Cz, 1))], C=dz, ld_c=Cz, mask=z, ld_mask=Cz)],
    }


FORMS = (1, 257, 0, 256, 4)
ROUNDS, REPS = 3, 53


def case_keys():
    return [(C, k) for C in (128, 512) for k in ("joint", "excite", "bwd_w")]


def report(trace):
    import csv
    rows = [r for r in csv.DictReader(open(trace)) if "k_gemm_f32" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    res, i = {}, 0
    for _ in range(ROUNDS):
        for f in FORMS:
            for key in case_keys():
                chunk = sorted(dur[i + 3:i + REPS])
                i += REPS
                res.setdefault((key, f), []).append(chunk[len(chunk) // 2])
    assert i == len(dur), (i, len(dur))
    for (key, f), ts in sorted(res.items()):
        ts.sort()
        print(f"C={key[0]:4d} {key[1]:7s} form={f:3d}: kernel median {ts[len(ts) // 2]:6.2f} us")


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "report":
        return report(sys.argv[2])
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import ops
    dev = torch.device("cuda:0")
    lib = L.load()
    cases = {(C, k): v for C in (128, 512) for k, v in problems(dev, 64, C).items()}
    assert list(cases) == case_keys()
    # a trivial torch kernel for the launch floor
    t = torch.empty(16, device=dev)
    cases[(0, "fill")] = t
    res = {}
    for _ in range(ROUNDS):
        for nw in FORMS:
            L.check(lib.gm_gemm_set_form(nw), "set_form")
            for key, probs in cases.items():
                run = (lambda: probs.fill_(1.0)) if key[1] == "fill" else (lambda: ops.gemm(probs, dev))
                for _ in range(REPS - 50):
                    run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(50):
                    run()
                e1.record()
                torch.cuda.synchronize()
                res.setdefault((key, nw), []).append(e0.elapsed_time(e1) / 50 * 1e3)
    for (key, nw), ts in sorted(res.items()):
        ts.sort()
        print(f"C={key[0]:4d} {key[1]:7s} form={nw}: median {ts[len(ts) // 2]:7.2f} us per launch")


if __name__ == "__main__":
    main()
