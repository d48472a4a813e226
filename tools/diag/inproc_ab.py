"""Interleaved in-process A/B on the bench (one box, one process, alternating arms):

    python tools/diag/inproc_ab.py ARMSET ROUNDS [bench args ...]

ARMSET: layout      - flat parameter layout: model.grad_order vs reverse registration order
        gemm_outer  - the outer-product GEMM kernel on vs off (gm_gemm_set_form bit 9)
        pipe        - k_conv_igemm_ut main loop: PIPE 2 (default) vs PIPE 0 (gm_conv_set_pipe)
        bind        - resident batches bound as graph inputs vs copied into the static buffers (bench args)
        wgrad_batch - weight-gradient launches handed to the side stream in batches of 8 / 4 / 2
        stem_wgrad  - the stem weight gradient forming its dy from the BN + pool backward's operands
                      (vtrunk.FUSED_STEM_WGRAD) vs the BN apply pass writing dy
        dres        - the block-output BN backward without dres (vtrunk.IDT_MASKED_ADDEND + DS_DZ_LINK)
                      vs writing it
        ds1x1       - the 1x1 / s2 downsample forwards on k_gemm_ring (gathered A rows) vs k_conv_igemm_ut
        bnchunk     - the single-launch BN backward over view chunks of <= 112 / 56 MB of x + dy vs one launch
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def arms(name):
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import model as M
    if name == "layout":
        orig = {c: c.grad_order for c in (M.MMTM_MVCNN, M.MMTM_MVCNN_N)}

        def setl(on):
            for c, f in orig.items():
                if on:
                    c.grad_order = f
                elif hasattr(c, "grad_order"):
                    del c.grad_order
        return [("grad_order", lambda: setl(True)), ("reverse_registration", lambda: setl(False))]
    if name == "gemm_outer":
        def setg(form):
            L.check(L.load().gm_gemm_set_form(form), "gemm form")
        return [("outer_on", lambda: setg(1)), ("outer_off", lambda: setg(1 | 512))]
    if name == "pipe":
        def setp(p):
            L.check(L.load().gm_conv_set_pipe(p), "pipe")
        return [("pipe2", lambda: setp(-1)), ("pipe0", lambda: setp(0))]
    if name == "stem_wgrad":
        from greedy_multimodal_learning_amd import vtrunk

        def setw(on):
            vtrunk.FUSED_STEM_WGRAD = on
        return [("fused", lambda: setw(True)), ("apply_pass", lambda: setw(False))]
    if name == "wgrad_batch":
        from greedy_multimodal_learning_amd import vtrunk

        def setb(n):
            vtrunk.WGRAD_BATCH = n
        return [(f"batch{n}", (lambda n=n: setb(n))) for n in (8, 4, 2)]
    if name == "dres":
        from greedy_multimodal_learning_amd import vtrunk

        def setd(on):
            vtrunk.IDT_MASKED_ADDEND = vtrunk.DS_DZ_LINK = on
        return [("no_dres", lambda: setd(True)), ("dres", lambda: setd(False))]
    if name == "bnchunk":
        from greedy_multimodal_learning_amd import vtrunk

        def setc(n):
            vtrunk.BN_BWD_CHUNK_BYTES = n
        return [("chunk112", lambda: setc(112 << 20)), ("one_launch", lambda: setc(0)),
                ("chunk56", lambda: setc(56 << 20))]
    if name == "ds1x1":
        def setm(m):
            L.check(L.load().gm_conv_set_1x1_gemm(m), "1x1 gemm")
        return [("ring_s2", lambda: setm(2)), ("igemm_s2", lambda: setm(1))]
    if name == "bind":
        return [("bound", lambda: None), ("copied", lambda: None)]
    raise SystemExit(f"unknown arm set {name}")


def main():
    name, rounds = sys.argv[1], int(sys.argv[2])
    extra = sys.argv[3:] or ["--no-cpu-baseline", "--steps", "40"]
    import bench
    sets = arms(name)
    for r in range(rounds):
        for arm, apply in sets:
            apply()
            print(f"round {r} {arm}", flush=True)
            sys.argv = ["bench.py"] + extra + (["--copy-inputs"] if arm == "copied" else [])
            bench.main()
    sets[0][1]()


if __name__ == "__main__":
    main()
