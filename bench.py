#!/usr/bin/env python3
"""Benchmark of the balanced multi-modal training step on MI355X.

Metric (BASELINE.json): multi-view images/sec + step ms, ModelNet40 2-view
MVCNN+MMTM.  One step = forward + blend_loss + backward (+ RCCL gradient
all-reduce when N > 1) + conditional-learning-speed gate (per-branch norm pass
fused with the SGD update, one host sync for the decision) on one synthetic
ModelNet40-shaped batch [B, 2, 3, 224, 224] resident in HBM.  Workload: config
C2 (B = 64 per GPU, bf16 trunk, training_guided gating: eps 0.01, window 5,
gate unlocked).  N > 1: weak scaling, 64 per GPU (config C3 = 512 at 8 GPUs).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
       torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)
"""
import argparse
import json
import os
import sys
import time

# A data-parallel rank runs more concurrent streams (main chain, weight gradients, the gradient
# bucket stream, RCCL's own) than HIP's default 4 hardware queues.  Streams that share a queue
# serialise: a long RCCL kernel would hold back every launch queued behind it on that queue
# (tests/test_gpu_rccl_residency.py measured a 393 ms stall behind a CU-holding kernel on a shared
# queue).  Set before the HIP runtime initialises; an operator's value wins.
if int(os.environ.get("WORLD_SIZE", "1")) > 1:
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_PARAMS = 23_773_008  # C2 (MMTM_MVCNN)
WORKLOADS = {
    "C2": dict(views=2, trunk="resnet18", batch=64, desc="C2: 2-view MVCNN(ResNet-18 x2)+MMTM x3"),
    "C4": dict(views=4, trunk="resnet18", batch=64, desc="C4: 4 synthetic modalities (ResNet-18 x4)+N-way MMTM x3"),
    "C5": dict(views=12, trunk="resnet50", batch=32, desc="C5: 12-view MVCNN (ResNet-50 x12)+N-way MMTM x3"),
}
HBM_PEAK_GBS = 8000.0
MFMA_PEAK_TFS = 2500.0  # dense bf16 (MI355X_MICROARCH.md)
MFMA_F32_PEAK_TFS = 157.3  # f32-input MFMA = the f32 vector rate (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="C2", choices=["C2", "C4", "C5"],
                    help="C2: 2-view ResNet-18 (BASELINE metric); C4: 4 ResNet-18 modalities; "
                         "C5: 12 ResNet-50 views (BASELINE.json configs)")
    ap.add_argument("--batch", type=int, default=None,
                    help="per-GPU batch (multi-view objects); default 64 (C2, C4) / 32 (C5)")
    ap.add_argument("--size", type=int, default=224)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--curate-all", action="store_true",
                    help="A/B: open a curation window longer than the run on the on-device gate before "
                         "the timed steps, so every timed step is a curated one")
    ap.add_argument("--miopen-find", action="store_true", help="torch.backends.cudnn.benchmark=True")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--eager", action="store_true", help="no hipGraph capture of the step")
    ap.add_argument("--copy-inputs", action="store_true",
                    help="copy each step's resident batch into the engine's static input buffers (the pre-r06 "
                         "form) instead of binding the two resident batches as graph inputs")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic_group_sumsq.json"))
    ap.add_argument("--conv-traffic-file", default=os.path.join(ROOT, "profiles", "r06g_traffic_conv_family.json"))
    ap.add_argument("--mmtm-traffic-file", default=os.path.join(ROOT, "profiles", "r03_traffic_mmtm.json"))
    ap.add_argument("--profile", action="store_true",
                    help="steps only (no roofline / cpu_baseline measurements): for rocprofv3 runs")
    return ap.parse_args()


def cpu_baseline(seconds, size):
    """Oracle (port) of the reference step on the host cores: config C1's
    shape (B = 4) for ~`seconds`, then B = 64 (the GPU workload's batch) for ten timed steps.
    Threads: torch's intra-op pool as the box configures it (OMP_NUM_THREADS = the CPU
    share of the job); os.cpu_count() reports the whole machine and is stated beside it."""
    from oracle import model_ref, step_ref, gating_ref, weights

    def run(B, secs, max_steps):
        torch.manual_seed(0)
        m = weights.apply_to_module(model_ref.MMTM_MVCNN_Ref(), seed=0)
        gate = gating_ref.BDRState(0.01, 5, starting_epoch=1)
        gate.on_epoch_begin(1)
        step = step_ref.RefStep(m, lr=0.1, gate=gate)
        g = torch.Generator().manual_seed(0)
        x = torch.randn(B, 2, 3, size, size, generator=g)
        y = torch.randint(0, 40, (B,), generator=g)
        step(x, y)  # warm-up
        n, t0 = 0, time.perf_counter()
        while True:
            step(x, y)
            n += 1
            dt = time.perf_counter() - t0
            if dt >= secs or n >= max_steps:
                break
        return n, dt

    th = torch.get_num_threads()
    n4, dt4 = run(4, seconds, 200)
    n64, dt64 = run(64, float("inf"), 10)  # ten timed steps at the bench batch (a median of 10)
    return {"value": round(n4 * 4 * 2 / dt4, 3), "unit": "view-images/s", "cores": th,
            "kind": "port", "ms_per_step": round(1e3 * dt4 / n4, 2),
            "b64": {"value": round(n64 * 64 * 2 / dt64, 3), "ms_per_step": round(1e3 * dt64 / n64, 1),
                    "steps": n64},
            "sample": f"{n4} oracle steps at B=4 (config C1 shape) + {n64} at B=64 (the bench batch); fp32 "
                      f"torch-CPU restatement of forward+blend_loss+backward+compute_BDR+SGD, two-view "
                      f"{size}x{size}; {th} threads (the job's CPU share; {os.cpu_count()} CPUs visible)"}


def time_trunk_convs(B, dev, dtype="bf16", G=2, arch="resnet18"):
    """Roofline of the dominant kernel family, the trunk convolutions: forward, input-
    and weight-gradient launches of every trunk shape of one view at the step's batch
    (tools/trunk_table.py; HIP events on the launch stream behind a device sleep; the
    launches rotate over more operand bytes than the 256 MiB Infinity Cache holds)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import trunk_table
    flops, secs, launches, _ = trunk_table.measure_family(B, dev, dtype=dtype, G=G, arch=arch)
    return flops, secs, launches


def conv_roofline(conv, traffic, dtype="bf16", workload="C2"):
    """The `roofline` object of the dominant kernel family (the trunk convolutions)."""
    if dtype == "fp32":
        if conv is None:
            return None
        flops, secs, launches = conv
        return {"kernel": "trunk convolutions, reference precision (k_conv_f32: exact-f32 MFMA "
                          "v_mfma_f32_32x32x2_f32 implicit GEMM fwd / input grad / weight grad; every trunk "
                          "shape of one view at the step's batch, tools/trunk_table.py)",
                "bound": "mfma", "achieved": round(flops / secs / 1e12, 2), "peak": MFMA_F32_PEAK_TFS,
                "unit": "TFLOP/s", "frac": round(flops / secs / 1e12 / MFMA_F32_PEAK_TFS, 4), "traffic": None,
                "alg_flops_per_launch": round(flops / launches), "avg_launch_us": round(secs / launches * 1e6, 2)}
    flops, secs, launches = conv
    what = {"C2": "every ResNet-18 trunk shape, both views per launch (the view-batched trunk)",
            "C4": "every ResNet-18 trunk shape, the 4 views per launch (the view-batched trunk)",
            "C5": "every ResNet-50 trunk shape, the 12 views per launch (the view-batched trunk)"}[workload]
    return {"kernel": "trunk convolutions (bf16 MFMA: k_conv_stem pixel-pair stem, k_conv_rw layer-1 "
                      "resident-weight, k_conv_h9 3x3 halo, k_conv_igemm_ut strided fwd + input grad, "
                      "k_gemm_ring 1x1/s1 fwd + input grad, k_wgrad_ring / k_wgrad_halo64 / k_conv_wgrad4 + "
                      "k_wgrad_sum weight grad; " + what + " at the step's batch, tools/trunk_table.py)",
            "bound": "mfma", "achieved": round(flops / secs / 1e12, 1), "peak": MFMA_PEAK_TFS, "unit": "TFLOP/s",
            "frac": round(flops / secs / 1e12 / MFMA_PEAK_TFS, 4), "traffic": traffic,
            "alg_flops_per_launch": round(flops / launches), "avg_launch_us": round(secs / launches * 1e6, 2)}


def time_mmtm_reduce(dev, B=256, reps=20):
    """HBM roofline of the MMTM squeeze (k_colreduce_nhwc via gm_mmtm_spatial_reduce) at the
    north-star batch 256, site s2, the launch MMTM_mitigate.forward issues; launches rotate
    over 4 distinct activation pairs (411 MB, more than the 256 MiB Infinity Cache) so each
    reads HBM (tools/mmtm_probe.py).  Returns (algorithmic bytes, seconds) per launch."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import mmtm_probe
    nbytes, secs, _ = mmtm_probe.measure(dev, B, pairs=4, reps=reps)
    return nbytes, secs


def time_group_sumsq(step, n):
    """Average duration of the fused norms+SGD launch, HIP events on its stream; a
    leading ~20 ms device sleep keeps the GPU busy while the host enqueues, so the
    events bracket kernel time, not host launch latency."""
    stream = torch.cuda.current_stream()
    torch.cuda.synchronize()
    torch.cuda._sleep(50_000_000)
    evs = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        step.norms.sums(grad_scale=1.0 / step.world, lr=step.lr)
        e1.record(stream)
        evs.append((e0, e1))
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in evs) / n / 1e3


def spawn_ranks(n, script, argv, poll_s=0.2):
    """`--gpus N` without a launcher: start N rank processes of `script` (one per GPU,
    RANK = LOCAL_RANK = i, rendezvous on 127.0.0.1) and return the job's exit code.
    Runs BEFORE anything touches the GPU (this process never initialises HIP: the
    ranks are children, not an exec).  If one rank fails the others are terminated,
    so a rank stuck in a collective cannot hang the job.  Only rank 0 prints the line."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:
                    q.terminate()
        time.sleep(poll_s)
    return rc


def dp_info(step, dist_on):
    """What the communicator saw: the backend and world size as the process
    groups report them, the gradient buckets in all-reduce order and whether the all-reduces were
    captured inside the step graph - so the driver's N > 1 record proves N RCCL ranks took part."""
    info = {"dist_backend": None, "world_size": 1, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}
    if not dist_on:
        return info
    pg = step.pg
    info.update(dist_backend=dist.get_backend(pg), world_size=dist.get_world_size(pg),
                collectives_in_graph=bool(step.graph_collectives),
                capture_group_size=(dist.get_world_size(step._capture_pg) if step._capture_pg is not None
                                    else None),
                nccl_max_nchannels=os.environ.get("NCCL_MAX_NCHANNELS"))
    if step.buckets is not None:
        info["buckets_mb"] = [round((e - s) * 4 / 2 ** 20, 2) for s, e, _ in step.buckets.buckets]
    return info


def main():
    a = parse()
    if "RANK" not in os.environ and a.gpus > 1:
        sys.exit(spawn_ranks(a.gpus, os.path.abspath(__file__), sys.argv[1:]))
    dist_on = "RANK" in os.environ and int(os.environ.get("WORLD_SIZE", "1")) > 1
    if int(os.environ.get("WORLD_SIZE", "1")) != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={os.environ.get('WORLD_SIZE', '1')}", file=sys.stderr)
        sys.exit(2)
    if dist_on:
        # rehearsal knobs (not used by the driver): gloo, and every rank on cuda:0, run the
        # N-rank code path on a one-GPU box
        from greedy_multimodal_learning_amd.engine import bound_rccl_channels
        bound_rccl_channels()  # before any communicator exists: the engine reserves that many CUs
        dist.init_process_group(os.environ.get("GM_BENCH_DIST_BACKEND", "nccl"))
        rank, world = dist.get_rank(), dist.get_world_size()
        # (ranks sharing one GPU are found by the engine: gm_set_residency's `sharers`)
        local = 0 if os.environ.get("GM_BENCH_SAME_DEVICE") == "1" else int(os.environ.get("LOCAL_RANK", "0"))
    else:
        rank, world, local = 0, 1, 0
    torch.cuda.set_device(local)
    torch.backends.cudnn.benchmark = a.miopen_find
    dev = torch.device("cuda", local)
    from greedy_multimodal_learning_amd import build
    build.build()  # no-op when up to date
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Strong
    from greedy_multimodal_learning_amd.engine import BalancedStep

    torch.manual_seed(0)
    WL = WORKLOADS[a.workload]
    V = WL["views"]
    if a.workload == "C2":
        model = MMTM_MVCNN().to(dev)
        bnames, mnames = ["net_view_0", "net_view_1"], ["visual", "skeleton"]
    else:
        from greedy_multimodal_learning_amd.model import MMTM_MVCNN_N
        model = MMTM_MVCNN_N(num_views=V, trunk=WL["trunk"]).to(dev)
        bnames, mnames = model.branch_names(), model.mmtm_names()
    gate = Bias_Mitigation_Strong(epsilon=0.01, curation_windowsize=5, branchnames=bnames, starting_epoch=1,
                                  MMTMnames=mnames)
    cdt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    step = BalancedStep(model, lr=0.1, gate=gate, compute_dtype=cdt, channels_last=True,
                        process_group=dist.group.WORLD if dist_on else None, graphs=not a.eager,
                        branchnames=bnames, MMTMnames=mnames)
    step.on_epoch_begin(1)
    B = a.batch if a.batch is not None else WL["batch"]
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    xdt = cdt
    # HBM layout of a batch: view-major, channels-last [V][B][H][W][3], exposed to the
    # model as the reference's [B, V, 3, H, W] (a permuted view); each view's slice is
    # then a dense channels_last image batch the first convolution reads directly.
    def batch():
        buf = torch.randn(V, B, a.size, a.size, 3, device=dev, generator=g).to(xdt)
        return buf.permute(1, 0, 4, 2, 3)
    xs = [batch() for _ in range(2)]
    ys = [torch.randint(0, 40, (B,), device=dev, generator=g) for _ in range(2)]
    if not dist_on and not a.copy_inputs:
        # the two resident batches are the graphs' static inputs (BalancedStep.bind_batches: a
        # loader's double buffer) - no per-step copy into the engine's own buffers; under data
        # parallelism the engine keeps one graph per curation setting (rank-identical keys) and copies
        step.bind_batches(*zip(xs, ys))
    for i in range(a.warmup):
        step(xs[i % 2], ys[i % 2])
    torch.cuda.synchronize()
    curation_steps = 0
    if a.curate_all and step.device_gate:
        st = step.gate_struct()
        st.curation_mode, st.curation_step, st.window, st.unlock = 1, 0, 1 << 30, 1
        st.caring = st.caring if st.caring >= 0 else 0
        step.set_gate_struct(st)
        torch.cuda.synchronize()
    n_cur0 = step.sync_gate()["n_curated"] if step.device_gate else 0
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        if not step.device_gate:  # host gate: the flags are current after every step
            curation_steps += int(step.flags.curation_mode)
        step(xs[i % 2], ys[i % 2])
    torch.cuda.synchronize()
    if step.device_gate:  # on-device gate: no per-step sync; read its counter once
        curation_steps = step.sync_gate()["n_curated"] - n_cur0
    if dist_on:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if dist_on:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    ms = 1e3 * elapsed / a.steps
    loss = float(step.last_loss)
    # roofline kernel: the fused per-branch norms + SGD pass (k_group_sumsq<SGD>), the
    # same launch the step runs (inside the graph), timed with HIP events on its stream
    if a.profile:
        if rank == 0:
            print(json.dumps({"profile_run": True, "ms_per_step": round(ms, 3), "steps": a.steps, "n_gpus": world,
                              "value": round(world * B * V * a.steps / elapsed, 2), "unit": "view-images/s"}),
                  flush=True)
        if dist_on:
            dist.destroy_process_group()
        return
    kern_avg_s = time_group_sumsq(step, 10)
    # the step's own launches: the view-batched trunk (vtrunk.py), all V views per launch
    # (C2: 2 x ResNet-18, C4: 4 x ResNet-18, C5: 12 x ResNet-50); the fp32 line's one view
    conv = time_trunk_convs(B, dev, a.dtype, G=V, arch=WL["trunk"])
    mmtm_bytes, mmtm_s = time_mmtm_reduce(dev)
    if rank == 0:
        views = V
        total_imgs = world * B * views * a.steps
        bytes_alg = 12 * step.flat.total  # read param + grad, write param (fp32)
        achieved = bytes_alg / kern_avg_s / 1e9
        traffic = conv_traffic = mmtm_traffic = None
        if os.path.exists(a.mmtm_traffic_file):
            with open(a.mmtm_traffic_file) as f:
                mmtm_traffic = json.load(f).get("hbm_bytes_per_launch")
        if os.path.exists(a.conv_traffic_file):
            with open(a.conv_traffic_file) as f:
                conv_traffic = json.load(f).get("hbm_bytes_per_launch")
        if os.path.exists(a.traffic_file):
            with open(a.traffic_file) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        line = {
            "metric": "multi-view images/sec + step ms, ModelNet40 2-view MVCNN+MMTM @1/2/4/8 GPU",
            "value": round(total_imgs / elapsed, 2),
            "unit": "view-images/s",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": a.dtype,
            "data": f"synthetic N(0,1) [B,{V},3,224,224] + uniform labels, resident in HBM; random-init weights",
            "config": {"workload": WL["desc"] + ", guided gating (training_guided.gin eps 0.01, window 5, unlocked;"
                                   " decided on bf16-trunk gradients: d_BDR within ~6.5e-3 of eps may decide"
                                   " unlike fp32, INTEGRATION.md section 3)",
                       "params": step.flat.total,
                       "global_batch": B * world, "per_gpu_batch": B, "image": a.size,
                       "parallelism": f"dp{world}", "samples_per_s": round(world * B * a.steps / elapsed, 2),
                       "hipgraph": bool(step.graphs), "device_gate": bool(step.device_gate),
                       "curation_steps_timed": curation_steps, "final_loss": round(loss, 4),
                       "dp": dp_info(step, dist_on)},
            "roofline": conv_roofline(conv, conv_traffic if a.dtype == "bf16" and a.workload == "C2" else None,
                                      a.dtype, a.workload),
            "roofline_hbm": {"kernel": "k_group_sumsq<SGD> (fused per-branch norms + SGD, gm_group_sumsq)",
                             "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                             # the PMC traffic file is measured on C2's parameter set
                             "traffic": traffic if a.workload == "C2" else None,
                             "alg_bytes_per_launch": bytes_alg,
                             "avg_launch_us": round(kern_avg_s * 1e6, 2)},
            "roofline_mmtm": {"kernel": "k_colreduce_nhwc (MMTM squeeze: GAP of both views, site s2, "
                                        "north-star batch 256, gm_mmtm_spatial_reduce; launches rotate over 4 "
                                        "distinct pairs = 411 MB > 256 MiB Infinity Cache)",
                              "bound": "hbm", "batch": 256,
                              "achieved": round(mmtm_bytes / mmtm_s / 1e9, 1), "peak": HBM_PEAK_GBS,
                              "unit": "GB/s", "frac": round(mmtm_bytes / mmtm_s / 1e9 / HBM_PEAK_GBS, 4),
                              "traffic": mmtm_traffic, "alg_bytes_per_launch": mmtm_bytes,
                              "avg_launch_us": round(mmtm_s * 1e6, 2)},
        }
        if not a.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(a.cpu_seconds, a.size)
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
