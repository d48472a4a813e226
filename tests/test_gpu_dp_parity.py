"""Data-parallel parity ON THE HIP PATH (fixture F4).

The reference trains on one device (src/training_loop.py:130-133); its data-parallel
oracle is the mean of per-shard gradients with per-rank BatchNorm statistics
(tests/golden/golden_ddp.npz, made from the reference itself by make_golden.py).  Here
two ranks share cuda:0 over gloo - the same engine code that runs RCCL on a node:
FlatParams + GradBuckets all-reduce from the HIP backward kernels' gradient sink - and
the all-reduced gradients are checked

* fp32 (the reference's arithmetic, every op on libgreedymml_hip.so), F4 shards
  (B = 4 split 2 + 2, 32x32): per-parameter norms of the mean gradient against the
  fixture's `ddp/gn`, eager and hipGraph steps;
* bf16 at the benchmark's per-rank shape (B = 64 per rank, 224x224, hipGraph steps):
  the gate's 8 group sums of the mean gradient against the fp32 oracle's mean of
  per-shard gradients on the same bf16-rounded inputs and weights.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import spec

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gn_of(step, model, world):
    g = (step.flat.grad / world).double()
    out = []
    for n, p in model.named_parameters():
        off, k = step.flat.slices[p]
        out.append(float((g[off:off + k] ** 2).sum()))
    return np.array(out)


def _worker_f32(rank, world, port, out_dir, case=None):
    import torch.distributed as dist
    from greedy_multimodal_learning_amd.engine import BalancedStep
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN
    from oracle import weights
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    m = weights.apply_to_module(MMTM_MVCNN(), seed=spec.SEED_MODEL).to(dev)
    names = [n for n, _ in m.named_parameters()]
    # lr 0: every step sees the fixture's weights; graphs: step 1 eager, 2 captured + replayed, 3 replayed
    st = BalancedStep(m, lr=0.0, gate=None, compute_dtype=torch.float32, process_group=dist.group.WORLD,
                      bucket_mb=2.0, graphs=True, dp_buckets=True)
    case = case or spec.DDP
    x, y = spec.model_inputs(case)
    lo = case["B"] // world
    xs = torch.from_numpy(np.ascontiguousarray(x[rank * lo:(rank + 1) * lo])).to(dev)
    ys = torch.from_numpy(np.ascontiguousarray(y[rank * lo:(rank + 1) * lo])).to(dev)
    gns = []
    for _ in range(3):
        st(xs, ys)
        torch.cuda.synchronize()
        gns.append(_gn_of(st, m, world))
    np.save(os.path.join(out_dir, f"f32_gn_{rank}.npy"), np.stack(gns))
    np.save(os.path.join(out_dir, "names.npy"), np.array(names))
    np.save(os.path.join(out_dir, f"f32_graphs_{rank}.npy"), np.array([st.graphs, len(st._graphs)]))
    dist.barrier()
    dist.destroy_process_group()


def _fp64_mean_of_shards(case=None):
    from oracle import gating_ref, model_ref, weights
    case = case or spec.DDP
    x, y = spec.model_inputs(case)
    lo = case["B"] // case["world"]
    acc = None
    for r in range(case["world"]):
        o = weights.apply_to_module(model_ref.MMTM_MVCNN_Ref(), seed=spec.SEED_MODEL).double()
        o.train(True)
        _, outs, _, _ = o(torch.from_numpy(x[r * lo:(r + 1) * lo]).double())
        gating_ref.blend_loss(outs, torch.from_numpy(y[r * lo:(r + 1) * lo])).backward()
        g = {n: p.grad.clone() for n, p in o.named_parameters()}
        acc = g if acc is None else {n: acc[n] + g[n] for n in acc}
    return {n: v / case["world"] for n, v in acc.items()}


def test_dp_f32_hip_gradients_match_mean_of_shards(golden, tmp_path):
    world = spec.DDP["world"]
    mp.start_processes(_worker_f32, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    fix = golden["ddp"]
    names = list(np.load(tmp_path / "names.npy"))
    assert names == list(fix["ddp/param_names"])
    g0, g1 = np.load(tmp_path / "f32_gn_0.npy"), np.load(tmp_path / "f32_gn_1.npy")
    assert bool(np.load(tmp_path / "f32_graphs_0.npy")[0]), "the graph steps did not run"
    np.testing.assert_array_equal(g0, g1)  # identical all-reduced gradients on both ranks
    np.testing.assert_array_equal(g0[1], g0[2])  # two graph replays of one batch: bit-identical
    g64 = _fp64_mean_of_shards()
    gn64 = np.array([float((g64[n] ** 2).sum()) for n in names])
    ref = fix["ddp/gn"]
    e_ref = np.abs(ref - gn64) / gn64
    for i, label in enumerate(("eager", "graph capture", "graph replay")):
        e_fix = np.abs(g0[i] - ref) / ref
        e_gpu = np.abs(g0[i] - gn64) / gn64
        print(f"F4 fp32 DP ({label}): vs fixture max {e_fix.max():.2e} rms {np.sqrt((e_fix ** 2).mean()):.2e}; "
              f"vs fp64 max {e_gpu.max():.2e} (reference vs fp64 max {e_ref.max():.2e})")
        # F4 is ill-conditioned by construction: B = 2 per shard at 32x32 puts a BatchNorm
        # over 2 values per channel at layer 4 (1x1 maps), whose gradient is mostly rounding
        # - the reference's OWN fp32 run is 9.3e-2 off the fp64 mean of shards (measured).
        # So this fixture pins the plumbing (shards, per-rank statistics, mean) within the
        # envelope of the reference's own error; the well-conditioned case below pins the
        # numbers.  Measured: 1.04e-1 vs fp64 (reference 9.32e-2).
        assert e_gpu.max() <= max(2 * e_ref.max(), 2e-4), (label, e_fix.max(), e_gpu.max())


DDP_WELL = dict(B=8, H=64, W=64, world=2, seed=21)  # 4 per shard, 64x64: layer-4 BN over 16 values


def test_dp_f32_hip_gradients_well_conditioned(tmp_path):
    """The same all-reduced fp32 HIP gradients on a well-conditioned shard size, against
    the oracle's fp64 mean of per-shard gradients (the oracle is pinned to the
    reference's fixtures at 1e-4: test_oracle_golden.py)."""
    c = DDP_WELL
    mp.start_processes(_worker_f32, args=(c["world"], _free_port(), str(tmp_path), c), nprocs=c["world"],
                       join=True, start_method="spawn")
    names = list(np.load(tmp_path / "names.npy"))
    g0, g1 = np.load(tmp_path / "f32_gn_0.npy"), np.load(tmp_path / "f32_gn_1.npy")
    np.testing.assert_array_equal(g0, g1)
    g64 = _fp64_mean_of_shards(c)
    gn64 = np.array([float((g64[n] ** 2).sum()) for n in names])
    e = np.abs(g0 - gn64[None]) / gn64[None]
    worst = names[int(np.argmax(e.max(0)))]
    print(f"DP fp32 2x4 @64x64 vs fp64 mean of shards: max {e.max():.2e} rms {np.sqrt((e ** 2).mean()):.2e} "
          f"(worst {worst})")
    # measured m64 single-device: max 4e-6 vs fp64 (test_gpu_model.py)
    assert e.max() < 1e-4


def _worker_bf16(rank, world, port, out_dir, B, H):
    import torch.distributed as dist
    from greedy_multimodal_learning_amd.engine import BalancedStep
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN
    from oracle import weights
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    m = weights.apply_to_module(MMTM_MVCNN(), seed=5).to(dev)
    st = BalancedStep(m, lr=0.0, gate=None, process_group=dist.group.WORLD, graphs=True, dp_buckets=True)
    g = torch.Generator().manual_seed(4040 + rank)
    buf = torch.randn(2, B, H, H, 3, generator=g).bfloat16()  # view-major channels_last (the bench layout)
    y = torch.randint(0, 40, (B,), generator=g)
    torch.save({"x": buf, "y": y}, os.path.join(out_dir, f"bf16_in_{rank}.pt"))
    x_dev = buf.to(dev).permute(1, 0, 4, 2, 3)
    for _ in range(3):  # eager, capture + replay, replay (lr 0: one state)
        st(x_dev, y.to(dev))
    sums = st.norms.sums(grad_scale=1.0 / world, lr=0.0).cpu().numpy()
    np.save(os.path.join(out_dir, f"bf16_sums_{rank}.npy"), sums)
    np.save(os.path.join(out_dir, f"bf16_res_{rank}.npy"), np.array(st.residency))
    dist.barrier()
    dist.destroy_process_group()


def test_dp_bf16_hip_group_sums_match_oracle_mean_of_shards(tmp_path):
    from oracle import gating_ref, model_ref, weights
    world, B, H = 2, 64, 224
    mp.start_processes(_worker_bf16, args=(world, _free_port(), str(tmp_path), B, H), nprocs=world, join=True,
                       start_method="spawn")
    s0, s1 = np.load(tmp_path / "bf16_sums_0.npy"), np.load(tmp_path / "bf16_sums_1.npy")
    np.testing.assert_array_equal(s0, s1)
    # the engine found both ranks on cuda:0 (gm_set_residency sharers = 2)
    assert int(np.load(tmp_path / "bf16_res_0.npy")[1]) == 2
    torch.set_num_threads(max(1, min(32, torch.get_num_threads())))
    acc = None
    for r in range(world):
        d = torch.load(tmp_path / f"bf16_in_{r}.pt", weights_only=True)
        o = weights.apply_to_module(model_ref.MMTM_MVCNN_Ref(), seed=5)
        _, outs, _, _ = o(d["x"].float().permute(1, 0, 4, 2, 3).contiguous())
        gating_ref.blend_loss(outs, d["y"]).backward()
        g = {n: p.grad.double() for n, p in o.named_parameters()}
        acc = g if acc is None else {n: acc[n] + g[n] for n in acc}
        named_p = {n: p.detach() for n, p in o.named_parameters()}
    os_ = gating_ref.group_sums([(n, named_p[n], acc[n] / world) for n in acc])
    ref = np.array([v for i in range(2) for v in (os_["wn_main"][i], os_["gn_main"][i])] +
                   [v for i in range(2) for v in (os_["wn_bypass"][i], os_["gn_bypass"][i])])
    e_w = np.abs(s0[0::2] - ref[0::2]) / ref[0::2]
    e_g = np.abs(s0[1::2] - ref[1::2]) / ref[1::2]
    print(f"bf16 DP 2x64 vs oracle mean of shards: weight sums rel {e_w.max():.2e}, gradient sums rel {e_g}")
    assert e_w.max() < 1e-6
    # the bf16 floor: PyTorch's own CPU bf16 autocast moves these sums by 4-8e-3 per branch
    # (test_gpu_c2_bf16.py); measured here (r04) 7.1e-3 / 7.5e-5 / 1.4e-3 / 6.5e-4 - which
    # branch lands high follows the weights (test_gpu_view_symmetry.py).  Bound: 2x the worst.
    assert e_g.max() < 1.5e-2
