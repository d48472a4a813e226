"""Co-residency of the launches whose workgroups wait on each other (single-launch
BatchNorm, split-K turnstile) beside a kernel that holds CUs and never yields - what the
RCCL all-reduce kernels do while they overlap backward under data parallelism.

The library's residency plan (gm_set_residency) reserves the held CUs: with ONE trunk
stream and the BatchNorm concurrency at 1 (the tightest plan), a layer-4 BatchNorm in one
launch and a layer-4 split-K convolution run while 64 CUs are held by a 160 KiB-LDS
spinning kernel on another stream; they must finish before that kernel ends (they ran
beside it, not behind it), raise no device fault and give bit-identical outputs.

The body runs in a spawned process with GPU_MAX_HW_QUEUES=8 (as bench.py gives data-parallel
ranks): with HIP's default of 4 hardware queues, the holding kernel's stream can land on the main
stream's queue once enough streams exist in the process (the other GPU tests create several),
and the work then queues BEHIND the holder - a queue-sharing stall, not a residency failure."""
import ctypes
import os

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HOLD_CUS, HOLD_US = 64, 300_000


def _worker(rank, out_dir):
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import bn, conv
    import testkit
    L.set_residency(streams=1, sharers=1, reserved_cus=HOLD_CUS)
    L.check(L.load().gm_bn_set_concurrency(1), "gm_bn_set_concurrency")
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(7)
    CL = torch.channels_last
    N, C, H = 64, 512, 7  # layer 4 at the benchmark batch
    x = torch.randn(N, C, H, H, device=dev, generator=g).bfloat16().contiguous(memory_format=CL)
    w = (0.02 * torch.randn(C, C, 3, 3, device=dev, generator=g)).bfloat16().contiguous(memory_format=CL)
    gamma = torch.ones(C, device=dev)
    beta = torch.zeros(C, device=dev)
    d = L.ConvDesc(N, H, H, C, C, 3, 3, 1, 1)
    split_k = L.load().gm_conv2d_splitk_ws_bytes(ctypes.byref(d), 0) > 0

    def work():
        y, _, _ = bn.bn_fwd_train(x, gamma, beta, None, None, None, 0.1, 1e-5, True, None)
        return y, conv.conv_fwd(y, w, 1, 1)

    ref = work()
    torch.cuda.synchronize()
    f0 = L.device_faults(clear=True)
    hold = torch.cuda.Stream(device=dev)
    e0 = torch.cuda.Event(enable_timing=True)
    e_hold = torch.cuda.Event(enable_timing=True)
    e_work = torch.cuda.Event(enable_timing=True)
    e0.record()
    hold.wait_stream(torch.cuda.current_stream())
    testkit.hold_cus(HOLD_CUS, 256, 160 * 1024, HOLD_US, hold.cuda_stream)
    e_hold.record(hold)
    torch.cuda._sleep(2_000_000)  # let the holding workgroups land first
    out = work()
    e_work.record()
    torch.cuda.synchronize()
    res = dict(split_k=split_k, f0=f0, f1=L.device_faults(clear=True), t_work=e0.elapsed_time(e_work),
               t_hold=e0.elapsed_time(e_hold), equal=all(torch.equal(a, b) for a, b in zip(out, ref)))
    torch.save(res, os.path.join(out_dir, "residency.pt"))


def test_spin_launches_beside_a_cu_holding_kernel(tmp_path, monkeypatch):
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "8")
    mp.start_processes(_worker, args=(str(tmp_path),), nprocs=1, join=True, start_method="spawn")
    r = torch.load(tmp_path / "residency.pt", weights_only=True)
    print(f"work done at {r['t_work']:.2f} ms, CU-holding kernel done at {r['t_hold']:.2f} ms")
    assert r["split_k"], "layer 4 must run split-K here"
    assert r["f0"] == 0 and r["f1"] == 0
    assert r["t_work"] < r["t_hold"], "the spin launches waited for the CU-holding kernel"
    assert r["equal"]
