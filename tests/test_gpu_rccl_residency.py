"""Pre-C3 robustness: the launches whose workgroups wait on each other
(single-launch BatchNorm, split-K turnstile) inside the data-parallel step graph, beside a
resident CU-holding kernel, under the residency plan the ENGINE sets for RCCL.

One process, a one-rank RCCL ("nccl") process group with NCCL_MAX_NCHANNELS = 64 (the bound
engine.bound_rccl_channels() sets before any communicator exists): BalancedStep(dp_buckets=True,
graphs=True) must plan 64 reserved CUs (engine.rccl_reserved_cus), capture the bucketed
all-reduces inside the step graph, and then replay steps while a kernel holds 64 CUs (one
160 KiB-LDS workgroup per CU, never yielding - the footprint of RCCL's one workgroup per channel
on a multi-rank node, which a one-rank all-reduce does not launch) on another stream.  The
replays must finish before the holder does (they ran beside it, not behind it), raise no device
fault, and equal the same steps run without the holder bit for bit.

CU budget per rank on an 8-GPU node (one process per GPU): 256 CUs - 64
reserved for RCCL = 192 CUs for the co-residency plan of the spin hand-off launches."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HOLD_CUS, HOLD_US = 64, 400_000


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, port, out_dir):
    import ctypes
    import torch.distributed as dist
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Strong
    from greedy_multimodal_learning_amd.engine import BalancedStep, bound_rccl_channels
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN
    os.environ.pop("NCCL_MAX_NCHANNELS", None)
    assert bound_rccl_channels() == 64
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=1)
    dev = torch.device("cuda:0")
    lib = L.load()
    B = 16
    d = L.ConvDesc(B, 7, 7, 512, 512, 3, 3, 1, 1)  # layer 4, both views in one grouped launch
    split_k = lib.gm_conv2d_splitk_ws_bytes_grouped(ctypes.byref(d), 2, 0) > 0
    g = torch.Generator(device=dev).manual_seed(3)
    xs = [torch.randn(B, 2, 3, 224, 224, device=dev, generator=g) for _ in range(2)]
    ys = [torch.randint(0, 40, (B,), device=dev, generator=g) for _ in range(2)]

    def engine():
        torch.manual_seed(0)
        m = MMTM_MVCNN().to(dev)
        gate = Bias_Mitigation_Strong(epsilon=2e-3, curation_windowsize=2,
                                      branchnames=["net_view_0", "net_view_1"], starting_epoch=1)
        st = BalancedStep(m, lr=0.05, gate=gate, process_group=dist.group.WORLD, bucket_mb=8.0,
                          graphs=os.environ.get("GM_TEST_GRAPHS", "1") != "0", dp_buckets=True)
        st.on_epoch_begin(1)
        return m, st

    res = {}
    for hold in (False, True):
        m, st = engine()
        losses = [float(st(xs[i % 2], ys[i % 2])) for i in range(3)]  # eager, then the captured graph
        plan = L.get_residency()
        torch.cuda.synchronize()
        assert L.device_faults(clear=True) == 0
        t_work = t_hold = None
        if hold:
            hs = torch.cuda.Stream(device=dev)
            e0, e_hold, e_work = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record()
            hs.wait_stream(torch.cuda.current_stream())
            import testkit
            testkit.hold_cus(HOLD_CUS, 256, 160 * 1024, HOLD_US, hs.cuda_stream)
            e_hold.record(hs)
            torch.cuda._sleep(2_000_000)  # the holding workgroups land first
        out = [st(xs[i % 2], ys[i % 2]) for i in range(3, 7)]
        if hold:
            e_work.record()
        torch.cuda.synchronize()
        if hold:
            t_work, t_hold = e0.elapsed_time(e_work), e0.elapsed_time(e_hold)
        losses += [float(v) for v in out]
        res[hold] = dict(losses=losses, sd={k: v.detach().cpu() for k, v in m.state_dict().items()},
                         plan=tuple(plan), graphs=bool(st.graphs), inline=bool(st.graph_collectives),
                         faults=int(L.device_faults(clear=True)), t_work=t_work, t_hold=t_hold, split_k=split_k)
    torch.save(res, os.path.join(out_dir, "rccl_residency.pt"))
    dist.destroy_process_group()


def test_spin_launches_in_the_rccl_step_graph_beside_held_cus(tmp_path, monkeypatch):
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    # as bench.py does for data-parallel ranks: more hardware queues than streams, so the holding
    # kernel's stream does not share a queue with the step's (HIP's default of 4 queues put it
    # behind the holder on one: a 393 ms stall that is queue sharing, not residency)
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "8")
    mp.start_processes(_worker, args=(_free_port(), str(tmp_path)), nprocs=1, join=True, start_method="spawn")
    res = torch.load(tmp_path / "rccl_residency.pt", weights_only=True)
    a, b = res[False], res[True]
    print(f"residency plan (streams, sharers, reserved CUs) = {b['plan']}; replays done at {b['t_work']:.2f} ms, "
          f"CU-holding kernel done at {b['t_hold']:.2f} ms; split-K at layer 4: {b['split_k']}")
    assert b["split_k"], "layer 4 should run split-K at this batch"
    assert b["plan"][2] == 64, "the engine must reserve RCCL's 64 channel CUs"
    assert a["graphs"] and b["graphs"] and a["inline"] and b["inline"], "collectives not captured in the graph"
    assert a["faults"] == 0 and b["faults"] == 0
    assert b["t_work"] < b["t_hold"], "the spin launches waited for the CU-holding kernel"
    assert a["losses"] == b["losses"]
    for k in a["sd"]:
        assert torch.equal(a["sd"][k], b["sd"][k]), k
