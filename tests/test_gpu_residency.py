"""Co-residency of the launches whose workgroups wait on each other (single-launch
BatchNorm, split-K turnstile) beside a kernel that holds CUs and never yields - what the
RCCL all-reduce kernels do while they overlap backward under data parallelism.

The library's residency plan (gm_set_residency) reserves the held CUs: with ONE trunk
stream and the BatchNorm concurrency at 1 (the tightest plan), a layer-4 BatchNorm in one
launch and a layer-4 split-K convolution run while 64 CUs are held by a 160 KiB-LDS
spinning kernel on another stream; they must finish before that kernel ends (they ran
beside it, not behind it), raise no device fault and give bit-identical outputs."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu

HOLD_CUS, HOLD_US = 64, 300_000


@pytest.fixture
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd import streams
    old = L.get_residency()
    L.set_residency(streams=1, sharers=1, reserved_cus=HOLD_CUS)
    L.check(L.load().gm_bn_set_concurrency(1), "gm_bn_set_concurrency")
    yield L
    L.set_residency(*old)
    L.check(L.load().gm_bn_set_concurrency(streams._bn_concurrency[0]), "gm_bn_set_concurrency")


def test_spin_launches_beside_a_cu_holding_kernel(lib):
    from greedy_multimodal_learning_amd import bn, conv
    L = lib
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(7)
    CL = torch.channels_last
    N, C, H = 64, 512, 7  # layer 4 at the benchmark batch
    x = torch.randn(N, C, H, H, device=dev, generator=g).bfloat16().contiguous(memory_format=CL)
    w = (0.02 * torch.randn(C, C, 3, 3, device=dev, generator=g)).bfloat16().contiguous(memory_format=CL)
    gamma = torch.ones(C, device=dev)
    beta = torch.zeros(C, device=dev)
    d = L.ConvDesc(N, H, H, C, C, 3, 3, 1, 1)
    assert L.load().gm_conv2d_splitk_ws_bytes(ctypes.byref(d), 0) > 0, "layer 4 must run split-K here"

    def work():
        y, _, _ = bn.bn_fwd_train(x, gamma, beta, None, None, None, 0.1, 1e-5, True, None)
        return y, conv.conv_fwd(y, w, 1, 1)

    ref = work()
    torch.cuda.synchronize()
    assert L.device_faults(clear=True) == 0
    hold = torch.cuda.Stream(device=dev)
    e0 = torch.cuda.Event(enable_timing=True)
    e_hold = torch.cuda.Event(enable_timing=True)
    e_work = torch.cuda.Event(enable_timing=True)
    e0.record()
    hold.wait_stream(torch.cuda.current_stream())
    import testkit
    testkit.hold_cus(HOLD_CUS, 256, 160 * 1024, HOLD_US, hold.cuda_stream)
    e_hold.record(hold)
    torch.cuda._sleep(2_000_000)  # let the holding workgroups land first
    out = work()
    e_work.record()
    torch.cuda.synchronize()
    t_work, t_hold = e0.elapsed_time(e_work), e0.elapsed_time(e_hold)
    print(f"work done at {t_work:.2f} ms, CU-holding kernel done at {t_hold:.2f} ms")
    assert L.device_faults(clear=True) == 0
    assert t_work < t_hold, "the spin launches waited for the CU-holding kernel"
    for a, b in zip(out, ref):
        assert torch.equal(a, b)
