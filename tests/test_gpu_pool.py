"""Stem max-pool kernels vs PyTorch's max_pool2d (exact: max and gradient routing,
including ties such as the zeros after ReLU)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
CL = torch.channels_last


@pytest.mark.parametrize("shape,k,s,p", [((2, 64, 112, 112), 3, 2, 1), ((3, 8, 9, 7), 3, 2, 1),
                                         ((2, 16, 10, 10), 2, 2, 0), ((1, 32, 13, 13), 3, 1, 1)])
def test_maxpool_matches_torch(shape, k, s, p):
    from greedy_multimodal_learning_amd.pool import GMMaxPool2d
    g = torch.Generator(device="cuda").manual_seed(1)
    x = F.relu(torch.randn(shape, device="cuda", generator=g)).bfloat16()  # many exact ties at 0
    x[0, 0, :3, :3] = float("-inf")
    x = x.contiguous(memory_format=CL)
    m = GMMaxPool2d(k, s, p)
    xa = x.clone().requires_grad_(True)
    y = m(xa)
    dy = torch.randn(y.shape, device="cuda", generator=g).bfloat16().contiguous(memory_format=CL)
    y.backward(dy)
    xr = x.float().contiguous().requires_grad_(True)
    yr = F.max_pool2d(xr, k, s, p)
    yr.backward(dy.float().contiguous())
    assert torch.equal(y.float(), yr)
    # gradient: same routing; sums of <= 4 bf16 values in fp32 then rounded
    torch.testing.assert_close(xa.grad.float(), xr.grad.bfloat16().float(), rtol=1e-2, atol=1e-2)
    assert torch.equal(xa.grad.float() != 0, xr.grad != 0)
