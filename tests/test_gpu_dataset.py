"""gm_views_normalize (csrc/views.hip) - the input pipeline's device launch (SURVEY §8
f2) - against the reference's own batches (golden_dataset.npz, made by running the
reference's get_mvdcndata) through the full loader, bit-exact, and against the numpy
oracle (oracle/views_ref.py) at the C2 batch shape in every output layout/dtype."""
import tempfile

import numpy as np
import pytest
import torch

import spec
from helpers import run_loaders, write_dataset_from_fixture
from oracle import views_ref

pytestmark = pytest.mark.gpu


def test_loader_matches_reference_batches_bitexact(golden):
    from greedy_multimodal_learning_amd import dataset as D
    fix = golden["dataset"]
    with tempfile.TemporaryDirectory() as root:
        write_dataset_from_fixture(fix, root)
        n = 0
        for ci, case in enumerate(spec.DATASET["cases"]):
            for ep, name, idx, y, x, nb in run_loaders(D, root, case, spec.DATASET["views"]):
                k = f"c{ci}/e{ep}/{name}"
                np.testing.assert_array_equal(idx, fix[k + "/idx"], err_msg=k)
                np.testing.assert_array_equal(y, fix[k + "/y"], err_msg=k)
                if len(idx):
                    assert np.array_equal(x.view(np.uint32), fix[k + "/x"].view(np.uint32)), k
                n += len(idx)
        assert n > 0


@pytest.mark.parametrize("layout,dtype", [("nchw", torch.float32), ("nchw", torch.bfloat16),
                                          ("views_nhwc", torch.float32), ("views_nhwc", torch.bfloat16)])
def test_views_normalize_c2_shape(layout, dtype):
    """B = 64 two-view 224x224 batch (config C2), random flips: bit-exact vs the oracle
    (bf16 = round-to-nearest-even of the oracle's fp32)."""
    from greedy_multimodal_learning_amd.dataset import ViewNormalize
    g = np.random.default_rng(5)
    u8 = g.integers(0, 256, (64, 2, 224, 224, 3), dtype=np.uint8)
    flips = torch.from_numpy(g.integers(0, 2, 128).astype(np.uint8))
    tf = ViewNormalize(True, out_layout=layout, dtype=dtype, device="cuda:0")
    out = tf(torch.from_numpy(u8), flips)
    assert out.shape == (64, 2, 3, 224, 224)
    if layout == "views_nhwc":  # view-major channels_last storage
        assert out.permute(1, 0, 3, 4, 2).is_contiguous()
    ref = torch.from_numpy(views_ref.normalize_views(u8, flips.numpy())).to(dtype)
    got = out.cpu()
    assert torch.equal(got.view(torch.int16) if dtype == torch.bfloat16 else got.view(torch.int32),
                       ref.view(torch.int16) if dtype == torch.bfloat16 else ref.view(torch.int32))


def test_views_normalize_rejects_bad_shapes():
    from greedy_multimodal_learning_amd import _lib as L
    from greedy_multimodal_learning_amd.dataset import ViewNormalize
    tf = ViewNormalize(False, device="cuda:0")
    with pytest.raises(L.GreedyMMLError):
        tf(torch.zeros(2, 2, 8, 10, 3, dtype=torch.uint8))  # W % 4 != 0
    with pytest.raises(ValueError):
        tf(torch.zeros(2, 2, 8, 8, 4, dtype=torch.uint8))
