"""Input pipeline host logic against the reference's own batches
(tests/golden/golden_dataset.npz, made by running the reference's get_mvdcndata,
src/dataset.py:15-128): split, sampler order, view selection, labels and the flip
decisions, with the normalisation done by the numpy oracle (oracle/views_ref.py) in
place of the device launch.  Bit-exact.  CPU only."""
import tempfile

import numpy as np
import pytest
import torch

import spec
from helpers import run_loaders, write_dataset_from_fixture
from oracle import views_ref


def test_views_oracle_matches_reference_batches(golden, monkeypatch):
    from greedy_multimodal_learning_amd import dataset as D
    fix = golden["dataset"]

    def oracle_launch(self, views_u8, flips):
        return torch.from_numpy(views_ref.normalize_views(views_u8.numpy(), None if flips is None else flips.numpy()))
    monkeypatch.setattr(D.ViewNormalize, "launch", oracle_launch)
    monkeypatch.setattr(D.ViewNormalize, "device", property(lambda self: torch.device("cpu")))
    with tempfile.TemporaryDirectory() as root:
        write_dataset_from_fixture(fix, root)
        n = 0
        for ci, case in enumerate(spec.DATASET["cases"]):
            for ep, name, idx, y, x, nb in run_loaders(D, root, case, spec.DATASET["views"]):
                k = f"c{ci}/e{ep}/{name}"
                np.testing.assert_array_equal(idx, fix[k + "/idx"], err_msg=k)
                np.testing.assert_array_equal(y, fix[k + "/y"], err_msg=k)
                np.testing.assert_array_equal(nb, fix[k + "/nb"], err_msg=k)
                if len(idx):
                    assert x.shape == fix[k + "/x"].shape, k
                    assert np.array_equal(x.view(np.uint32), fix[k + "/x"].view(np.uint32)), k  # bit-exact
                n += len(idx)
        assert n > 0


def test_split_indices_reference_rule():
    from greedy_multimodal_learning_amd.dataset import split_indices
    import random
    tr, va = split_indices(10, 0.2, 10)
    ind = list(range(10))
    random.Random(10).shuffle(ind)
    assert va == ind[:2] and tr == ind[2:]
    assert split_indices(7, 0.0, 10)[1] == []
    with pytest.raises(AssertionError):
        split_indices(5, 1.5, 10)


def test_view_stack_loader_formats(tmp_path):
    from greedy_multimodal_learning_amd.dataset import load_view_stack
    a = np.random.default_rng(0).integers(0, 256, (3, 4, 8, 3), dtype=np.uint8)
    np.save(tmp_path / "a.npy", a)
    torch.save(a, tmp_path / "b.npy")          # the reference's own format (torch.load of a numpy array)
    torch.save(torch.from_numpy(a), tmp_path / "c.npy")
    for f in ("a.npy", "b.npy", "c.npy"):
        assert np.array_equal(load_view_stack(tmp_path / f), a)
    np.save(tmp_path / "bad.npy", a.astype(np.float32))
    with pytest.raises(ValueError):
        load_view_stack(tmp_path / "bad.npy")
