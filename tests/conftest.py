import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    d = os.path.join(ROOT, "tests", "golden")
    return {k: np.load(os.path.join(d, f"golden_{k}.npz")) for k in
            ("mmtm", "model", "trace", "ddp", "cur", "dataset")}



@pytest.fixture(autouse=True)
def _default_cuda_generator_usable(request):
    """After every GPU test: the default CUDA generator still works outside a capture.

    A capture that fails after torch put the generator into its capture state (capture_begin
    refused, or a body that invalidated the stream capture) leaves it there, and the next eager
    random op of the process raises "Offset increment outside graph capture ..." - in whatever
    test happens to run next (round 5: test_xent_bad_label_is_nan).  Checked here, the error
    names the test that left it.  The generator's state is restored, so no test's random
    numbers change."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import torch
    if not torch.cuda.is_available() or not torch.cuda.is_initialized():
        return
    state = torch.cuda.get_rng_state()
    try:
        torch.empty(1, device="cuda").uniform_()
    finally:
        torch.cuda.set_rng_state(state)
