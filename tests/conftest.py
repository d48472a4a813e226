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


# fp32 parity mode: keep MIOpen off its Winograd / FFT convolution algorithms,
# whose fp32 error is 3-8x that of the direct/implicit-GEMM ones (measured on the
# m224b2 gradient norms vs a float64 oracle: rms 1.0e-3 -> 3.0e-4).  Must be set
# before the first convolution of the process.
os.environ.setdefault("MIOPEN_DEBUG_CONV_WINOGRAD", "0")
os.environ.setdefault("MIOPEN_DEBUG_CONV_FFT", "0")
