"""ctypes binding of the test-only kernel library tests/native/libgm_testkit.so (built beside the
product library by greedy_multimodal_learning_amd/build.py; never loaded by the product path)."""
import ctypes
import os

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "libgm_testkit.so")
_lib = None


def load():
    global _lib
    if _lib is None:
        import torch  # noqa: F401  (share PyTorch's HIP runtime)
        _lib = ctypes.CDLL(LIB)
        _lib.gmt_hold_cus.restype = ctypes.c_int
        _lib.gmt_hold_cus.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_void_p]
    return _lib


def hold_cus(blocks, threads, lds_bytes, usec, stream):
    """Launch `blocks` CU-holding workgroups on `stream` (a torch.cuda.Stream's cuda_stream)."""
    rc = load().gmt_hold_cus(int(blocks), int(threads), int(lds_bytes), int(usec), stream)
    if rc != 0:
        raise RuntimeError(f"gmt_hold_cus failed ({rc})")
