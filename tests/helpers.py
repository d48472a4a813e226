"""Shared test helpers: fixture comparison (full arrays or signatures)."""
import numpy as np

import spec


def close(fix, key, arr, rtol=1e-4, atol=1e-5):
    """Compare `arr` with fixture entry `key` (full array or spec.signature form)."""
    arr = np.asarray(arr)
    if key in fix.files:
        ref = fix[key]
        assert ref.shape == arr.shape, (key, ref.shape, arr.shape)
        np.testing.assert_allclose(arr, ref, rtol=rtol, atol=atol, err_msg=key)
        return
    sig = spec.signature(key, arr)
    assert len(sig) > 1, f"fixture {key} missing"
    for suf, v in sig.items():
        ref = fix[key + suf]
        scale = max(1.0, float(np.abs(ref).max())) if suf != ".samples" else 1.0
        np.testing.assert_allclose(v, ref, rtol=rtol, atol=atol * scale * (arr.size ** 0.5 if suf != ".samples" else 1),
                                   err_msg=key + suf)
