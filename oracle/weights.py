"""Seeded, framework-independent parameter generator (numpy PCG64).

Fixtures and tests must agree on model weights without committing a 95 MB
state dict.  `generate(named_shapes, seed)` walks the parameters in the given
(sorted-by-name) order and draws each from a distribution that mimics the
reference's init (conv: kaiming-normal fan_out; BN: around 1 / 0 with a small
perturbation so BN gradients are exercised; Linear: U(-1/sqrt(fan_in), ..)).
Only the *names* and *shapes* determine the values, so the reference model
(imported with shims), the oracle and the HIP product get identical tensors.
"""
import numpy as np


def _draw(rng, name, shape):
    n = int(np.prod(shape)) if len(shape) else 1
    leaf = name.rsplit(".", 1)[-1]
    if len(shape) == 4:  # conv weight [Cout, Cin, kh, kw]
        fan_out = shape[0] * shape[2] * shape[3]
        return rng.standard_normal(n).astype(np.float32) * np.float32(np.sqrt(2.0 / fan_out))
    if len(shape) == 2:  # linear weight [out, in]
        b = 1.0 / np.sqrt(shape[1])
        return rng.uniform(-b, b, n).astype(np.float32)
    if len(shape) == 1:
        if leaf == "weight":  # BN gamma
            return (1.0 + 0.1 * rng.standard_normal(n)).astype(np.float32)
        if leaf == "bias":
            return (0.05 * rng.standard_normal(n)).astype(np.float32)
        if leaf == "running_mean":
            return np.zeros(n, np.float32)
        if leaf == "running_var":
            return np.ones(n, np.float32)
    return (0.05 * rng.standard_normal(n)).astype(np.float32)


def generate(named_shapes, seed=0):
    """named_shapes: iterable of (name, shape). Returns {name: np.ndarray}."""
    out = {}
    for name, shape in sorted(named_shapes, key=lambda t: t[0]):
        # one independent stream per tensor: stable under adding/removing tensors
        h = np.frombuffer(name.encode(), dtype=np.uint8).astype(np.uint64)
        key = int((h * np.arange(1, len(h) + 1, dtype=np.uint64)).sum() % (2**32))
        rng = np.random.Generator(np.random.PCG64([seed, key, len(name)]))
        out[name] = _draw(rng, name, tuple(shape)).reshape(shape)
    return out


def apply_to_module(module, seed=0):
    """Overwrite every float parameter (and BN running stats) of a torch module."""
    import torch
    sd = module.state_dict()
    shapes = [(k, tuple(v.shape)) for k, v in sd.items() if v.dtype.is_floating_point]
    vals = generate(shapes, seed)
    with torch.no_grad():
        for k, v in vals.items():
            sd[k].copy_(torch.from_numpy(v))
    return module
