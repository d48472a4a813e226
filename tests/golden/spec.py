"""Fixture specification shared by make_golden.py and the tests.

Every input is regenerated from a seed here (numpy PCG64), so the committed
.npz files only need the reference's OUTPUTS.  No reference code lives here.
"""
import zlib

import numpy as np

SEED_MMTM = 11
SEED_MODEL = 0

# F1 - MMTM_mitigate unit cases (C/HW mirror the real sites s2/s3/s4 at small and real spatial size)
MMTM_CASES = [
    dict(id="n128", B=3, C=128, H=8, W=8, mode="normal"),
    dict(id="n256", B=2, C=256, H=4, W=4, mode="normal", warm=2),
    dict(id="n512", B=4, C=512, H=2, W=2, mode="normal"),
    dict(id="n512r", B=2, C=512, H=7, W=7, mode="normal"),
    dict(id="n128r", B=1, C=128, H=28, W=28, mode="normal"),
    dict(id="c0", B=3, C=128, H=5, W=5, mode="cur0", warm=3),
    dict(id="c1", B=3, C=128, H=5, W=5, mode="cur1", warm=3),
    dict(id="c1b", B=2, C=256, H=3, W=3, mode="cur1", warm=1),
    dict(id="off", B=3, C=128, H=4, W=4, mode="turnoff"),
    dict(id="off512", B=2, C=512, H=2, W=2, mode="turnoff", warm=1),
    dict(id="se", B=2, C=128, H=4, W=4, mode="normal_se", SEonly=True),
    dict(id="sw", B=2, C=128, H=4, W=4, mode="normal", shareweight=True),
    dict(id="b1", B=1, C=256, H=1, W=1, mode="normal"),
]

# F2 - whole model, forward + backward
# `gpu_tol`: cases whose train-mode BatchNorm normalises over <= 49 values per
# channel (32x32 input -> 1x1 layer4 maps; B=1) amplify fp32 rounding differences
# of ANY implementation (one ReLU mask flip spreads over a whole channel; measured
# on the HIP fp32 path: tools/f32_precision_probe.py).  They pin the CPU oracle
# at 1e-4 and the GPU at the relaxed tolerance; the well-conditioned cases pin
# the GPU at 1e-4.
MODEL_CASES = [
    dict(id="m64", B=2, H=64, W=64, seed=1),
    dict(id="m64c0", B=3, H=64, W=64, seed=9, cur=True, caring=0),
    dict(id="m64c1", B=3, H=64, W=64, seed=10, cur=True, caring=1),
    dict(id="m224b2", B=2, H=224, W=224, seed=11),
    dict(id="m32c0", B=3, H=32, W=32, seed=2, cur=True, caring=0, gpu_tol=5e-3),
    dict(id="m32c1", B=3, H=32, W=32, seed=3, cur=True, caring=1, gpu_tol=5e-3),
    dict(id="m224", B=1, H=224, W=224, seed=4, gpu_tol=1e-3),  # measured 5.6e-7 (r04)
]

# F3 - gating trace through the reference's own Model_.train_loop
TRACE = dict(B=4, H=32, W=32, steps=4, nval=1, ntest=1, epochs=3, lr=0.1,
             epsilon=0.01, window=2, starting_epoch=2, seed=5)
TRACE_EVAL = dict(B=2, H=32, W=32, seed=6)
# the same guided run, well conditioned for cross-device comparison (64x64 maps,
# lr 1e-3, B 8): the lr-0.1 / 32x32 run above diverges (loss 7 -> 11) and
# amplifies 1e-6 differences to 1e-2 within two steps on any device.  epsilon
# 0.008 keeps every |d_BDR| >= 1.6e-3 away from the threshold (4 curation steps).
TRACE_GPU = dict(B=8, H=64, W=64, steps=4, nval=1, ntest=1, epochs=3, lr=0.001,
                 epsilon=0.008, window=2, starting_epoch=2, seed=12)
TRACE_GPU_EVAL = dict(B=2, H=64, W=64, seed=13)
TRACE_PARAMS = ["mmtm3.fc_visual.bias", "mmtm2.fc_squeeze.bias", "net_view_0.fc.bias",
                "net_view_1.layer1.0.bn1.weight"]

# F4 - data-parallel oracle: mean of per-shard gradients
DDP = dict(B=4, H=32, W=32, world=2, seed=7)

# F5 - conditional utilisation rate: mmtm_off forward from recorded squeezes
CUR = dict(B=2, H=32, W=32, seed=8)
CUR_NTRAIN = 10


def _rng(*key):
    return np.random.Generator(np.random.PCG64(list(key)))


def mmtm_inputs(c):
    r = _rng(SEED_MMTM, zlib.crc32(c["id"].encode()))
    shp = (c["B"], c["C"], c["H"], c["W"])
    xv = r.standard_normal(shp).astype(np.float32)
    xs = (0.5 + r.standard_normal(shp)).astype(np.float32)
    dyv = r.standard_normal(shp).astype(np.float32)
    dys = r.standard_normal(shp).astype(np.float32)
    return xv, xs, dyv, dys


def mmtm_warm_inputs(c, k):
    r = _rng(SEED_MMTM, zlib.crc32(c["id"].encode()), 100 + k)
    shp = (c["B"], c["C"], c["H"], c["W"])
    return r.standard_normal(shp).astype(np.float32), r.standard_normal(shp).astype(np.float32)


def mmtm_avg(c):
    r = _rng(SEED_MMTM, zlib.crc32(c["id"].encode()), 7)
    return (r.standard_normal(c["C"]).astype(np.float32),
            r.standard_normal(c["C"]).astype(np.float32))


def model_inputs(c):
    r = _rng(SEED_MODEL, c["seed"])
    x = r.standard_normal((c["B"], 2, 3, c["H"], c["W"])).astype(np.float32)
    y = r.integers(0, 40, c["B"]).astype(np.int64)
    return x, y


def trace_loaders(t=None):
    t = TRACE if t is None else t
    r = _rng(SEED_MODEL, t["seed"])
    def batches(n, base):
        out = []
        for i in range(n):
            x = r.standard_normal((t["B"], 2, 3, t["H"], t["W"])).astype(np.float32)
            y = r.integers(0, 40, t["B"]).astype(np.int64)
            out.append((np.arange(base + i * t["B"], base + (i + 1) * t["B"]), x, y))
        return out
    return batches(t["steps"], 0), batches(t["nval"], 1000), batches(t["ntest"], 2000)


def sample_idx(name, n, k=16):
    r = _rng(SEED_MODEL, zlib.crc32(name.encode()))
    return r.integers(0, n, min(k, n))


def cur_histories():
    """Synthetic recording history (eval.py + recording.gin format) and training history."""
    r = _rng(SEED_MODEL, 99)
    n = CUR_NTRAIN
    order = r.permutation(n)
    batches = []
    for b0 in range(0, n, 4):
        b = order[b0:b0 + 4]
        batches.append([[r.standard_normal((len(b), C)).astype(np.float32) for _ in range(2)]
                        for C in (128, 256, 512)])
    ev = {"test_squeezedmaps_array_list": [batches], "test_indices": [order]}
    tr = {"train_indices": [np.sort(r.permutation(n)[:7])], "val_indices": [np.arange(3)]}
    return ev, tr


FULL_LIMIT = 16384


def signature(key, arr):
    """Compact fixture form of a large array: axis sums + seeded samples.

    Returns {suffix: array}; small arrays are kept whole under suffix ''.
    """
    a = np.asarray(arr)
    if a.size <= FULL_LIMIT:
        return {"": a}
    flat = a.reshape(-1)
    out = {".samples": flat[sample_idx(key, flat.size, 256)]}
    if a.ndim == 2:
        out[".sum_rows"] = a.astype(np.float64).sum(1)
        out[".sum_cols"] = a.astype(np.float64).sum(0)
    elif a.ndim > 2:
        m = a.reshape(a.shape[0], a.shape[1], -1).astype(np.float64)
        out[".sum_last"] = m.sum(-1)
        out[".sum_first"] = m.sum(0).sum(-1)
    out[".abs_total"] = np.array(np.abs(a.astype(np.float64)).sum())
    return out

# F6 - input pipeline (src/dataset.py): a synthetic ModelNet40-shaped dataset of uint8
# 12-view stacks (H, W small; W % 4 == 0 as gm_views_normalize needs), two loader cases
DATASET = dict(seed=2024, views=12, H=8, W=12, n_train=11, n_test=5,
               classnames=["airplane", "bathtub", "bed", "chair"],
               cases=[dict(batch_size=3, valid_size=0.2, specific_views=[0, 6], epochs=2),
                      dict(batch_size=4, valid_size=0.0, specific_views=[1, 2, 5], epochs=1)])
