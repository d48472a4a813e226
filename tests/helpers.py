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


def write_dataset_from_fixture(fix, root):
    """Recreate the synthetic dataset of golden_dataset.npz on disk (metadata.json +
    {split}/{model}.npy as plain .npy files) in the order make_golden_dataset.py wrote it."""
    import json
    import os
    d = spec.DATASET
    meta = {"classnames": list(d["classnames"]), "train": [], "test": []}
    for split in ("train", "test"):
        os.makedirs(os.path.join(root, split), exist_ok=True)
        data, cls = fix[f"data/{split}"], fix[f"data/{split}_class"]
        for i in range(len(data)):
            cname = d["classnames"][int(cls[i])]
            model = f"{cname}_{split}_{i:04d}"
            meta[split].append({"classname": cname, "model": model})
            np.save(os.path.join(root, split, model + ".npy"), data[i])
    with open(os.path.join(root, "metadata.json"), "w") as f:
        json.dump(meta, f)


def run_loaders(D, root, case, views):
    """Every (case, epoch, loader) batch stream of the fixture through `D.get_mvdcndata`;
    yields (key, idx, y, x) with x as a numpy fp32 [n, V, 3, H, W]."""
    train, valid, test = D.get_mvdcndata(root_dir=root, batch_size=case["batch_size"],
                                         valid_size=case["valid_size"], num_views=views,
                                         specific_views=case["specific_views"], num_workers=0,
                                         use_cuda=False)
    for ep in range(case["epochs"]):
        for name, loader in (("train", train), ("valid", valid), ("test", test)):
            idx, ys, xs = [], [], []
            for i, x, y in loader:
                idx.append(i.cpu().numpy()), ys.append(y.cpu().numpy()), xs.append(x.float().cpu().numpy())
            yield (ep, name, np.concatenate(idx) if idx else np.zeros(0, np.int64),
                   np.concatenate(ys) if ys else np.zeros(0, np.int64),
                   np.concatenate(xs) if xs else np.zeros((0,), np.float32), [len(v) for v in idx])
