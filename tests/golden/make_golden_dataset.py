#!/usr/bin/env python3
"""Generate tests/golden/golden_dataset.npz by running the REFERENCE input pipeline
(src/dataset.py: get_mvdcndata / MultiviewModelDataset) on a small synthetic
ModelNet40-shaped dataset written here.

Runs only in the build container (needs /root/reference, read-only).  Shims, none
carrying reference code: those of make_golden.py (gin, argh, CUDA redirect ...), and
`torchvision.transforms` restated from torchvision's published algorithm (torchvision
is not installed here and is unpinned upstream, README.md:8):
  ToPILImage(ndarray HWC uint8)  -> PIL.Image.fromarray
  RandomHorizontalFlip(p)        -> `if torch.rand(1) < p: img.transpose(FLIP_LEFT_RIGHT)`
  ToTensor(PIL / ndarray HWC)    -> from_numpy(HWC).permute(2, 0, 1).float().div(255)
  Normalize(mean, std)           -> tensor.sub_(mean[:, None, None]).div_(std[:, None, None])
The data files are torch.save'd numpy arrays (the reference reads `{model}.npy` with
torch.load, src/dataset.py:121); the generator reads its OWN files with
weights_only=False.  The fixture stores the dataset (uint8) and, per loader and epoch,
the batches' indices, labels and fp32 data as the reference produced them.

Usage:  python tests/golden/make_golden_dataset.py [--ref /root/reference]
"""
import argparse
import json
import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden  # noqa: E402
import spec  # noqa: E402


def restated_transforms():
    from PIL import Image
    tvt = types.ModuleType("torchvision.transforms")

    class Compose:
        def __init__(self, ts):
            self.ts = ts

        def __call__(self, x):
            for t in self.ts:
                x = t(x)
            return x

    class ToPILImage:
        def __call__(self, a):
            return Image.fromarray(np.asarray(a), mode="RGB")

    class RandomHorizontalFlip:
        def __init__(self, p=0.5):
            self.p = p

        def __call__(self, img):
            if torch.rand(1) < self.p:
                return img.transpose(Image.FLIP_LEFT_RIGHT)
            return img

    class ToTensor:
        def __call__(self, pic):
            a = np.array(pic, dtype=np.uint8, copy=True)
            return torch.from_numpy(a).permute(2, 0, 1).contiguous().to(torch.float32).div(255)

    class Normalize:
        def __init__(self, mean, std):
            self.mean, self.std = mean, std

        def __call__(self, t):
            m = torch.as_tensor(self.mean, dtype=t.dtype)
            s = torch.as_tensor(self.std, dtype=t.dtype)
            return t.sub(m[:, None, None]).div(s[:, None, None])

    for c in (Compose, ToPILImage, RandomHorizontalFlip, ToTensor, Normalize):
        setattr(tvt, c.__name__, c)
    return tvt


def write_dataset(root, R):
    """metadata.json + {split}/{model}.npy, uint8 [12, H, W, 3] per model."""
    d = spec.DATASET
    meta = {"classnames": list(d["classnames"]), "train": [], "test": []}
    arrays = {}
    for split, n in (("train", d["n_train"]), ("test", d["n_test"])):
        os.makedirs(os.path.join(root, split), exist_ok=True)
        for i in range(n):
            cname = d["classnames"][int(R.integers(len(d["classnames"])))]
            model = f"{cname}_{split}_{i:04d}"
            meta[split].append({"classname": cname, "model": model})
            a = R.integers(0, 256, size=(d["views"], d["H"], d["W"], 3), dtype=np.uint8)
            torch.save(a, os.path.join(root, split, model + ".npy"))
            arrays[f"{split}/{i}"] = a
    with open(os.path.join(root, "metadata.json"), "w") as f:
        json.dump(meta, f)
    return meta, arrays


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    a = ap.parse_args()
    make_golden.install_shims(a.ref)
    sys.modules["torchvision.transforms"] = restated_transforms()
    sys.modules["torchvision"].transforms = sys.modules["torchvision.transforms"]
    orig_load = torch.load
    torch.load = lambda p, *x, **k: orig_load(p, *x, **{**k, "weights_only": False})  # our own files
    import src.dataset as D
    d = spec.DATASET
    out = {}
    with tempfile.TemporaryDirectory() as root:
        meta, arrays = write_dataset(root, np.random.default_rng(d["seed"]))
        for split in ("train", "test"):
            out[f"data/{split}"] = np.stack([arrays[f"{split}/{i}"] for i in range(len(meta[split]))])
            out[f"data/{split}_class"] = np.array([meta["classnames"].index(s["classname"]) for s in meta[split]])
        for ci, case in enumerate(d["cases"]):
            train, valid, test = D.get_mvdcndata(root_dir=root, batch_size=case["batch_size"],
                                                 valid_size=case["valid_size"], num_views=d["views"],
                                                 specific_views=case["specific_views"], num_workers=0,
                                                 use_cuda=False)
            for ep in range(case["epochs"]):
                for name, loader in (("train", train), ("valid", valid), ("test", test)):
                    idx, ys, xs = [], [], []
                    for i, x, y in loader:
                        idx.append(i.numpy()), ys.append(y.numpy()), xs.append(x.numpy())
                    k = f"c{ci}/e{ep}/{name}"
                    out[k + "/idx"] = np.concatenate(idx) if idx else np.zeros(0, np.int64)
                    out[k + "/y"] = np.concatenate(ys) if ys else np.zeros(0, np.int64)
                    out[k + "/x"] = np.concatenate(xs) if xs else np.zeros((0,), np.float32)
                    out[k + "/nb"] = np.array([len(v) for v in idx])
    path = os.path.join(HERE, "golden_dataset.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(out)} arrays")


if __name__ == "__main__":
    main()
