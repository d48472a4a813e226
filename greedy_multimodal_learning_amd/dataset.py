"""Multi-view input pipeline on MI355X: drop-in for the reference's `src.dataset`
(SURVEY §8 f2).

Reference (src/dataset.py:15-128): `get_mvdcndata(...)` builds three DataLoaders
over `MultiviewModelDataset`s whose items are `(idx, data[V,3,H,W] fp32, class_id)`;
each view of `{split}/{model}.npy` (a V x H x W x 3 uint8 stack) goes through
`ToPILImage -> RandomHorizontalFlip -> ToTensor -> Normalize(ImageNet)` (train and
validation) or `ToTensor -> Normalize` (test) ON THE CPU, one image at a time.

Here the host only reads and stacks the raw uint8 views of a batch; the batch goes to
the GPU as bytes (3 B/pixel instead of 12) and ONE HIP launch (`gm_views_normalize`,
csrc/views.hip) applies flip + ToTensor + Normalize to every view, writing either the
reference's `[B, V, 3, H, W]` fp32 tensor or the engine's view-major channels_last
bf16 layout.  Same gin name and parameters as the reference; same seeding, the same
80/20 split (`random.Random(random_seed_for_validation)`, :73-75), the same sampler
order and the same flip decisions: one `torch.rand(1) < 0.5` per view, drawn sample
by sample from torch's global generator exactly as the reference's per-item
transforms draw them (num_workers=0).
"""
import ctypes
import json
import os
import random
from pathlib import Path

import numpy as np
import torch
import torch.utils.data

from . import _lib as L
from .gin_lite import configurable

SEED_FIXED = 100000
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def load_view_stack(path):
    """uint8 [V, H, W, 3] of one model.  The reference reads `{model}.npy` with
    `torch.load` (src/dataset.py:121): a real .npy file is read with numpy (no pickle),
    a torch-serialised tensor or numpy array with `torch.load(weights_only=True)`
    (numpy's array reconstructors allow-listed; nothing else is unpickled)."""
    path = str(path)
    with open(path, "rb") as f:
        magic = f.read(6)
    if magic == b"\x93NUMPY":
        arr = np.load(path, allow_pickle=False)
    else:
        safe = [np.ndarray, np.dtype, type(np.dtype(np.uint8))]
        try:
            from numpy._core.multiarray import _reconstruct
        except ImportError:  # numpy < 2
            from numpy.core.multiarray import _reconstruct
        safe.append(_reconstruct)
        with torch.serialization.safe_globals(safe):
            arr = torch.load(path, weights_only=True)
    if torch.is_tensor(arr):
        arr = arr.numpy()
    arr = np.asarray(arr)
    if arr.dtype != np.uint8 or arr.ndim != 4 or arr.shape[-1] != 3:
        raise ValueError(f"{path}: expected a uint8 [V, H, W, 3] view stack, got {arr.dtype} {arr.shape}")
    return arr


class MultiviewModelDataset(torch.utils.data.Dataset):
    """Same constructor as the reference (src/dataset.py:95-112).  An item is
    `(idx, views, class_id)` where `views` is the uint8 [V, H, W, 3] stack of the
    selected views (`imgs[specific_view]`, :121-122).  `transform` (a per-image CPU
    callable, the reference's form) is applied if given; the device pipeline leaves it
    None and normalises whole batches on the GPU (`ViewNormalize`)."""

    def __init__(self, root_dir, split, ending='.png', num_views=12, shuffle=True, specific_view=None,
                 transform=None):
        self.root_dir = Path(root_dir)
        with open(str(self.root_dir / 'metadata.json')) as f:
            self.metadata = json.load(f)
        self.samples = self.metadata[split]
        self.classnames = self.metadata['classnames']
        self.split = split
        self.num_views = num_views
        self.specific_view = specific_view
        self.transform = transform

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, idx):
        sample = self.samples[idx]
        class_id = self.classnames.index(sample['classname'])
        imgs = load_view_stack(self.root_dir / self.split / f"{sample['model']}.npy")
        # the reference iterates zip(imgs[specific_view], specific_view): None selects
        # nothing there (an error downstream); keep all views instead
        views = imgs if self.specific_view is None else imgs[list(self.specific_view)]
        if self.transform is not None:
            return idx, torch.stack([self.transform(v) for v in views]), class_id
        return idx, torch.from_numpy(np.ascontiguousarray(views)), class_id


class ViewNormalize:
    """The reference's per-image transforms (src/dataset.py:35-47) for a whole batch on
    the GPU: `train=True` draws one RandomHorizontalFlip decision per view from torch's
    global generator (`torch.rand(1) < p`, sample-major, view-minor: the order the
    reference's per-item transforms consume it) and flips on the device.

    out_layout "nchw" -> fp32 [B, V, 3, H, W] (the reference's batch tensor);
    "views_nhwc" -> view-major channels_last [V][B][H][W][3] exposed as [B, V, 3, H, W]
    (the engine's layout), dtype bf16 or fp32."""

    def __init__(self, train, mean=IMAGENET_MEAN, std=IMAGENET_STD, p=0.5, out_layout="nchw",
                 dtype=torch.float32, device=None):
        self.train = bool(train)
        self.mean = tuple(float(m) for m in mean)
        self.std = tuple(float(s) for s in std)
        self.p = float(p)
        if out_layout not in ("nchw", "views_nhwc"):
            raise ValueError(f"out_layout must be 'nchw' or 'views_nhwc', got {out_layout!r}")
        if dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"dtype must be fp32 or bf16, got {dtype}")
        self.out_layout = out_layout
        self.dtype = dtype
        self._device = device

    @property
    def device(self):
        if self._device is not None:
            return torch.device(self._device)
        return torch.device("cuda", torch.cuda.current_device())

    def draw_flips(self, B, V):
        """uint8 [B*V] flip flags, drawn exactly as V RandomHorizontalFlip calls per
        sample would draw them (torchvision: `if torch.rand(1) < self.p: hflip`)."""
        if not self.train:
            return None
        return torch.tensor([1 if float(torch.rand(1)) < self.p else 0 for _ in range(B * V)], dtype=torch.uint8)

    def __call__(self, views_u8, flips=None):
        """views_u8: uint8 [B, V, H, W, 3] (host, ideally pinned, or device)."""
        if views_u8.dtype != torch.uint8 or views_u8.dim() != 5 or views_u8.shape[-1] != 3:
            raise ValueError(f"expected uint8 [B, V, H, W, 3], got {views_u8.dtype} {tuple(views_u8.shape)}")
        B, V = views_u8.shape[:2]
        if flips is None:
            flips = self.draw_flips(B, V)
        return self.launch(views_u8, flips)

    def launch(self, views_u8, flips):
        """One gm_views_normalize launch on the current stream of the device."""
        B, V, H, W, _ = views_u8.shape
        x = views_u8.to(self.device, non_blocking=True).contiguous()
        fl = flips.to(self.device, non_blocking=True) if flips is not None else None
        if self.out_layout == "nchw":
            out = torch.empty(B, V, 3, H, W, dtype=self.dtype, device=self.device)
            ret, layout = out, L.GM_NCHW
        else:
            out = torch.empty(V, B, H, W, 3, dtype=self.dtype, device=self.device)
            ret, layout = out.permute(1, 0, 4, 2, 3), L.GM_NHWC
        d = L.ViewsNorm(x.data_ptr(), L.ptr(fl), B, V, H, W, 3,
                        (ctypes.c_float * 4)(*self.mean, 0.0),
                        (ctypes.c_float * 4)(*self.std, 1.0), out.data_ptr(),
                        L.GM_BF16 if self.dtype == torch.bfloat16 else L.GM_F32, layout)
        L.check(L.load().gm_views_normalize(ctypes.byref(d), L.stream_of(self.device)), "gm_views_normalize")
        return ret


def _collate(batch):
    idx = torch.tensor([b[0] for b in batch], dtype=torch.int64)
    views = torch.stack([b[1] for b in batch])
    y = torch.tensor([b[2] for b in batch], dtype=torch.int64)
    return idx, views, y


class DeviceViewLoader:
    """Iterates a DataLoader of raw uint8 view stacks and yields the reference's
    `(idx, data, class_id)` batches with `data` normalised on the GPU.  `len()` and
    re-iteration (one pass per epoch) behave like the reference's DataLoader."""

    def __init__(self, loader, transform, pin_memory=True):
        self.loader = loader
        self.transform = transform
        self.pin = pin_memory and torch.cuda.is_available()
        self.dataset = loader.dataset

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        dev = self.transform.device
        for idx, views, y in self.loader:
            if self.pin:
                views = views.pin_memory()
            data = self.transform(views)
            yield idx, data, y.to(dev, non_blocking=True)


@configurable
def get_mvdcndata(ending='.png', root_dir=None, make_npy_files=False, valid_size=0.2,
                  batch_size=8, random_seed_for_validation=10, num_views=12, num_workers=0, specific_views=None,
                  seed=777, use_cuda=True, out_layout="nchw", dtype=torch.float32, device=None):
    """Reference src/dataset.py:15-92 with the per-image CPU transforms replaced by one
    device launch per batch.  Returns (train, valid, test) loaders yielding
    (idx, data, class_id); validation draws flips like the reference (a Subset of the
    training dataset, :77-83).  `out_layout`/`dtype`/`device` are additions (defaults =
    the reference's fp32 [B, V, 3, H, W])."""
    root_dir = root_dir if root_dir is not None else os.environ.get("DATA_DIR")  # reference default (:18)
    if root_dir is None:
        raise ValueError("get_mvdcndata: no root_dir and $DATA_DIR unset (the reference reads $DATA_DIR)")
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if use_cuda and torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    kw = dict(out_layout=out_layout, dtype=dtype, device=device)
    test_tf, train_tf = ViewNormalize(False, **kw), ViewNormalize(True, **kw)

    test_dataset = MultiviewModelDataset(root_dir, 'test', ending=ending, num_views=num_views,
                                         specific_view=specific_views)
    test_loader = torch.utils.data.DataLoader(test_dataset, batch_size=batch_size, shuffle=False,
                                              num_workers=num_workers, collate_fn=_collate)
    training = MultiviewModelDataset(root_dir, 'train', ending=ending, num_views=num_views,
                                     specific_view=specific_views)
    train_idx, valid_idx = split_indices(len(training), valid_size, random_seed_for_validation)
    valid_loader = torch.utils.data.DataLoader(torch.utils.data.Subset(training, valid_idx), batch_size=batch_size,
                                               shuffle=False, num_workers=num_workers, collate_fn=_collate)
    train_loader = torch.utils.data.DataLoader(torch.utils.data.Subset(training, train_idx), batch_size=batch_size,
                                               shuffle=True, num_workers=num_workers, collate_fn=_collate)
    return (DeviceViewLoader(train_loader, train_tf), DeviceViewLoader(valid_loader, train_tf),
            DeviceViewLoader(test_loader, test_tf))


def split_indices(num_train, valid_size, random_seed_for_validation):
    """The reference's train/validation split (src/dataset.py:67-75): shuffle
    range(num_train) with random.Random(seed), the first floor(valid_size*n) are
    validation, the rest training."""
    if not (0 <= valid_size <= 1):
        raise AssertionError("[!] valid_size should be in the range [0, 1].")
    indices = list(range(num_train))
    split = int(np.floor(valid_size * num_train))
    random.Random(random_seed_for_validation).shuffle(indices)
    return indices[split:], indices[:split]
