"""train.py / eval.py entry surface of the reference on MI355X (verdict row g1).

Reference train.py:43-70: `train(save_path, wd, lr, momentum, batch_size, callbacks)`
is gin-configurable; it builds `MMTM_MVCNN()` (gin-bound), the loaders
(`get_mvdcndata`), SGD, and the callbacks named in `train.callbacks` that exist in
`src.callbacks`, then hands everything to `training_loop` (src/training_loop.py:86-143),
whose step is Model_.train_loop (src/framework.py:295-322).

Here the same gin names and parameters (`train.*`, `training_loop.*`, `MMTM_MVCNN.*`,
`get_mvdcndata.*`, `Bias_Mitigation_Strong.*`) build the MI355X path: the device input
pipeline (dataset.py) delivers view-major channels_last batches, and every training
step is one `engine.BalancedStep` (forward, blend_loss, backward, gate, SGD fused; a
hipGraph replay).  The callbacks of training_guided.gin - `CompletedStopping`,
`ReduceLROnPlateau_PyTorch` (which lowers the engine's learning rate through the
optimizer object) and the gate - run on their reference hooks; names missing from
`src.callbacks` are skipped exactly as the reference skips them.
The loop keeps the reference's per-epoch history keys (`loss`, `acc`,
`acc_modal_{i}`, `train_indices`, `val_*`, `test_*`, plus the gate's `d_BDR`,
`curation_mode`, `caring_modality` lists) in `history.pickle` / `history.csv`, and
`model_best_val.pt` / `model_last_epoch.pt` hold `{'model', 'optimizer'}` state dicts
(src/training_loop.py:26-48, 78-83).

Arithmetic: `training_loop.compute_dtype` defaults to 'fp32', the reference's own precision,
so a reference gin config reproduces the reference's logits and CUR numbers (north_star:
1e-4); bind `training_loop.compute_dtype = 'bf16'` for the fast (benchmarked) trunk.

CLI (reference: `train.py save_path configs/x.gin [bindings]`, src/utils.py:58-68):
    python -m greedy_multimodal_learning_amd.train SAVE_PATH CONFIG[#CONFIG...] [BINDINGS]
"""
import argparse
import csv
import os
import pickle

import numpy as np
import torch

from . import _lib as L
from . import callbacks as avail_callbacks
from .gin_lite import _CONFIG, configurable, parse_config_files_and_bindings
from .losses import acc, blend_loss  # noqa: F401  (reference train.py exports both)

_DTYPES = {"bf16": torch.bfloat16, "fp32": torch.float32}


def construct_callbacks(names):
    """Reference train.py:53-57: instantiate (gin-bound) every named callback that the
    callbacks module provides (Bias_Mitigation_Strong / _Random, CompletedStopping,
    ReduceLROnPlateau_PyTorch); names the reference's src.callbacks does not export are
    skipped as the reference skips them."""
    out = []
    for name in names:
        cls = avail_callbacks.__dict__.get(name)
        if isinstance(cls, type) and issubclass(cls, avail_callbacks.Callback):
            out.append(cls())
    return out


def _metrics(lm, outs, y):
    return float(acc(lm, y)), [float(acc(o, y)) for o in outs]


def evaluate(model, loader, phase, compute_dtype, steps=None, record_squeezed=False, curation=(False, None)):
    """Reference Model_._eval_generator (src/framework.py:216-248): eval mode, no grad,
    size-weighted loss and accuracies, the batches' indices, and (recording runs) the
    squeezed maps per batch (`{phase}_squeezedmaps_array_list`, :160-161).  `curation`:
    the (curation_mode, caring_modality) the model is called with, as Model_ passes its
    own flags in evaluation too (src/framework.py:146-148)."""
    model.eval()
    n, loss_sum, acc_sum, accm_sum, idxs, squeezed = 0, 0.0, 0.0, None, [], []
    with torch.no_grad():
        for bi, (idx, x, y) in enumerate(loader):
            if steps is not None and bi >= steps:
                break
            with torch.autocast("cuda", dtype=compute_dtype, enabled=compute_dtype != torch.float32):
                lm, outs, _, sq = model(x, curation_mode=curation[0], caring_modality=curation[1])
            outs = [o.float() for o in outs]
            b = len(y)
            loss_sum += float(blend_loss(outs, y)) * b
            a, am = _metrics(lm.float(), outs, y)
            acc_sum += a * b
            accm_sum = np.array(am) * b if accm_sum is None else accm_sum + np.array(am) * b
            n += b
            idxs.append(idx.numpy())
            if record_squeezed:
                squeezed.append([[v.detach().float().cpu().numpy() if torch.is_tensor(v) else np.asarray(v) for v in site]
                                 for site in sq if site is not None])
    out = {f"{phase}_loss": loss_sum / max(n, 1), f"{phase}_acc": acc_sum / max(n, 1),
           f"{phase}_indices": np.concatenate(idxs) if idxs else np.zeros(0, np.int64)}
    for i, v in enumerate(accm_sum if accm_sum is not None else []):
        out[f"{phase}_acc_modal_{i}"] = v / n
    if record_squeezed:
        out[f"{phase}_squeezedmaps_array_list"] = squeezed
    model.train(True)
    return out


def save_history(H, save_path, save_with_structure=True):
    """Reference _save_history_csv (src/training_loop.py:53-67): scalar columns to
    history.csv, the whole history (lists per epoch) to history.pickle."""
    scalars = [k for k, v in H.items() if isinstance(v[-1], (int, float, bool, str, np.floating, np.integer))]
    with open(os.path.join(save_path, "history.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(scalars)
        for row in zip(*[H[k] for k in scalars]):
            w.writerow(row)
    if save_with_structure:
        with open(os.path.join(save_path, "history.pickle"), "wb") as f:
            pickle.dump(H, f, pickle.HIGHEST_PROTOCOL)


@configurable
def training_loop(model, loss_function, metrics, optimizer, config, save_path, steps_per_epoch, train=None,
                  valid=None, test=None, test_steps=None, validation_steps=None, use_gpu=True, device_numbers=[0],
                  custom_callbacks=[], checkpoint_monitor="val_acc", n_epochs=100, verbose=True, nummodalities=2,
                  compute_dtype="fp32", graphs=True):
    """Reference src/training_loop.py:86-143 + Model_.train_loop (src/framework.py:
    250-330) on the fused engine.  `optimizer` is the (lr, momentum, wd) triple of the
    reference's SGD (only momentum = wd = 0, as every config uses, is fused; a torch SGD
    over the model's parameters holds the learning rate and the state_dict the
    checkpoints carry, and ReduceLROnPlateau_PyTorch drives it); `metrics` and
    `loss_function` are the reference's acc / blend_loss (fixed in the engine).
    Epochs 1 .. n_epochs-1 as the reference (`epochs=n_epochs - 1`).  Per epoch the
    history gets the reference's train_dict keys (`loss`, `acc`, `acc_modal_{i}`,
    `train_indices`), the validation / test dicts, and the gate's per-step lists; a NaN
    step loss or CompletedStopping ends training after that epoch (:321-322, :343);
    `model_best_val.pt` (best `checkpoint_monitor`) and `model_last_epoch.pt` (every
    epoch) hold {'model', 'optimizer'} (src/training_loop.py:26-48, src/utils.py:107-115)."""
    import math

    from .engine import BalancedStep
    lr, momentum, wd = optimizer
    if momentum != 0 or wd != 0:
        raise NotImplementedError("the fused step implements SGD with momentum = weight_decay = 0 "
                                  "(train.momentum / train.wd of every reference config)")
    dev = torch.device("cuda", device_numbers[0])
    model = model.to(dev)
    gates = [c for c in custom_callbacks if hasattr(c, "on_backward_end")
             and isinstance(c, (avail_callbacks.Bias_Mitigation_Strong, avail_callbacks.Bias_Mitigation_Random))]
    if len(gates) > 1:
        raise ValueError("at most one gating callback")
    gate = gates[0] if gates else None
    cdt = _DTYPES[compute_dtype]
    step = BalancedStep(model, lr=lr, gate=gate, compute_dtype=cdt, channels_last=True, graphs=graphs)
    # the reference's optimizer object (never stepped: the engine's fused pass applies the
    # update with the learning rate read from it)
    opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=momentum, weight_decay=wd)
    flags = step.flags  # the gate's model_pytoune; every other callback shares it
    flags.stop_training = False
    others = [c for c in custom_callbacks if c is not gate]
    for c in custom_callbacks:
        c.set_save_path(save_path)
        c.set_config(config)
        c.set_optimizer(opt)
        if c is not gate:
            c.set_model(model, ignore=False)
            c.set_model_pytoune(flags)
    for c in others:
        c.on_train_begin({})
    H = {}
    best = None
    for epoch in range(1, n_epochs):
        step.on_epoch_begin(epoch)
        for c in others:
            c.on_epoch_begin(epoch, {})
        # Per-step numbers stay on the device and are read once per epoch (no host sync per
        # step): loss / accuracy sums as device scalars, the device gate's state snapshotted
        # per step.  A callback that overrides on_batch_end gets its batch_logs every step
        # (the only case that reads them), at the cost of that sync.
        per_batch = [c for c in others if type(c).on_batch_end is not avail_callbacks.Callback.on_batch_end]
        n = 0
        loss_sum = torch.zeros((), device=dev, dtype=torch.float64)
        acc_sum = torch.zeros((), device=dev, dtype=torch.float64)
        accm_sum = torch.zeros(nummodalities, device=dev, dtype=torch.float64)
        idxs, d_bdr, cur, caring, snaps = [], [], [], [], []
        for bi, (idx, x, y) in enumerate(train):
            if steps_per_epoch is not None and bi >= steps_per_epoch:
                break
            for c in others:
                c.on_batch_begin(bi + 1, {})
            step.lr = float(opt.param_groups[0]["lr"])
            loss = step(x, y)
            outs = step.last_outs
            with torch.no_grad():  # Model_._compute_loss_and_metrics (src/framework.py:152-156)
                a = acc(list(outs), y)
                am = torch.stack([acc(o, y) for o in outs])
            b = len(y)
            loss_sum += loss.double() * b
            acc_sum += a.double() * b
            accm_sum += am.double() * b
            n += b
            idxs.append(idx.numpy())
            if gate is not None:
                if step.device_gate:
                    snaps.append(step.gate_state.clone())
                else:  # host gate: its decision is already on the host
                    d_bdr.append(float(getattr(gate, "d_BDR", 0.0) or 0.0))
                    cur.append(bool(step.flags.curation_mode))
                    caring.append(step.flags.caring_modality)
            if per_batch:
                batch_logs = {"batch": bi + 1, "size": b, "loss": float(loss), "acc": float(a),
                              **{f"acc_modal_{i}": float(v) for i, v in enumerate(am)}}
                for c in per_batch:
                    c.on_batch_end(bi + 1, batch_logs)
        if snaps:  # decode the device gate's per-step states (one copy)
            cls = L.GateStateN if step.gate_n else L.GateState
            for raw in torch.stack(snaps).cpu().numpy():
                st = cls.from_buffer_copy(raw.tobytes())
                d_bdr.append(float(st.d_bdr))
                cur.append(bool(st.curation_mode))
                caring.append(None if st.caring < 0 else int(st.caring))
        loss_mean = float(loss_sum) / max(n, 1)
        if math.isnan(loss_mean):  # a NaN step loss ends training after this epoch (:321-322)
            flags.stop_training = True
        logs = {"epoch": epoch, "loss": loss_mean, "acc": float(acc_sum) / max(n, 1),
                **{f"acc_modal_{i}": float(v) / max(n, 1) for i, v in enumerate(accm_sum.cpu())},
                "train_indices": np.concatenate(idxs) if idxs else np.zeros(0, np.int64)}
        if gate is not None:
            logs.update({"d_BDR": d_bdr, "curation_mode": cur, "caring_modality": caring})
        # validation / test with the model's current curation flags (src/framework.py:146-148)
        if step.device_gate:
            step.sync_gate()
        fl = (bool(step.flags.curation_mode), step.flags.caring_modality)
        if valid is not None:
            logs.update(evaluate(model, valid, "val", cdt, validation_steps, curation=fl))
        if test is not None:
            logs.update(evaluate(model, test, "test", cdt, test_steps, curation=fl))
        for k, v in logs.items():
            H.setdefault(k, []).append(v)
        # the reference's callback order: the custom callbacks (ReduceLROnPlateau_PyTorch,
        # CompletedStopping) before the default checkpoint callbacks (src/training_loop.py:98-110),
        # so a checkpoint carries the optimizer state after this epoch's learning-rate change
        for c in others:
            c.on_epoch_end(epoch, logs)
        if save_path:
            save_history(H, save_path)
            ck = {"model": model.state_dict(), "optimizer": opt.state_dict()}
            mon = logs.get(checkpoint_monitor)
            if mon is not None and (best is None or mon > best):
                best = mon
                torch.save(ck, os.path.join(save_path, "model_best_val.pt"))
            torch.save(ck, os.path.join(save_path, "model_last_epoch.pt"))
        if verbose:
            print(f"epoch {epoch}: loss {logs['loss']:.4f} acc {logs['acc']:.2f} lr {step.lr:g}" +
                  (f" val_acc {logs['val_acc']:.2f}" if "val_acc" in logs else ""), flush=True)
        if flags.stop_training:
            break
    for c in others:
        c.on_train_end({})
    return H


@configurable
def train(save_path, wd, lr, momentum, batch_size, callbacks=[]):
    """Reference train.py:43-70."""
    from .dataset import get_mvdcndata
    from .model import MMTM_MVCNN
    model = MMTM_MVCNN()
    dt = _DTYPES[_CONFIG.get(("", "training_loop"), {}).get("compute_dtype", "fp32")]
    train_l, valid_l, test_l = get_mvdcndata(batch_size=batch_size, out_layout="views_nhwc", dtype=dt)
    return training_loop(model=model, loss_function=blend_loss, metrics=[acc], optimizer=(lr, momentum, wd),
                         config=_CONFIG, save_path=save_path, steps_per_epoch=len(train_l), train=train_l,
                         valid=valid_l, test=test_l, validation_steps=len(valid_l), test_steps=len(test_l),
                         custom_callbacks=construct_callbacks(callbacks))


def gin_main(fn, argv=None):
    """Reference src/utils.py:58-68 (argh CLI): SAVE_PATH CONFIG[#CONFIG] [BINDINGS]."""
    ap = argparse.ArgumentParser()
    ap.add_argument("save_path")
    ap.add_argument("config")
    ap.add_argument("bindings", nargs="?", default="")
    a = ap.parse_args(argv)
    parse_config_files_and_bindings(a.config.split("#"), a.bindings.replace("#", "\n"))
    os.makedirs(a.save_path, exist_ok=True)
    return fn(a.save_path)


if __name__ == "__main__":
    gin_main(train)
