"""Conditional-utilisation-rate inputs: dataset-average squeezes for the
turn-off (mmtm_off) evaluation.

Reference: `get_mmtm_outputs` / `get_rescale_weights`
(src/balanced_mmtm.py:157-206).  eval.py + configs/recording.gin record, per
batch, the squeezed maps of the 3 MMTM sites for both views
(`test_squeezedmaps_array_list`, src/framework.py:160-161) together with
`test_indices`; they are re-ordered into dataset order and averaged over the
training run's `train_indices` (or `val_indices`).  The histories are the
user's own pickles written by the training/eval loops (trusted local files).
"""
import os
import pickle

import numpy as np
import torch


def _history(path):
    with open(os.path.join(path, "history.pickle"), "rb") as f:
        return pickle.load(f)


def mmtm_outputs(eval_save_path, mmtm_recorded, key):
    h = _history(eval_save_path)
    data = []
    for batch in h[key][0]:
        assert mmtm_recorded == len(batch)
        for sid, views in enumerate(batch):
            if len(data) < sid + 1:
                data.append({})
            for v, arr in enumerate(views):
                data[sid].setdefault("view_%d" % v, []).append(np.array(arr))
    order = np.argsort(h["test_indices"][0])
    for site in data:
        for k in site:
            site[k] = np.concatenate(site[k])[order]
    return data


def rescale_weights(eval_save_path, training_save_path, key="test_squeezedmaps_array_list",
                    validation=False, starting_mmtmindice=1, mmtmpositions=4, device=None):
    data = mmtm_outputs(eval_save_path, mmtmpositions - starting_mmtmindice, key)
    h = _history(training_save_path)
    sel = h["val_indices"][0] if validation else h["train_indices"][0]
    out = []
    for i in range(mmtmpositions):
        if i < starting_mmtmindice:
            out.append(None)
            continue
        d = data[i - starting_mmtmindice]
        w = [d[k][sel].mean(0) for k in sorted(d)]
        if device is not None:
            w = [torch.from_numpy(np.ascontiguousarray(a)).to(device) for a in w]
        out.append(w)
    return out
