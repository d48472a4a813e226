"""Conditional-utilisation evaluation inputs (oracle side).

Restates `get_mmtm_outputs` / `get_rescale_weights` (`src/balanced_mmtm.py:157-206`):
the recorded per-batch squeezes (`test_squeezedmaps_array_list`, written by
eval.py + configs/recording.gin through `src/framework.py:160-161` and
`src/training_loop.py:65-67`) are concatenated per MMTM site and view, put back
in dataset order with argsort(test_indices), and averaged over the training
run's `train_indices` (or `val_indices`).  Result: [None, [avg_v, avg_s]@C=128,
@256, @512].  These histories are the user's own pickles (trusted local files).
"""
import os
import pickle

import numpy as np


def _load(path):
    with open(os.path.join(path, "history.pickle"), "rb") as f:
        return pickle.load(f)


def mmtm_outputs(eval_save_path, mmtm_recorded, key):
    h = _load(eval_save_path)
    sites = None
    for batch in h[key][0]:
        assert mmtm_recorded == len(batch)
        if sites is None:
            sites = [dict() for _ in range(len(batch))]
        for sid, views in enumerate(batch):
            for v, arr in enumerate(views):
                sites[sid].setdefault("view_%d" % v, []).append(np.asarray(arr))
    order = np.argsort(h["test_indices"][0])
    return [{k: np.concatenate(v)[order] for k, v in s.items()} for s in sites]


def rescale_weights(eval_save_path, training_save_path, key="test_squeezedmaps_array_list",
                    validation=False, starting_mmtmindice=1, mmtmpositions=4):
    data = mmtm_outputs(eval_save_path, mmtmpositions - starting_mmtmindice, key)
    h = _load(training_save_path)
    sel = h["val_indices"][0] if validation else h["train_indices"][0]
    out = []
    for i in range(mmtmpositions):
        if i < starting_mmtmindice:
            out.append(None)
        else:
            d = data[i - starting_mmtmindice]
            out.append([d[k][sel].mean(0) for k in sorted(d)])
    return out
