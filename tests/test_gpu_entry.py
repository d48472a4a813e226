"""End-to-end entry surface on the GPU (verdict row g1 + f1 + f2): gin bindings with
configs/training_guided.gin's values drive `train` (device input pipeline ->
BalancedStep with the guided gate -> history + checkpoint), then the recording run
(configs/recording.gin's bindings: `eval_` on the training split with
`saving_mmtm_squeeze_array`) writes the squeezed maps, and the turn-off evaluation
(configs/eval.gin's bindings: `mmtm_off` with the recorded averages, CUR) reads them
back through `get_rescale_weights`.  Synthetic 12-view uint8 dataset, 64x64 views."""
import json
import os
import pickle

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

# values of configs/training_guided.gin (model, train, gate, loop, dataset sections)
GUIDED = """
MMTM_MVCNN.pretraining=False
MMTM_MVCNN.num_views=2
train.batch_size=4
train.lr=0.1
train.wd=0.0
train.momentum=0
train.callbacks=['CompletedStopping', 'ReduceLROnPlateau_PyTorch', 'Bias_Mitigation_Strong']
ReduceLROnPlateau_PyTorch.metric='loss'
CompletedStopping.patience=5
CompletedStopping.monitor='acc'
Bias_Mitigation_Strong.epsilon=0.01
Bias_Mitigation_Strong.curation_windowsize=5
Bias_Mitigation_Strong.starting_epoch=1
Bias_Mitigation_Strong.branchnames=['net_view_0', 'net_view_1']
Bias_Mitigation_Strong.MMTMnames = ['visual', 'skeleton']
training_loop.nummodalities=2
training_loop.n_epochs=3
training_loop.device_numbers=[0]
training_loop.checkpoint_monitor='val_acc'
get_mvdcndata.num_views=2
get_mvdcndata.num_workers=0
get_mvdcndata.specific_views=[0, 6]
"""


def _dataset(root, n_train=14, n_test=5, H=64, views=12, seed=3):
    R = np.random.default_rng(seed)
    meta = {"classnames": [f"c{i}" for i in range(40)], "train": [], "test": []}
    for split, n in (("train", n_train), ("test", n_test)):
        os.makedirs(os.path.join(root, split))
        for i in range(n):
            c = int(R.integers(40))
            meta[split].append({"classname": f"c{c}", "model": f"m{split}{i}"})
            np.save(os.path.join(root, split, f"m{split}{i}.npy"),
                    R.integers(0, 256, (views, H, H, 3), dtype=np.uint8))
    with open(os.path.join(root, "metadata.json"), "w") as f:
        json.dump(meta, f)


def _run(fn, text, save):
    from greedy_multimodal_learning_amd import gin_lite
    gin_lite.clear_config()
    try:
        gin_lite.parse_config(text)
        os.makedirs(save, exist_ok=True)
        return fn(save)
    finally:
        gin_lite.clear_config()


def test_train_record_cur_eval(tmp_path):
    from greedy_multimodal_learning_amd.evaluate import eval_
    from greedy_multimodal_learning_amd.train import train
    data = str(tmp_path / "data")
    _dataset(data)
    tsave, rsave, esave = str(tmp_path / "guided"), str(tmp_path / "rec"), str(tmp_path / "eval")
    ds = f"\nget_mvdcndata.root_dir='{data}'\n"
    H = _run(train, GUIDED + ds, tsave)
    assert len(H["loss"]) == 2 and all(np.isfinite(H["loss"]))
    assert all(len(d) == 3 for d in H["d_BDR"])  # 12 training samples (80 % of 14) at batch 4 -> 3 steps
    assert sorted(np.concatenate([H["train_indices"][0], H["val_indices"][0]]).tolist()) == list(range(14))
    for f in ("model_best_val.pt", "model_last_epoch.pt"):  # src/training_loop.py:39-48, src/utils.py:107-115
        ck = torch.load(os.path.join(tsave, f), weights_only=True)
        assert set(ck) == {"model", "optimizer"} and ck["optimizer"]["param_groups"][0]["lr"] == 0.1
    # the reference's train_dict metrics (src/framework.py:324-327)
    assert all(0 <= a <= 100 for k in ("acc", "acc_modal_0", "acc_modal_1") for a in H[k])
    with open(os.path.join(tsave, "history.pickle"), "rb") as f:
        assert "train_indices" in pickle.load(f)

    # recording (configs/recording.gin): squeezed maps of every training sample
    rec = ds + f"""
MMTM_MVCNN.num_views=2
MMTM_MVCNN.saving_mmtm_squeeze_array=True
eval_.target_data_split='train'
eval_.batch_size=4
eval_.pretrained_weights_path='{tsave}/model_best_val.pt'
evalution_loop.save_with_structure=True
get_mvdcndata.valid_size=0
get_mvdcndata.specific_views=[0, 6]
"""
    R = _run(eval_, rec, rsave)
    sq = R["test_squeezedmaps_array_list"][0]
    assert len(sq) == 4 and len(sq[0]) == 3 and sq[0][0][0].shape == (4, 128)  # site s2, view 0: [B, C]
    assert sorted(R["test_indices"][0].tolist()) == list(range(14))

    # CUR evaluation (configs/eval.gin): cross-modal flow off, averages from the recording
    ev = ds + f"""
MMTM_MVCNN.num_views=2
MMTM_MVCNN.mmtm_off=True
MMTM_MVCNN.mmtm_rescale_eval_file_path='{rsave}/eval_history_batch'
MMTM_MVCNN.mmtm_rescale_training_file_path='{tsave}'
eval_.target_data_split='test'
eval_.batch_size=8
eval_.pretrained_weights_path='{tsave}/model_best_val.pt'
get_mvdcndata.specific_views=[0, 6]
"""
    E = _run(eval_, ev, esave)
    assert np.isfinite(E["test_loss"][0]) and 0 <= E["test_acc"][0] <= 100
    assert "test_acc_modal_0" in E and "test_acc_modal_1" in E
