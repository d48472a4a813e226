"""eval.py entry of the reference on MI355X (verdict row g1).

Reference eval.py:23-58: `eval_(save_path, target_data_split, pretrained_weights_path,
batch_size=128, callbacks=[])`, gin-configurable, builds `MMTM_MVCNN()` (gin-bound:
configs/eval.gin turns the cross-modal flow off with the recorded averages,
configs/recording.gin records the squeezed maps), picks the 'train' / 'val' / 'test'
loader (else NotImplementedError), and runs `evalution_loop`
(src/training_loop.py:161-200): load `{'model': state_dict}` non-strictly, one pass
over the split, history written per epoch to `{save_path}/eval_history_batch/`
(`history.pickle` when `evalution_loop.save_with_structure`, the file
`get_rescale_weights` / cur.py read back: keys `test_indices`,
`test_squeezedmaps_array_list`, each a list over epochs).

CLI:  python -m greedy_multimodal_learning_amd.evaluate SAVE_PATH CONFIG[#CONFIG...] [BINDINGS]
"""
import os

import torch

from .gin_lite import _CONFIG, configurable
from .train import _DTYPES, construct_callbacks, evaluate, gin_main, save_history


def load_pretrained(model, path):
    """Reference _load_pretrained_model (src/training_loop.py:78-83): update the model's
    state_dict with checkpoint['model'] and load it non-strictly.  Tensors only
    (weights_only=True: nothing in the file is executed)."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    sd = model.state_dict()
    sd.update(ck["model"])
    model.load_state_dict(sd, strict=False)


@configurable
def evalution_loop(model, loss_function, metrics, config, save_path, test=None, test_steps=None, use_gpu=True,
                   device_numbers=[0], custom_callbacks=[], pretrained_weights_path=None, save_with_structure=False,
                   nummodalities=2, compute_dtype="fp32"):
    """Reference src/training_loop.py:161-200 (one evaluation epoch, `test_*` keys).
    Runs in fp32 by default (the reference's arithmetic: its recorded averages feed the
    turn-off evaluation)."""
    dev = torch.device("cuda", device_numbers[0])
    if pretrained_weights_path:
        load_pretrained(model, pretrained_weights_path)
    model = model.to(dev)
    hist_dir = os.path.join(save_path, "eval_history_batch")
    os.makedirs(hist_dir, exist_ok=True)
    for c in custom_callbacks:
        c.set_save_path(save_path)
        c.set_model(model, ignore=False)
        c.set_config(config)
    logs = evaluate(model, test, "test", _DTYPES[compute_dtype], test_steps,
                    record_squeezed=bool(getattr(model, "saving_mmtm_squeeze_array", False)))
    logs["epoch"] = 0
    H = {k: [v] for k, v in logs.items()}
    save_history(H, hist_dir, save_with_structure=save_with_structure)
    for c in custom_callbacks:
        c.on_epoch_end(0, logs)
    return H


@configurable
def eval_(save_path, target_data_split, pretrained_weights_path, batch_size=128, callbacks=[]):
    """Reference eval.py:23-58."""
    from .dataset import get_mvdcndata
    from .model import MMTM_MVCNN
    from .train import acc, blend_loss
    model = MMTM_MVCNN()
    dt = _DTYPES[_CONFIG.get(("", "evalution_loop"), {}).get("compute_dtype", "fp32")]
    train, val, testing = get_mvdcndata(batch_size=batch_size, out_layout="views_nhwc", dtype=dt)
    splits = {"test": testing, "train": train, "val": val}
    if target_data_split not in splits:
        raise NotImplementedError
    target = splits[target_data_split]
    return evalution_loop(model=model, loss_function=blend_loss, metrics=[acc], config=_CONFIG, save_path=save_path,
                          test=target, test_steps=len(target), custom_callbacks=construct_callbacks(callbacks),
                          pretrained_weights_path=pretrained_weights_path)


if __name__ == "__main__":
    gin_main(eval_)
