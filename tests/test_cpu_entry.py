"""train.py / eval.py entry surface (verdict row g1) on the CPU: the `gin` shim resolves
the reference's imports, the reference configs bind the entry points' parameters and
callbacks (all three of training_guided.gin's), unknown callback names are skipped as in
the reference (train.py:53-57), and the two epoch-level callbacks behave like the
reference's (src/callbacks.py:305-348)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIGS = os.path.join(os.environ.get("GREEDYMML_REF", "/root/reference"), "configs")


def test_gin_shim_surface():
    sys.path.insert(0, os.path.join(ROOT, "compat"))
    try:
        import gin
        from gin.config import _CONFIG, _OPERATIVE_CONFIG  # noqa: F401  (src/model.py:10, src/callbacks.py:22)
        assert callable(gin.configurable) and callable(gin.parse_config_files_and_bindings)
        from greedy_multimodal_learning_amd import gin_lite
        assert _CONFIG is gin_lite._CONFIG
    finally:
        sys.path.remove(os.path.join(ROOT, "compat"))


def test_training_guided_binds_train_and_callbacks():
    from greedy_multimodal_learning_amd import gin_lite
    from greedy_multimodal_learning_amd.train import construct_callbacks
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Strong
    if not os.path.exists(os.path.join(CONFIGS, "training_guided.gin")):
        pytest.skip("reference configs not mounted")
    gin_lite.clear_config()
    try:
        gin_lite.parse_config_files_and_bindings([os.path.join(CONFIGS, "training_guided.gin")], "train.batch_size=4")
        assert gin_lite.query("train", "lr") == 0.1 and gin_lite.query("train", "batch_size") == 4
        assert gin_lite.query("get_mvdcndata", "specific_views") == [0, 6]
        from greedy_multimodal_learning_amd.callbacks import CompletedStopping, ReduceLROnPlateau_PyTorch
        cbs = construct_callbacks(gin_lite.query("train", "callbacks") + ["NotACallback"])
        assert [type(c) for c in cbs] == [CompletedStopping, ReduceLROnPlateau_PyTorch, Bias_Mitigation_Strong]
        assert (cbs[0].monitor, cbs[0].patience) == ("acc", 5) and cbs[1].metric == "loss"
        g = cbs[2]
        assert (g.epsilon, g.curation_windowsize, g.starting_epoch) == (0.01, 5, 1)
        assert g.branchnames == ["net_view_0", "net_view_1"]
    finally:
        gin_lite.clear_config()


def test_train_rejects_momentum():
    from greedy_multimodal_learning_amd.train import training_loop
    with pytest.raises(NotImplementedError):
        training_loop(model=None, loss_function=None, metrics=[], optimizer=(0.1, 0.9, 0.0), config={},
                      save_path=None, steps_per_epoch=1)


class _Loop:
    stop_training = False


def test_completed_stopping_counts_epochs_at_100():
    """src/callbacks.py:305-331: the count of epochs with acc == 100 is cumulative."""
    from greedy_multimodal_learning_amd.callbacks import CompletedStopping
    c = CompletedStopping(patience=3)
    loop = _Loop()
    c.set_model_pytoune(loop)
    c.on_train_begin({})
    for ep, a in enumerate([100, 90, 100, 99.9], 1):
        c.on_epoch_end(ep, {"acc": a})
        assert not loop.stop_training
    c.on_epoch_end(5, {"acc": 100.0})
    assert loop.stop_training and c.stopped_epoch == 5


def test_reduce_lr_on_plateau_matches_torch_scheduler():
    """src/callbacks.py:334-348: factor 0.3 after `patience` epochs without a 1e-3 relative
    improvement of the training loss, floor 1e-6; the engine reads the optimizer's lr."""
    import torch
    from greedy_multimodal_learning_amd.callbacks import ReduceLROnPlateau_PyTorch
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=0.1)
    ref_opt = torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=0.1)
    ref = torch.optim.lr_scheduler.ReduceLROnPlateau(ref_opt, mode="min", factor=0.3, patience=2, threshold=1e-3,
                                                     threshold_mode="rel", cooldown=0, min_lr=1e-6, eps=1e-8)
    c = ReduceLROnPlateau_PyTorch(metric="loss", patience=2)
    c.set_optimizer(opt)
    c.on_train_begin({})
    losses = [3.0, 2.9, 2.899, 2.8995, 2.9, 2.5, 2.6, 2.6, 2.6, 2.6, 2.6, 2.6] + [2.6] * 40
    lrs = []
    for ep, l in enumerate(losses, 1):
        c.on_epoch_end(ep, {"loss": l})
        ref.step(l)
        lrs.append(opt.param_groups[0]["lr"])
        assert opt.param_groups[0]["lr"] == ref_opt.param_groups[0]["lr"]
    assert lrs[4] == pytest.approx(0.03) and min(lrs) == pytest.approx(1e-6)
