"""Loss and metric of the reference's train.py (train.py:23-40)."""
import torch
import torch.nn.functional as F


def blend_loss(y_hat, y):
    """Sum over branches of the mean cross-entropy of each branch's logits
    (the loss never sees the averaged logits).  HIP tensors: one fused launch each
    way (head.branch_xent)."""
    from .head import branch_xent, xent_ok
    if len(y_hat) and xent_ok(y_hat, y):
        return branch_xent(y_hat, y)
    return sum(F.cross_entropy(logits, y) for logits in y_hat)


def acc(y_pred, y_true):
    """Top-1 accuracy in percent; a list of branch logits is averaged first.
    Reference quirk kept: labels of length 2 are read as (y, ...) (train.py:36-37)."""
    if isinstance(y_pred, list):
        y_pred = torch.stack([o.detach() for o in y_pred]).mean(0)
    target = y_true[0] if len(y_true) == 2 else y_true
    return (y_pred.argmax(1) == target).float().mean() * 100
