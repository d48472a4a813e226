"""Conditional-learning-speed gating, loss and metric (oracle side).

* `param_group(name, branchnames, MMTMnames)` - the substring grouping of
  `Bias_Mitigation_Strong.compute_BDR` (`src/callbacks.py:207-223`): names with
  'mmtm' go to bypass[i] if they contain MMTMnames[i], to ALL bypass groups if
  they contain none (the shared fc_squeeze); other names go to main[i] if they
  contain branchnames[i].
* `group_sums(named)` - per-group sum of w^2 and g^2 (`:203-205`: fp32
  `(p**2).sum()` per tensor, python-float accumulation).
* `BDRState` - accumulation of M's and d_BDR (`:225-233`), and the
  `on_backward_end` / `on_epoch_begin` state machine (`:240-267`).
* `RandomGate` - `Bias_Mitigation_Random` (`:269-302`).
* `blend_loss` / `acc` - `train.py:23-40`.
"""
import math
import random

import numpy as np
import torch


def param_group(name, branchnames=("net_view_0", "net_view_1"), MMTMnames=("visual", "skeleton")):
    """Return (main_mask, bypass_mask) as tuples of bools, one per branch."""
    nb = len(branchnames)
    if "mmtm" in name:
        hit = [m in name for m in MMTMnames]
        if not any(hit):
            return (False,) * nb, (True,) * len(MMTMnames)
        return (False,) * nb, tuple(hit)
    return tuple(b in name for b in branchnames), (False,) * len(MMTMnames)


def group_sums(named, branchnames=("net_view_0", "net_view_1"), MMTMnames=("visual", "skeleton")):
    """named: iterable of (name, param_tensor, grad_tensor). Returns dict of lists."""
    nb = len(branchnames)
    wn_main, gn_main = [0.0] * nb, [0.0] * nb
    wn_by, gn_by = [0.0] * len(MMTMnames), [0.0] * len(MMTMnames)
    for name, p, g in named:
        wn = float((p.detach().float() ** 2).sum())
        gn = float((g.detach().float() ** 2).sum())
        main, by = param_group(name, branchnames, MMTMnames)
        for i, f in enumerate(main):
            if f:
                wn_main[i] += wn
                gn_main[i] += gn
        for i, f in enumerate(by):
            if f:
                wn_by[i] += wn
                gn_by[i] += gn
    return dict(wn_main=wn_main, gn_main=gn_main, wn_bypass=wn_by, gn_bypass=gn_by)


class BDRState:
    """Bias_Mitigation_Strong without the framework plumbing."""

    def __init__(self, epsilon, curation_windowsize, starting_epoch=2):
        self.epsilon = epsilon
        self.curation_windowsize = curation_windowsize
        self.starting_epoch = starting_epoch
        self.on_train_begin()

    def on_train_begin(self):
        self.M_bypass = [0.0, 0.0]
        self.M_main = [0.0, 0.0]
        self.curation_mode = False
        self.caring_modality = None
        self.unlock = False
        self.d_BDR = None
        self.curation_step = 0

    def on_epoch_begin(self, epoch):
        if epoch >= self.starting_epoch:
            self.unlock = True

    def update(self, sums):
        for i in range(2):
            self.M_bypass[i] += sums["gn_bypass"][i] / sums["wn_bypass"][i]
            self.M_main[i] += sums["gn_main"][i] / sums["wn_main"][i]
        bdr0 = np.log10(self.M_bypass[0] / self.M_main[0])
        bdr1 = np.log10(self.M_bypass[1] / self.M_main[1])
        return bdr0 - bdr1

    def needs_sums(self):
        return (not self.unlock) or (not self.curation_mode)

    def on_backward_end(self, sums_fn):
        if self.unlock:
            if not self.curation_mode:
                self.d_BDR = self.update(sums_fn())
                if abs(self.d_BDR) > self.epsilon:
                    self.curation_mode = True
                    self.curation_step = 0
                    s = np.sign(self.d_BDR)
                    if s == -1:
                        self.caring_modality = 1
                    elif s == 1:
                        self.caring_modality = 0
                else:
                    self.curation_mode = False
                    self.caring_modality = 0
            else:
                self.curation_step += 1
                if self.curation_step == self.curation_windowsize:
                    self.curation_mode = False
        else:
            self.d_BDR = self.update(sums_fn())
            self.curation_mode = False
            self.caring_modality = 0


class RandomGate:
    def __init__(self, starting_epoch=2, rng=random):
        self.rng = rng
        self.starting_epoch = starting_epoch
        self.curation_mode = False
        self.caring_modality = None
        self.unlock = False

    def on_epoch_begin(self, epoch):
        if epoch >= self.starting_epoch:
            self.unlock = True

    def on_backward_end(self):
        if self.unlock:
            mode = self.rng.choice([0, 1, 2])
            self.curation_mode, self.caring_modality = {0: (False, 0), 1: (True, 1), 2: (True, 0)}[mode]
        else:
            self.curation_mode, self.caring_modality = False, 0


def blend_loss(y_hat, y):
    return sum(torch.nn.functional.cross_entropy(p, y) for p in y_hat)


def acc(y_pred, y_true):
    if isinstance(y_pred, list):
        y_pred = torch.stack([o.detach() for o in y_pred], 0).mean(0)
    pred = y_pred.argmax(1) if y_pred.dim() == 2 else y_pred
    tgt = y_true[0] if len(y_true) == 2 else y_true
    return (pred == tgt).float().mean() * 100


def isnan(x):
    return math.isnan(x)
