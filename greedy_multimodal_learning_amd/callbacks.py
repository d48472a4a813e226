"""Conditional-learning-speed gating on MI355X: drop-in for the gating classes
of the reference's `src.callbacks`.

`Bias_Mitigation_Strong(epsilon, curation_windowsize, branchnames,
starting_epoch=2, MMTMnames=['visual','skeleton'])` and
`Bias_Mitigation_Random()` keep the reference's gin parameters, hook protocol
(`set_model`, `set_model_pytoune`, `on_train_begin`, `on_epoch_begin`,
`on_backward_end`, `on_batch_end`; src/callbacks.py:94-170) and state machine
(src/callbacks.py:173-302).  `compute_BDR` replaces the reference's per-tensor
`(p**2).sum().item()` / `(g**2).sum().item()` loop (284 host syncs per step,
:203-205) by ONE multi-tensor HIP pass (`gm_group_sumsq`) that produces every
group's sums at once, followed by a single 8-double device->host copy.

Group semantics (:207-223): names containing 'mmtm' go to bypass[i] when they
contain MMTMnames[i], to all bypass groups when they contain none (the shared
fc_squeeze); other names go to main[i] when they contain branchnames[i].
"""
import ctypes
import random

import numpy as np
import torch

from . import _lib as L
from .gin_lite import configurable


class Callback(object):
    """Hook protocol of the reference (src/callbacks.py:94-170)."""

    def __init__(self):
        pass

    def set_config(self, config):
        self.config = config

    def set_meta_data(self, meta_data):
        self.meta_data = meta_data

    def set_save_path(self, save_path):
        self.save_path = save_path

    def set_optimizer(self, optimizer):
        self.optimizer = optimizer

    def set_model(self, model, ignore=True):
        if ignore:
            return
        self.model = model

    def set_model_pytoune(self, model_pytoune):
        self.model_pytoune = model_pytoune

    def set_params(self, params):
        self.params = params

    def set_dataloader(self, data):
        self.data = data

    def on_epoch_begin(self, epoch, logs):
        pass

    def on_epoch_end(self, epoch, logs):
        pass

    def on_batch_begin(self, batch, logs):
        pass

    def on_batch_end(self, batch, logs):
        pass

    def on_forward_begin(self, batch, data):
        pass

    def on_backward_end(self, batch):
        pass

    def on_train_begin(self, logs):
        pass

    def on_train_end(self, logs):
        pass

    def on_val_batch_end(self, batch, logs):
        pass


def group_masks(names, branchnames, MMTMnames):
    """Bit i = main[i] (i < len(branchnames)); bit nb+j = bypass[j].

    Substring matching as in the reference (src/callbacks.py:207-223); when one
    branch name contains another (net_view_1 / net_view_10 in the 12-view
    config) the longest matching name wins."""
    nb = len(branchnames)
    out = []
    for name in names:
        m = 0
        if "mmtm" in name:
            hit = [j for j, mod in enumerate(MMTMnames) if mod in name]
            for j in (hit if hit else range(len(MMTMnames))):
                m |= 1 << (nb + j)
        else:
            hit = [i for i, b in enumerate(branchnames) if b in name]
            if hit:
                longest = max(len(branchnames[i]) for i in hit)
                for i in hit:
                    if len(branchnames[i]) == longest:
                        m |= 1 << i
        out.append(m)
    return out


def _dense(t):
    return t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last))


class GroupNorms:
    """Device-side per-group sum(w^2), sum(g^2) over a fixed parameter list.

    `sums(grad_scale=1.0, lr=0.0)` launches gm_group_sumsq (optionally fused with
    the SGD update) and returns a float64 device tensor [2*ngroups] (no sync).
    """

    def __init__(self, named_params, branchnames, MMTMnames):
        self.names = [n for n, _ in named_params]
        self.params = [p for _, p in named_params]
        self.ngroups = len(branchnames) + len(MMTMnames)
        self.masks = group_masks(self.names, branchnames, MMTMnames)
        self.total = int(sum(p.numel() for p in self.params))
        self.device = self.params[0].device
        self._key = None
        self._table = None
        self._scratch = None
        self._out = None

    def _build(self):
        key = tuple((p.data_ptr(), 0 if p.grad is None else p.grad.data_ptr()) for p in self.params)
        if key == self._key:
            return
        for p in self.params:
            if p.dtype != torch.float32 or not _dense(p):
                raise L.GreedyMMLError("group norms need dense fp32 parameters")
            if p.grad is not None and (p.grad.dtype != torch.float32 or not _dense(p.grad)
                                       or p.grad.stride() != p.stride()):
                raise L.GreedyMMLError("group norms need dense fp32 gradients laid out like the parameter")
        n = len(self.params)
        tab = (L.Tensor * n)()
        off = 0
        for i, p in enumerate(self.params):
            tab[i] = L.Tensor(p.data_ptr(), 0 if p.grad is None else p.grad.data_ptr(),
                              p.numel(), off, self.masks[i], 0)
            off += p.numel()
        host = torch.frombuffer(bytearray(bytes(tab)), dtype=torch.uint8)
        self._table = host.to(self.device)
        self._key = key
        if self._scratch is None:
            need = L.load().gm_group_sumsq_scratch(self.total)
            self._scratch = torch.empty(need, dtype=torch.uint8, device=self.device)
            self._out = torch.empty(2 * self.ngroups, dtype=torch.float64, device=self.device)

    def sums(self, grad_scale=1.0, lr=0.0, gate=None, gate_n=False):
        """The step's group sums (and the fused SGD when lr != 0); gate (a device gm_gate_state /
        gm_gate_state_n tensor): the on-device gate's step runs in the same finalize launch."""
        L.load()
        if not self.params[0].is_cuda:
            raise L.GreedyMMLError("group norms run on HIP devices only (no CPU fallback)")
        self._build()
        out = torch.empty(2 * self.ngroups, dtype=torch.float64, device=self.device)
        args = (self._table.data_ptr(), len(self.params), self.total, self.ngroups, float(grad_scale), float(lr),
                out.data_ptr(), self._scratch.data_ptr(), self._scratch.numel())
        if gate is not None:
            L.check(L.load().gm_group_sumsq_gate(*args, gate.data_ptr(), int(bool(gate_n)),
                                                 L.stream_of(self.device)), "gm_group_sumsq_gate")
        else:
            L.check(L.load().gm_group_sumsq(*args, L.stream_of(self.device)), "gm_group_sumsq")
        return out


def bdr_values(M_bypass, M_main, s, nb):
    """Accumulate the M's from one step's group sums (host float64) and return the
    per-branch BDR_i = log10(M_bypass_i / M_main_i) (src/callbacks.py:225-232).
    s = [w_main0, g_main0, ..., w_main{nb-1}, g_main{nb-1}, w_by0, g_by0, ...]."""
    for i in range(nb):
        M_main[i] += s[2 * i + 1] / s[2 * i]
        M_bypass[i] += s[2 * (nb + i) + 1] / s[2 * (nb + i)]
    return [np.log10(M_bypass[i] / M_main[i]) for i in range(nb)]


def bdr_update(M_bypass, M_main, s, nb):
    """Two branches: d_BDR = BDR_0 - BDR_1 (src/callbacks.py:233)."""
    b = bdr_values(M_bypass, M_main, s, nb)
    return b[0] - b[1]


def bdr_decision(bdr):
    """N-branch generalisation (build decision): spread = max - min of
    the BDRs and the branch to care for = argmax (first on ties).  At two branches
    this is |BDR_0 - BDR_1| with caring = 1 iff d_BDR < 0, the reference's rule
    (src/callbacks.py:244-252)."""
    hi = int(np.argmax(bdr))
    return float(np.max(bdr) - np.min(bdr)), hi


@configurable
class Bias_Mitigation_Strong(Callback):
    def __init__(self, epsilon, curation_windowsize, branchnames, starting_epoch=2,
                 MMTMnames=['visual', 'skeleton']):
        self.epsilon = epsilon
        self.branchnames = list(branchnames)
        self.MMTMnames = list(MMTMnames)
        self.curation_windowsize = curation_windowsize
        self.starting_epoch = starting_epoch
        self._norms = None
        # set by a fused engine: group sums already computed this step (device tensor)
        self.pending_sums = None
        super().__init__()

    def on_train_begin(self, logs):
        self.M_bypass_modal_0 = 0
        self.M_bypass_modal_1 = 0
        self.M_main_modal_0 = 0
        self.M_main_modal_1 = 0
        nb = len(self.branchnames)
        self.M_bypass = [0.0] * nb  # N-branch accumulators (nb > 2)
        self.M_main = [0.0] * nb
        self.BDR = None
        self.model_pytoune.curation_mode = False
        self.model_pytoune.caring_modality = None
        self.unlock = False

    def group_sums(self):
        """Device float64 [8]: (w, g) sums of main0, main1, bypass0, bypass1."""
        if self.pending_sums is not None:
            s, self.pending_sums = self.pending_sums, None
            return s
        named = list(self.model.named_parameters())
        if self._norms is None or self._norms.names != [n for n, _ in named]:
            self._norms = GroupNorms(named, self.branchnames, self.MMTMnames)
        return self._norms.sums()

    def compute_BDR(self):
        s = self.group_sums().cpu().numpy()  # the step's single host sync
        nb = len(self.branchnames)
        if nb != 2:
            # N branches: d_BDR reports the BDR spread (max - min), decision = argmax
            self.BDR = bdr_values(self.M_bypass, self.M_main, s, nb)
            d, self._argmax = bdr_decision(self.BDR)
            return d
        M_by = [self.M_bypass_modal_0, self.M_bypass_modal_1]
        M_main = [self.M_main_modal_0, self.M_main_modal_1]
        d = bdr_update(M_by, M_main, s, len(self.branchnames))
        self.M_bypass_modal_0, self.M_bypass_modal_1 = M_by
        self.M_main_modal_0, self.M_main_modal_1 = M_main
        return d

    def on_batch_end(self, batch, logs):
        logs['curation_mode'] = float(self.model_pytoune.curation_mode)
        logs['caring_modality'] = self.model_pytoune.caring_modality
        logs['d_BDR'] = self.d_BDR

    def needs_bdr(self):
        """True when on_backward_end of this step will call compute_BDR."""
        return (not self.unlock) or (not self.model_pytoune.curation_mode)

    def on_backward_end(self, batch):
        mp = self.model_pytoune
        if self.unlock:
            if not mp.curation_mode:
                self.d_BDR = self.compute_BDR()
                if abs(self.d_BDR) > self.epsilon:
                    biased_direction = np.sign(self.d_BDR)
                    mp.curation_mode = True
                    self.curation_step = 0
                    if len(self.branchnames) != 2:
                        mp.caring_modality = self._argmax
                    elif biased_direction == -1:
                        mp.caring_modality = 1
                    elif biased_direction == 1:
                        mp.caring_modality = 0
                else:
                    mp.curation_mode = False
                    mp.caring_modality = 0
            else:
                self.pending_sums = None
                self.curation_step += 1
                if self.curation_step == self.curation_windowsize:
                    mp.curation_mode = False
        else:
            self.d_BDR = self.compute_BDR()
            mp.curation_mode = False
            mp.caring_modality = 0

    def on_epoch_begin(self, epoch, logs):
        if epoch >= self.starting_epoch:
            self.unlock = True


@configurable
class Bias_Mitigation_Random(Callback):
    """Random gating (src/callbacks.py:269-302): python `random` global RNG."""

    def on_train_begin(self, logs):
        self.model_pytoune.curation_mode = False
        self.model_pytoune.caring_modality = None
        self.unlock = False
        self.starting_epoch = 2

    def on_batch_end(self, batch, logs):
        logs['curation_mode'] = float(self.model_pytoune.curation_mode)
        logs['caring_modality'] = self.model_pytoune.caring_modality

    def needs_bdr(self):
        return False

    def on_backward_end(self, batch):
        mp = self.model_pytoune
        if self.unlock:
            mode = random.choice([0, 1, 2])
            if mode == 0:
                mp.curation_mode, mp.caring_modality = False, 0
            elif mode == 1:
                mp.curation_mode, mp.caring_modality = True, 1
            else:
                mp.curation_mode, mp.caring_modality = True, 0
        else:
            mp.curation_mode, mp.caring_modality = False, 0

    def on_epoch_begin(self, epoch, logs):
        if epoch >= self.starting_epoch:
            self.unlock = True


@configurable
class CompletedStopping(Callback):
    """Reference src/callbacks.py:305-331: stop training once the monitored epoch metric
    (training accuracy by default) has been exactly 100 in `patience` epochs.  The count
    is cumulative (never reset when the metric drops), as in the reference."""

    def __init__(self, *, monitor='acc', patience=5, verbose=True):
        super().__init__()
        self.monitor = monitor
        self.patience = patience
        self.verbose = verbose
        self.stopped_epoch = 0

    def on_train_begin(self, logs):
        self.stopped_epoch = 0
        self.counter = 0

    def on_epoch_end(self, epoch, logs):
        if logs[self.monitor] == 100:
            self.counter += 1
        if self.counter >= self.patience:
            self.stopped_epoch = epoch
            self.model_pytoune.stop_training = True

    def on_train_end(self, logs):
        if self.stopped_epoch > 0 and self.verbose:
            print('Epoch %05d: completed stopping' % (self.stopped_epoch + 1))


@configurable
class ReduceLROnPlateau_PyTorch(Callback):
    """Reference src/callbacks.py:334-348: torch's ReduceLROnPlateau on an epoch metric
    (`loss` in training_guided.gin), mode 'min', threshold 1e-3 relative, min_lr 1e-6.
    It drives the optimizer the loop hands over (set_optimizer); the fused engine reads
    that optimizer's learning rate before every step (a new rate is a new captured graph).
    The reference's verbose=True is dropped: a TypeError on torch >= 2.7."""

    def __init__(self, metric, factor=0.3, patience=10):
        super().__init__()
        self.metric = metric
        self.factor = factor
        self.patience = patience

    def on_train_begin(self, logs):
        self.scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(
            self.optimizer, mode='min', factor=self.factor, patience=self.patience, threshold=0.001,
            threshold_mode='rel', cooldown=0, min_lr=1e-6, eps=1e-08)

    def on_epoch_end(self, epoch, logs):
        self.scheduler.step(logs[self.metric])
