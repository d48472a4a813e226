"""One balanced training step on the CPU, in the reference's order (oracle side).

`src/framework.py:307-322`: zero_grad -> forward(curation flags held by the
step engine, `:137-138,146-148`) -> blend_loss (`train.py:23-29`) -> backward ->
on_backward_end (gating, `src/callbacks.py:240-263`) -> SGD.step
(`train.py:48-51`) -> loss.item().  This is also the `cpu_baseline` leg of
bench.py (kind "port").
"""
import torch

from .gating_ref import blend_loss, group_sums
from .loop_ref import metrics


class RefStep:
    def __init__(self, model, lr=0.1, gate=None, branchnames=("net_view_0", "net_view_1")):
        self.model = model
        self.opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=0, weight_decay=0)
        self.gate = gate
        self.branchnames = branchnames

    def sums(self):
        named = [(n, p, p.grad) for n, p in self.model.named_parameters()]
        return group_sums(named, self.branchnames)

    def __call__(self, x, y):
        self.model.train(True)
        self.opt.zero_grad()
        cm = self.gate.curation_mode if self.gate is not None else False
        cmod = self.gate.caring_modality if self.gate is not None else None
        mean, logits, _, _ = self.model(x, curation_mode=cm, caring_modality=cmod)
        loss = blend_loss(logits, y)
        self.last_metrics = metrics(mean, logits, y)
        loss.backward()
        if self.gate is not None:
            self.gate.on_backward_end(self.sums)
        self.opt.step()
        return float(loss.item())
