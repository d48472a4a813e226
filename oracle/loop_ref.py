"""Epoch loop in the reference's order (oracle side), for whole-run traces.

Mirrors the sequence of `Model_.train_loop` (`src/framework.py:270-345`) that
matters for the hot path: `on_epoch_begin` (gating unlock,
`src/callbacks.py:265-267`), the train steps, then the validation and test
passes under no_grad in eval mode (`:330-332`), which also advance the MMTM
running averages.  Per step it records what `on_batch_end` logs:
(loss, d_BDR, curation_mode, caring_modality, acc, acc_modal_0, acc_modal_1).
"""
import torch

from .gating_ref import acc


def run(model, step, gate, train, valid, test, epochs, to=lambda t: t):
    rows = []
    for epoch in range(1, epochs + 1):
        gate.on_epoch_begin(epoch)
        for _, x, y in train:
            x, y = to(x), to(y)
            loss = step(x, y)
            rows.append((loss, gate.d_BDR, float(gate.curation_mode),
                         -1 if gate.caring_modality is None else gate.caring_modality,
                         *step.last_metrics))
        model.eval()
        with torch.no_grad():
            for L in (valid, test):
                for _, x, y in L:
                    model(to(x), curation_mode=gate.curation_mode,
                          caring_modality=gate.caring_modality)
        model.train(True)
    return rows


def metrics(out_mean, outs, y):
    with torch.no_grad():
        return (float(acc(out_mean, y)), float(acc(outs[0], y)), float(acc(outs[1], y)))
