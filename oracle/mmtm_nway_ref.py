"""N-modality MMTM, CPU restatement (oracle side; TEST INFRASTRUCTURE ONLY).

The reference's MMTM (`src/balanced_mmtm.py:15-154`) is two-way; configs C4 (4
modalities) and C5 (12 views) need N-way fusion.  This restates, in plain torch,
the generalisation the build documents in `greedy_multimodal_learning_amd/mmtm_n.py`:

* squeeze: sq = [GAP(X_0) | ... | GAP(X_{N-1})]           (`:95-97` per modality, `:99` concat)
* joint FC: z = relu(fc_squeeze(sq)), dim_out = int(4*sum(C) / (N*ratio))
  (the reference's int(2*(Cv+Cs)/ratio), `:25-26`, at N = 2)
* excitation: e_i = sigmoid(fc_excite[i](z))               (`:107-111`)
* running averages (`:113-116`), detached, every forward: ra_source "first" updates
  every average from modality 0's batch-mean scale (the reference's e_v quirk at
  N = 2), "own" from each modality's own scale; then step += 1
* curation (`:135-152`): e_caring <- ra_caring broadcast over the batch (detached)
* turn-off (`:72-91`): modality i's joint-FC input is its own squeeze in its own
  segment, the dataset-average squeezes elsewhere
* Y_i = X_i * e_i                                           (`:154`)

At N = 2 this is `oracle.mmtm_ref.MMTMRef` (fc_excite.{0,1} = fc_visual/fc_skeleton),
which the golden fixtures pin to the reference; for N > 2 there is no reference
(parity unpinned w.r.t. the reference - the check is HIP vs this restatement).
"""
import torch
import torch.nn as nn


def dim_out_rule(dims, ratio):
    return int(4 * sum(dims) / (len(dims) * ratio))


class MMTMNRef(nn.Module):
    def __init__(self, dims, ratio, ra_source="first"):
        super().__init__()
        self.dims = list(dims)
        self.N = len(self.dims)
        self.ra_source = ra_source
        dim_out = dim_out_rule(self.dims, ratio)
        self.fc_squeeze = nn.Linear(sum(self.dims), dim_out)
        self.fc_excite = nn.ModuleList([nn.Linear(dim_out, d) for d in self.dims])
        self.running_avg = [torch.zeros(d) for d in self.dims]
        self.step = 0

    def forward(self, xs, return_scale=False, return_squeezed_mps=False, turnoff_cross_modal_flow=False,
                average_squeezemaps=None, curation_mode=False, caring_modality=0):
        B = xs[0].shape[0]
        sqs = [x.reshape(B, x.shape[1], -1).mean(-1) for x in xs]
        if not turnoff_cross_modal_flow:
            z = torch.relu(self.fc_squeeze(torch.cat(sqs, 1)))
            es = [torch.sigmoid(fc(z)) for fc in self.fc_excite]
        else:
            if return_squeezed_mps:  # the reference's UnboundLocalError (:123-124)
                raise UnboundLocalError("local variable 'squeeze_array' referenced before assignment")
            avg = [torch.as_tensor(a).to(xs[0].dtype).reshape(1, -1).expand(B, -1) for a in average_squeezemaps]
            es = []
            for i in range(self.N):
                inp = torch.cat([sqs[j] if j == i else avg[j] for j in range(self.N)], 1)
                es.append(torch.sigmoid(self.fc_excite[i](torch.relu(self.fc_squeeze(inp)))))
        with torch.no_grad():
            self.running_avg = [r.to(xs[0].dtype) for r in self.running_avg]
            for i in range(self.N):
                src = es[0] if self.ra_source == "first" else es[i]
                self.running_avg[i] = (src.mean(0) + self.running_avg[i] * self.step) / (self.step + 1)
        self.step += 1
        if curation_mode:
            c = int(caring_modality)
            es[c] = self.running_avg[c].detach().reshape(1, -1).expand(B, -1)
        ys = [x * e.reshape(B, -1, 1, 1) for x, e in zip(xs, es)]
        scales = [e.detach().cpu() for e in es] if return_scale else None
        squeeze = [s.detach().cpu() for s in sqs] if return_squeezed_mps else None
        return ys, scales, squeeze
