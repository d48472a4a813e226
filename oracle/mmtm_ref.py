"""MMTM squeeze-excite fusion, CPU fp32 restatement (oracle side).

Follows `src/balanced_mmtm.py` of the reference:

* ctor  `:17-47`  dim = dv+ds, dim_out = int(2*dim/ratio); fc_squeeze (or the
  SE-only pair fc_squeeze_{visual,skeleton}); fc_visual/fc_skeleton (or the
  shared fc_excite); running averages sized by dim_visual for BOTH modalities
  (`:30-31`) and a python step counter (`:32`).
* normal mode `:93-111`: sq_m = mean_hw(X_m); z = relu(W_sq [sq_v;sq_s] + b);
  e_m = sigmoid(W_m z + b_m).
* turn-off mode `:72-91`: each modality's squeeze is its own GAP concatenated
  with the OTHER modality's dataset-average squeeze, through fc_squeeze+relu and
  its own excite FC.
* SE-only `:60-69`: no cross-modal flow at all.
* running averages `:113-116`: BOTH use the visual scale (reference quirk).
* curation `:135-152`: the caring modality's scale is replaced by its running
  average (post-update, detached).
* return `:154`: (X_v * e_v, X_s * e_s, scales|None, squeeze_array|None).
"""
import torch
import torch.nn as nn


class MMTMRef(nn.Module):
    def __init__(self, dim_visual, dim_skeleton, ratio, SEonly=False, shareweight=False):
        super().__init__()
        dim = dim_visual + dim_skeleton
        dim_out = int(2 * dim / ratio)
        self.SEonly = SEonly
        self.shareweight = shareweight
        self.running_avg_weight_visual = torch.zeros(dim_visual)
        self.running_avg_weight_skeleton = torch.zeros(dim_visual)
        self.step = 0
        if SEonly:
            self.fc_squeeze_visual = nn.Linear(dim_visual, dim_out)
            self.fc_squeeze_skeleton = nn.Linear(dim_skeleton, dim_out)
        else:
            self.fc_squeeze = nn.Linear(dim, dim_out)
        if shareweight:
            assert dim_visual == dim_skeleton
            self.fc_excite = nn.Linear(dim_out, dim_visual)
        else:
            self.fc_visual = nn.Linear(dim_out, dim_visual)
            self.fc_skeleton = nn.Linear(dim_out, dim_skeleton)

    @staticmethod
    def _gap(x):
        return x.reshape(x.shape[0], x.shape[1], -1).mean(-1)

    def _exc(self, which):
        if self.shareweight:
            return self.fc_excite
        return self.fc_visual if which == 0 else self.fc_skeleton

    def forward(self, visual, skeleton, return_scale=False, return_squeezed_mps=False,
                turnoff_cross_modal_flow=False, average_squeezemaps=None,
                curation_mode=False, caring_modality=0):
        squeeze_array = None
        if self.SEonly:
            a_v = self.fc_visual(torch.relu(self.fc_squeeze_visual(self._gap(visual))))
            a_s = self.fc_skeleton(torch.relu(self.fc_squeeze_skeleton(self._gap(skeleton))))
        elif turnoff_cross_modal_flow:
            B = visual.shape[0]
            avg_v, avg_s = average_squeezemaps[0], average_squeezemaps[1]
            in_v = torch.cat([self._gap(visual), avg_s.reshape(1, -1).expand(B, -1)], 1)
            in_s = torch.cat([avg_v.reshape(1, -1).expand(skeleton.shape[0], -1),
                              self._gap(skeleton)], 1)
            a_v = self._exc(0)(torch.relu(self.fc_squeeze(in_v)))
            a_s = self._exc(1)(torch.relu(self.fc_squeeze(in_s)))
        else:
            squeeze_array = [self._gap(visual), self._gap(skeleton)]
            z = torch.relu(self.fc_squeeze(torch.cat(squeeze_array, 1)))
            a_v = self._exc(0)(z)
            a_s = self._exc(1)(z)
        e_v = torch.sigmoid(a_v)
        e_s = torch.sigmoid(a_s)

        m = e_v.mean(0).detach()
        k = self.step
        self.running_avg_weight_visual = (m + self.running_avg_weight_visual * k) / (k + 1)
        self.running_avg_weight_skeleton = (m + self.running_avg_weight_skeleton * k) / (k + 1)
        self.step += 1

        scales = [e_v.detach().clone(), e_s.detach().clone()] if return_scale else None
        if return_squeezed_mps:
            if squeeze_array is None:  # reference raises here (`:123-124`)
                raise UnboundLocalError("squeeze_array referenced before assignment")
            squeeze_array = [t.detach().clone() for t in squeeze_array]
        else:
            squeeze_array = None

        if curation_mode and caring_modality == 0:
            e_v = self.running_avg_weight_visual.reshape(1, -1).expand(e_v.shape[0], -1)
        elif curation_mode and caring_modality == 1:
            e_s = self.running_avg_weight_skeleton.reshape(1, -1).expand(e_s.shape[0], -1)
        ev = e_v.reshape(e_v.shape + (1,) * (visual.dim() - 2))
        es = e_s.reshape(e_s.shape + (1,) * (skeleton.dim() - 2))
        return visual * ev, skeleton * es, scales, squeeze_array
