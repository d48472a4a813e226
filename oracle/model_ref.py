"""MMTM_MVCNN, CPU fp32 restatement (oracle side).

Follows `src/model.py:15-108`: two unshared torchvision ResNet-18 trunks
`net_view_{0,1}` with `fc = Linear(512, nclasses)` (`:53-56`) and MMTM fusion
after layer2/3/4 (`mmtm2/3/4`, C = 128/256/512, ratio 4; `:58-60`).  forward
(`:63-108`) returns ((x0+x1)/2, [x0, x1], scales[3], squeezed[3]).

`MMTM_MVCNN_N_Ref(num_views, trunk="resnet18"|"resnet50")` generalises to configs
C4/C5 (N trunks, the N-way MMTM of `oracle.mmtm_nway_ref`; same parameter names as
the build's `MMTM_MVCNN_N`); the reference itself is 2-way ResNet-18 only.
"""
import torch
import torch.nn as nn

from .resnet_ref import resnet18, resnet50
from .mmtm_ref import MMTMRef
from .mmtm_nway_ref import MMTMNRef


class MMTM_MVCNN_Ref(nn.Module):
    def __init__(self, nclasses=40, num_views=2, mmtm_off=False, mmtm_rescale=None,
                 saving_mmtm_scales=False, saving_mmtm_squeeze_array=False):
        super().__init__()
        self.nclasses = nclasses
        self.num_views = num_views
        self.mmtm_off = mmtm_off
        self.mmtm_rescale = mmtm_rescale
        self.saving_mmtm_scales = saving_mmtm_scales
        self.saving_mmtm_squeeze_array = saving_mmtm_squeeze_array
        self.net_view_0 = resnet18()
        self.net_view_0.fc = nn.Linear(512, nclasses)
        self.net_view_1 = resnet18()
        self.net_view_1.fc = nn.Linear(512, nclasses)
        self.mmtm2 = MMTMRef(128, 128, 4)
        self.mmtm3 = MMTMRef(256, 256, 4)
        self.mmtm4 = MMTMRef(512, 512, 4)

    @staticmethod
    def _stem(net, x):
        return net.layer1(net.maxpool(net.relu(net.bn1(net.conv1(x)))))

    def forward(self, x, curation_mode=False, caring_modality=None):
        f0 = self._stem(self.net_view_0, x[:, 0])
        f1 = self._stem(self.net_view_1, x[:, 1])
        scales, squeezed = [], []
        for i in (2, 3, 4):
            f0 = getattr(self.net_view_0, f"layer{i}")(f0)
            f1 = getattr(self.net_view_1, f"layer{i}")(f1)
            f0, f1, sc, sq = getattr(self, f"mmtm{i}")(
                f0, f1, self.saving_mmtm_scales, self.saving_mmtm_squeeze_array,
                turnoff_cross_modal_flow=bool(self.mmtm_off),
                average_squeezemaps=self.mmtm_rescale[i - 1] if self.mmtm_off else None,
                curation_mode=curation_mode, caring_modality=caring_modality)
            scales.append(sc)
            squeezed.append(sq)
        x0 = self.net_view_0.fc(torch.flatten(self.net_view_0.avgpool(f0), 1))
        x1 = self.net_view_1.fc(torch.flatten(self.net_view_1.avgpool(f1), 1))
        return (x0 + x1) / 2, [x0, x1], scales, squeezed


class MMTM_MVCNN_N_Ref(nn.Module):
    """N unshared trunks `net_view_{i}` (resnet18 / resnet50, fc -> Linear(512*exp,
    nclasses)) fused by MMTMNRef after layer2/3/4 (C = 128/256/512 x expansion)."""

    def __init__(self, nclasses=40, num_views=4, trunk="resnet18", ratio=4, ra_source="first"):
        super().__init__()
        make = {"resnet18": resnet18, "resnet50": resnet50}[trunk]
        exp = 1 if trunk == "resnet18" else 4
        self.num_views = num_views
        for i in range(num_views):
            net = make()
            net.fc = nn.Linear(512 * exp, nclasses)
            setattr(self, f"net_view_{i}", net)
        for i, c in ((2, 128), (3, 256), (4, 512)):
            setattr(self, f"mmtm{i}", MMTMNRef([c * exp] * num_views, ratio, ra_source=ra_source))

    def forward(self, x, curation_mode=False, caring_modality=None):
        nets = [getattr(self, f"net_view_{i}") for i in range(self.num_views)]
        fs = [MMTM_MVCNN_Ref._stem(n, x[:, i]) for i, n in enumerate(nets)]
        scales, squeezed = [], []
        for li in (2, 3, 4):
            fs = [getattr(n, f"layer{li}")(f) for n, f in zip(nets, fs)]
            fs, sc, sq = getattr(self, f"mmtm{li}")(fs, curation_mode=curation_mode,
                                                    caring_modality=caring_modality or 0)
            scales.append(sc)
            squeezed.append(sq)
        outs = [n.fc(torch.flatten(n.avgpool(f), 1)) for n, f in zip(nets, fs)]
        return sum(outs) / len(outs), outs, scales, squeezed
