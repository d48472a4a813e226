"""MMTM_MVCNN on MI355X: drop-in for the reference's `src.model`.

Same constructor signature, gin name, parameter names and forward contract as
reference src/model.py:15-108: two unshared ResNet-18 trunks `net_view_0/1`
(fc -> Linear(512, nclasses)) and MMTM fusion after layer2/3/4
(`mmtm2/3/4`, C = 128/256/512, ratio 4).  forward(x[B,V,3,H,W],
curation_mode, caring_modality) returns ((x0+x1)/2, [x0, x1], scales[3],
squeezed[3]).  The MMTM sites run on libgreedymml_hip.so; `Model_`
(src/framework.py:158-161) reads `saving_mmtm_scales` /
`saving_mmtm_squeeze_array` from this object.
"""
import torch
import torch.nn as nn

from .balanced_mmtm import MMTM_mitigate as MMTM
from .balanced_mmtm import get_rescale_weights
from .gin_lite import configurable
from . import vtrunk
from .head import head_ok, pooled_linear, pooled_linear_stacked
from .resnet import resnet18
from .streams import ViewStreams

CLASSNAMES = ['airplane', 'bathtub', 'bed', 'bench', 'bookshelf', 'bottle', 'bowl', 'car', 'chair',
              'cone', 'cup', 'curtain', 'desk', 'door', 'dresser', 'flower_pot', 'glass_box',
              'guitar', 'keyboard', 'lamp', 'laptop', 'mantel', 'monitor', 'night_stand',
              'person', 'piano', 'plant', 'radio', 'range_hood', 'sink', 'sofa', 'stairs',
              'stool', 'table', 'tent', 'toilet', 'tv_stand', 'vase', 'wardrobe', 'xbox']


def grad_order(model):
    """The model's parameters in the order the view-batched backward produces their gradients:
    the heads (`net_view_*.fc`), the MMTM site after layer 4, layer 4 of every view, the site
    after layer 3, layer 3, ..., layer 1, the stems.  Inside a stage: reversed registration order
    of the per-view name, views interleaved (the grouped launches write every view's gradient of
    a layer together).  The engine lays its flat gradient buffer out in this order, so each
    data-parallel all-reduce bucket (a contiguous slice) completes as early as backward allows -
    with the reverse registration order, net_view_1's whole trunk sat between net_view_0's layer-4
    and stem gradients, and half of C2's 95 MB could only be reduced after the stem."""
    named = list(model.named_parameters())

    def split(n):
        head, _, rest = n.partition(".")
        if head.startswith("net_view_") and head[9:].isdigit():
            return int(head[9:]), rest
        return -1, n

    def stage(n):
        v, rest = split(n)
        if v >= 0:
            sub = rest.split(".")[0]
            if sub == "fc":
                return 100
            if sub.startswith("layer") and sub[5:].isdigit():
                return 10 * int(sub[5:])
            return 0  # stem: conv1, bn1
        head = n.split(".")[0]
        if head.startswith("mmtm") and head[4:].isdigit():
            return 10 * int(head[4:]) + 5
        return 100
    first = {}  # per-view name -> its registration index within the view (or the global index)
    for i, (n, _) in enumerate(named):
        first.setdefault(split(n)[1], i)
    keyed = sorted(named, key=lambda np_: (-stage(np_[0]), -first[split(np_[0])[1]], split(np_[0])[0]))
    return [p for _, p in keyed]


@configurable
class MMTM_MVCNN(nn.Module):
    def __init__(self, nclasses=40, num_views=2, pretraining=False, mmtm_off=False,
                 mmtm_rescale_eval_file_path=None, mmtm_rescale_training_file_path=None,
                 device='cuda:0', saving_mmtm_scales=False, saving_mmtm_squeeze_array=False):
        super().__init__()
        self.classnames = list(CLASSNAMES)
        self.nclasses = nclasses
        self.num_views = num_views
        self.mmtm_off = mmtm_off
        if mmtm_off:
            self.mmtm_rescale = get_rescale_weights(
                mmtm_rescale_eval_file_path, mmtm_rescale_training_file_path, validation=False,
                starting_mmtmindice=1, mmtmpositions=4, device=torch.device(device))
        self.saving_mmtm_scales = saving_mmtm_scales
        self.saving_mmtm_squeeze_array = saving_mmtm_squeeze_array
        self.net_view_0 = resnet18(pretrained=pretraining)
        self.net_view_0.fc = nn.Linear(512, nclasses)
        self.net_view_1 = resnet18(pretrained=pretraining)
        self.net_view_1.fc = nn.Linear(512, nclasses)
        mdev = device if torch.cuda.is_available() else "cpu"
        self.mmtm2 = MMTM(128, 128, 4, device=mdev)
        self.mmtm3 = MMTM(256, 256, 4, device=mdev)
        self.mmtm4 = MMTM(512, 512, 4, device=mdev)

    @staticmethod
    def _stem(net, x):
        y = net.conv1(x)
        if hasattr(net.bn1, "relu_maxpool"):  # bn1 + relu + maxpool fused (bn.py)
            return net.layer1(net.bn1.relu_maxpool(y, net.maxpool))
        return net.layer1(net.maxpool(net.relu(net.bn1(y))))

    @staticmethod
    def _head(net, f):
        return net.fc(torch.flatten(net.avgpool(f), 1))

    @staticmethod
    def _fused_head(nets, fs):
        """All branches' avgpool + fc in one launch each way (head.py), or None."""
        fcs = [n.fc for n in nets]
        if not (all(isinstance(n.avgpool, nn.AdaptiveAvgPool2d) and n.avgpool.output_size in ((1, 1), 1)
                    and isinstance(n.fc, nn.Linear) for n in nets) and head_ok(fs, fcs)):
            return None
        return pooled_linear(fs, fcs)

    def _forward_stacked(self, x, curation_mode, caring_modality):
        """The two trunks as ONE view-batched trunk (vtrunk.py): every convolution /
        BatchNorm position is one grouped launch over [x0; x1], the MMTM sites and the
        heads read and write the stacked activation."""
        nets = [self.net_view_0, self.net_view_1]
        X = vtrunk.vstem(x, nets)
        X = vtrunk.vlayer(nets, 1, X)
        scales, squeezed = [], []
        for i in (2, 3, 4):
            X = vtrunk.vlayer(nets, i, X)
            X, sc, sq = getattr(self, f"mmtm{i}").forward_stacked(
                X, self.saving_mmtm_scales, self.saving_mmtm_squeeze_array,
                turnoff_cross_modal_flow=bool(self.mmtm_off),
                average_squeezemaps=self.mmtm_rescale[i - 1] if self.mmtm_off else None,
                curation_mode=curation_mode, caring_modality=caring_modality)
            scales.append(sc)
            squeezed.append(sq)
        B = X.shape[0] // 2
        if head_ok([X[:B], X[B:]], [n.fc for n in nets]) and all(
                isinstance(n.avgpool, nn.AdaptiveAvgPool2d) and n.avgpool.output_size in ((1, 1), 1) for n in nets):
            x0, x1 = pooled_linear_stacked(X, [n.fc for n in nets])
        else:
            x0, x1 = self._head(nets[0], X[:B]), self._head(nets[1], X[B:])
        mean = None if getattr(self, "_no_mean", False) else (x0 + x1) / 2
        return mean, [x0, x1], scales, squeezed

    def grad_order(self):
        """Parameters in backward-production order (module function grad_order)."""
        return grad_order(self)

    def forward(self, x, curation_mode=False, caring_modality=None):
        if vtrunk.usable(self, [self.net_view_0, self.net_view_1], x):
            return self._forward_stacked(x, curation_mode, caring_modality)
        # view 1's trunk segments run on a side HIP stream (streams.py): the two
        # trunks only meet at the MMTM sites, which run on the main stream
        vs = ViewStreams.for_tensor(x, 2)
        run = vs.run if vs is not None else (lambda i, fn, *a: fn(*a))
        if vs is not None:
            vs.fork()
        f1 = run(1, self._stem, self.net_view_1, x[:, 1])
        f0 = self._stem(self.net_view_0, x[:, 0])
        scales, squeezed = [], []
        for i in (2, 3, 4):
            f1 = run(1, getattr(self.net_view_1, f"layer{i}"), f1)
            f0 = getattr(self.net_view_0, f"layer{i}")(f0)
            if vs is not None:
                vs.join([f1])
            f0, f1, sc, sq = getattr(self, f"mmtm{i}")(
                f0, f1, self.saving_mmtm_scales, self.saving_mmtm_squeeze_array,
                turnoff_cross_modal_flow=bool(self.mmtm_off),
                average_squeezemaps=self.mmtm_rescale[i - 1] if self.mmtm_off else None,
                curation_mode=curation_mode, caring_modality=caring_modality)
            if vs is not None:
                vs.fork([(1, f1)])
            scales.append(sc)
            squeezed.append(sq)
        fused = self._fused_head([self.net_view_0, self.net_view_1], [f0, f1])
        if fused is not None:  # both heads on the main stream (f1 was joined at mmtm4)
            x0, x1 = fused
        else:
            x1 = run(1, self._head, self.net_view_1, f1)
            x0 = self._head(self.net_view_0, f0)
            if vs is not None:
                vs.join([x1])
        # (the engine's step reads only the branch logits: no averaging launches there)
        mean = None if getattr(self, "_no_mean", False) else (x0 + x1) / 2
        return mean, [x0, x1], scales, squeezed


@configurable
class MMTM_MVCNN_N(nn.Module):
    """N-branch generalisation: `num_views` unshared trunks
    `net_view_{i}` (resnet18 for C4, resnet50 for C5) fused by `MMTM_N` after
    layer2/3/4.  forward(x[B,V,3,H,W]) returns (mean of the branch logits,
    [logits_i], scales[3], squeezed[3]) like MMTM_MVCNN; caring_modality may
    be any branch index.  At num_views=2 / resnet18 it computes what
    MMTM_MVCNN computes (parameter names differ only inside the MMTM sites:
    fc_excite.{0,1} for fc_visual/fc_skeleton)."""

    def __init__(self, nclasses=40, num_views=4, trunk="resnet18", ratio=4, ra_source="first",
                 saving_mmtm_scales=False, saving_mmtm_squeeze_array=False):
        super().__init__()
        from .mmtm_n import MMTM_N
        from .resnet import resnet50
        make = {"resnet18": resnet18, "resnet50": resnet50}[trunk]
        self.nclasses = nclasses
        self.num_views = num_views
        self.saving_mmtm_scales = saving_mmtm_scales
        self.saving_mmtm_squeeze_array = saving_mmtm_squeeze_array
        exp = 1 if trunk == "resnet18" else 4
        for i in range(num_views):
            net = make(pretrained=False)
            net.fc = nn.Linear(512 * exp, nclasses)
            setattr(self, f"net_view_{i}", net)
        for i, c in ((2, 128), (3, 256), (4, 512)):
            setattr(self, f"mmtm{i}", MMTM_N([c * exp] * num_views, ratio, ra_source=ra_source))

    def branch_names(self):
        return [f"net_view_{i}" for i in range(self.num_views)]

    def mmtm_names(self):
        return [f"fc_excite.{i}." for i in range(self.num_views)]

    def _forward_stacked(self, nets, x, curation_mode, caring_modality):
        """All views' trunks as ONE view-batched trunk (vtrunk.py: every convolution /
        BatchNorm position one grouped launch over the V views stacked along the batch),
        the MMTM sites and the heads on the stacked activation (MMTM_N.forward_stacked,
        head.pooled_linear_stacked)."""
        X = vtrunk.vstem(x, nets)
        X = vtrunk.vlayer(nets, 1, X)
        scales, squeezed = [], []
        for li in (2, 3, 4):
            X = vtrunk.vlayer(nets, li, X)
            X, sc, sq = getattr(self, f"mmtm{li}").forward_stacked(
                X, self.saving_mmtm_scales, self.saving_mmtm_squeeze_array, curation_mode=curation_mode,
                caring_modality=caring_modality if caring_modality is not None else 0)
            scales.append(sc)
            squeezed.append(sq)
        B = X.shape[0] // self.num_views
        fcs = [n.fc for n in nets]
        if head_ok([X[i * B:(i + 1) * B] for i in range(self.num_views)], fcs) and all(
                isinstance(n.avgpool, nn.AdaptiveAvgPool2d) and n.avgpool.output_size in ((1, 1), 1) for n in nets):
            outs = pooled_linear_stacked(X, fcs)
        else:
            outs = [MMTM_MVCNN._head(n, X[i * B:(i + 1) * B]) for i, n in enumerate(nets)]
        mean = None if getattr(self, "_no_mean", False) else sum(outs) / len(outs)
        return mean, outs, scales, squeezed

    def grad_order(self):
        """Parameters in backward-production order (module function grad_order)."""
        return grad_order(self)

    def forward(self, x, curation_mode=False, caring_modality=None):
        nets = [getattr(self, f"net_view_{i}") for i in range(self.num_views)]
        if vtrunk.usable(self, nets, x):
            return self._forward_stacked(nets, x, curation_mode, caring_modality)
        vs = ViewStreams.for_tensor(x, self.num_views)
        run = vs.run if vs is not None else (lambda i, fn, *a: fn(*a))
        order = list(range(self.num_views))[::-1]  # side streams first, main last
        if vs is not None:
            vs.fork()
        fs = [None] * self.num_views
        for i in order:
            fs[i] = run(i, MMTM_MVCNN._stem, nets[i], x[:, i])
        scales, squeezed = [], []
        for li in (2, 3, 4):
            for i in order:
                fs[i] = run(i, getattr(nets[i], f"layer{li}"), fs[i])
            if vs is not None:
                vs.join(fs[1:])
            fs, sc, sq = getattr(self, f"mmtm{li}")(
                fs, self.saving_mmtm_scales, self.saving_mmtm_squeeze_array, curation_mode=curation_mode,
                caring_modality=caring_modality if caring_modality is not None else 0)
            if vs is not None:
                vs.fork(list(enumerate(fs)))
            scales.append(sc)
            squeezed.append(sq)
        outs = MMTM_MVCNN._fused_head(nets, fs)
        if outs is None:
            outs = [None] * self.num_views
            for i in order:
                outs[i] = run(i, MMTM_MVCNN._head, nets[i], fs[i])
            if vs is not None:
                vs.join(outs[1:])
        mean = None if getattr(self, "_no_mean", False) else sum(outs) / len(outs)
        return mean, outs, scales, squeezed
