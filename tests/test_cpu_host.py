"""CPU-only checks: the C-ABI library loads and exports every declared symbol,
and the host-side logic (gin subset, gating state machine, grouping, CUR
averaging) matches the oracle.  No kernel is launched here."""
import ctypes
import os
import pickle
import random
import re

import numpy as np
import pytest
import torch

import spec
from oracle import cur_ref, gating_ref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "greedymml.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gm_[a-z0-9_]+)\s*\(", src)))


def test_library_builds_and_exports_every_declared_symbol():
    from greedy_multimodal_learning_amd import build, _lib
    build.build()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    syms = _declared_symbols()
    assert len(syms) >= 9
    for s in syms:
        assert hasattr(lib, s), s
    assert set(_lib.EXPORTS) == set(syms)
    L = _lib.load()
    assert L.gm_abi_version() == _lib.ABI_VERSION


def test_abi_argument_errors_without_gpu():
    """Argument validation runs before any launch, so it is testable on the CPU."""
    from greedy_multimodal_learning_amd import _lib as L
    lib = L.load()
    rc = lib.gm_gemm_f32(None, 0, None)
    assert rc == -1 and b"nprob" in lib.gm_last_error()
    rc = lib.gm_group_sumsq(None, 0, 0, 4, 1.0, 0.0, None, None, 0, None)
    assert rc == -1 and b"empty" in lib.gm_last_error()
    rc = lib.gm_mmtm_spatial_reduce(None, 1, 1, 0, 0, None, 0, None)
    assert rc == -1


def test_struct_layouts_match_header(tmp_path):
    """ctypes mirrors of every ABI struct have the C compiler's size and field offsets."""
    import shutil
    import subprocess
    from greedy_multimodal_learning_amd import _lib as L
    assert ctypes.sizeof(L.Tensor) == 40
    assert ctypes.sizeof(L.Operand) == 16
    assert ctypes.sizeof(L.SpatialReduce) == 56
    assert ctypes.sizeof(L.ChannelScale) == 56
    pairs = [("gm_tensor", L.Tensor), ("gm_operand", L.Operand), ("gm_spatial_reduce", L.SpatialReduce),
             ("gm_channel_scale", L.ChannelScale), ("gm_gemm", L.Gemm), ("gm_conv_desc", L.ConvDesc),
             ("gm_bn_fwd", L.BnFwd), ("gm_bn_bwd", L.BnBwd), ("gm_pool_desc", L.PoolDesc),
             ("gm_conv_f32", L.ConvF32), ("gm_conv_desc_hw", L.ConvDescHW), ("gm_stem_pack", L.StemPack),
             ("gm_stem_bn_src", L.StemBnSrc),
             ("gm_wprep", L.WPrep), ("gm_views_norm", L.ViewsNorm), ("gm_gate_state", L.GateState),
             ("gm_gate_state_n", L.GateStateN)]
    # every struct the header declares has a mirror in this list
    hdr = open(os.path.join(ROOT, "include", "greedymml.h")).read()
    declared = set(re.findall(r"typedef struct (gm_[a-z0-9_]+)", hdr))
    assert declared == {c for c, _ in pairs}, declared ^ {c for c, _ in pairs}
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "greedymml.h"', "int main(void){"]
    for cname, py in pairs:
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call([cc, "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = dict(line.split() for line in subprocess.check_output([str(exe)]).decode().splitlines())
    for cname, py in pairs:
        assert int(got[cname]) == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(py, f).offset, f"{cname}.{f}"


def test_product_ops_refuse_cpu_tensors():
    from greedy_multimodal_learning_amd import ops
    from greedy_multimodal_learning_amd._lib import GreedyMMLError
    with pytest.raises(GreedyMMLError):
        ops.linear(torch.randn(2, 3), torch.randn(4, 3))
    # the trunk modules have no CPU / vendor-library path either
    from greedy_multimodal_learning_amd.bn import GMBatchNorm2d
    from greedy_multimodal_learning_amd.conv import GMConv2d
    from greedy_multimodal_learning_amd.pool import GMMaxPool2d
    for mod, x in ((GMConv2d(8, 8, 3, padding=1, bias=False), torch.randn(1, 8, 5, 5)),
                   (GMBatchNorm2d(8), torch.randn(2, 8, 5, 5)),
                   (GMMaxPool2d(3, 2, 1), torch.randn(1, 8, 5, 5))):
        with pytest.raises(GreedyMMLError):
            mod(x)


@pytest.mark.parametrize("cfg", ["training_guided", "training_random", "training", "recording", "eval"])
def test_gin_lite_parses_reference_configs(cfg):
    from greedy_multimodal_learning_amd import gin_lite as g
    path = os.path.join(os.environ.get("GREEDYMML_REF", "/root/reference"), "configs", cfg + ".gin")
    if not os.path.exists(path):
        pytest.skip("reference configs not mounted")
    g.clear_config()
    g.parse_config_files_and_bindings([path], "train.lr=0.05#MMTM_MVCNN.num_views=2")
    assert g.query("MMTM_MVCNN", "pretraining") is False
    assert g.query("get_mvdcndata", "specific_views") == [0, 6]
    if cfg in ("training_guided", "training"):
        assert g.query("Bias_Mitigation_Strong", "epsilon") == 0.01
        assert g.query("Bias_Mitigation_Strong", "branchnames") == ["net_view_0", "net_view_1"]
        assert g.query("train", "lr") == 0.05
    g.clear_config()


def test_gin_lite_fills_configurable_defaults():
    from greedy_multimodal_learning_amd import gin_lite as g
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Strong
    g.clear_config()
    g.parse_config("Bias_Mitigation_Strong.epsilon=0.02\nBias_Mitigation_Strong.curation_windowsize=3\n"
                   "Bias_Mitigation_Strong.branchnames=['net_view_0', 'net_view_1']\n")
    cb = Bias_Mitigation_Strong()
    assert (cb.epsilon, cb.curation_windowsize, cb.starting_epoch) == (0.02, 3, 2)
    cb = Bias_Mitigation_Strong(epsilon=0.5)
    assert cb.epsilon == 0.5
    g.clear_config()


def test_group_masks_follow_reference_substring_rules():
    from greedy_multimodal_learning_amd.callbacks import group_masks
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN
    m = MMTM_MVCNN()
    names = [n for n, _ in m.named_parameters()]
    assert len(names) == 142
    assert sum(p.numel() for p in m.parameters()) == 23773008
    masks = group_masks(names, ["net_view_0", "net_view_1"], ["visual", "skeleton"])
    for n, mk in zip(names, masks):
        main, by = gating_ref.param_group(n)
        want = sum(1 << i for i, f in enumerate(main) if f) + sum(1 << (2 + j) for j, f in enumerate(by) if f)
        assert mk == want, n
    assert sum(1 for mk in masks if mk == 1) == 62 and sum(1 for mk in masks if mk == 2) == 62
    assert sum(1 for mk in masks if mk & 12) == 18


class _MP:
    curation_mode = False
    caring_modality = None


def test_gating_state_machine_matches_oracle():
    """Drive product and oracle state machines with identical random group sums."""
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Strong
    rng = np.random.default_rng(0)
    cb = Bias_Mitigation_Strong(epsilon=0.01, curation_windowsize=3,
                                branchnames=["net_view_0", "net_view_1"], starting_epoch=2)
    mp = _MP()
    cb.set_model_pytoune(mp)
    cb.on_train_begin({})
    ref = gating_ref.BDRState(0.01, 3, starting_epoch=2)
    for epoch in range(1, 5):
        cb.on_epoch_begin(epoch, {})
        ref.on_epoch_begin(epoch)
        for step in range(10):
            s = np.exp(rng.normal(size=8))
            cb.group_sums = lambda s=s: torch.from_numpy(s.copy())
            d = dict(wn_main=[s[0], s[2]], gn_main=[s[1], s[3]], wn_bypass=[s[4], s[6]],
                     gn_bypass=[s[5], s[7]])
            cb.on_backward_end(step)
            ref.on_backward_end(lambda d=d: d)
            assert (mp.curation_mode, mp.caring_modality) == (ref.curation_mode, ref.caring_modality)
            assert cb.d_BDR == pytest.approx(ref.d_BDR, abs=1e-12)
            logs = {}
            cb.on_batch_end(step, logs)
            assert logs["d_BDR"] == cb.d_BDR


def test_group_masks_many_branches_longest_match():
    from greedy_multimodal_learning_amd.callbacks import group_masks
    branches = [f"net_view_{i}" for i in range(12)]
    mods = [f"fc_excite.{i}." for i in range(12)]
    names = ["net_view_1.conv1.weight", "net_view_10.conv1.weight", "net_view_11.fc.bias",
             "mmtm2.fc_squeeze.weight", "mmtm3.fc_excite.1.weight", "mmtm4.fc_excite.11.bias"]
    m = group_masks(names, branches, mods)
    assert m[0] == 1 << 1 and m[1] == 1 << 10 and m[2] == 1 << 11
    assert m[3] == sum(1 << (12 + j) for j in range(12))
    assert m[4] == 1 << (12 + 1) and m[5] == 1 << (12 + 11)


def test_n_branch_decision_reduces_to_reference_at_two():
    """bdr_decision (N-branch rule) == the reference rule on two branches."""
    from greedy_multimodal_learning_amd.callbacks import bdr_decision
    rng = np.random.default_rng(3)
    for _ in range(200):
        b = rng.normal(size=2)
        spread, care = bdr_decision(b)
        d = b[0] - b[1]
        assert spread == pytest.approx(abs(d))
        assert care == (1 if d < 0 else 0)


def test_n_branch_gate_cares_for_argmax():
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Strong
    nb = 4
    cb = Bias_Mitigation_Strong(epsilon=0.01, curation_windowsize=2,
                                branchnames=[f"net_view_{i}" for i in range(nb)], starting_epoch=1,
                                MMTMnames=[f"fc_excite.{i}." for i in range(nb)])
    mp = _MP()
    cb.set_model_pytoune(mp)
    cb.on_train_begin({})
    cb.on_epoch_begin(1, {})
    s = np.ones(4 * nb)
    s[2 * (nb + 2) + 1] = 5.0  # bypass_2 gradient ratio 5x: BDR_2 is the largest
    cb.group_sums = lambda: torch.from_numpy(s.copy())
    cb.on_backward_end(0)
    assert mp.curation_mode and mp.caring_modality == 2
    assert cb.d_BDR == pytest.approx(np.log10(5.0))
    cb.on_backward_end(1)
    cb.on_backward_end(2)  # window 2 ends
    assert not mp.curation_mode


def test_random_gate_matches_oracle():
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Random
    cb = Bias_Mitigation_Random()
    mp = _MP()
    cb.set_model_pytoune(mp)
    cb.on_train_begin({})
    ref = gating_ref.RandomGate(rng=random.Random(5))
    random.seed(5)
    for epoch in range(1, 4):
        cb.on_epoch_begin(epoch, {})
        ref.on_epoch_begin(epoch)
        for _ in range(20):
            cb.on_backward_end(0)
            ref.on_backward_end()
            assert (mp.curation_mode, mp.caring_modality) == (ref.curation_mode, ref.caring_modality)


def test_cur_rescale_weights_match_oracle(tmp_path):
    from greedy_multimodal_learning_amd.cur import rescale_weights
    ev, tr = spec.cur_histories()
    for sub, h in (("eval", ev), ("train", tr)):
        os.makedirs(tmp_path / sub)
        with open(tmp_path / sub / "history.pickle", "wb") as f:
            pickle.dump(h, f)
    a = rescale_weights(str(tmp_path / "eval"), str(tmp_path / "train"))
    b = cur_ref.rescale_weights(str(tmp_path / "eval"), str(tmp_path / "train"))
    assert a[0] is None and b[0] is None
    for i in range(1, 4):
        for j in range(2):
            np.testing.assert_array_equal(a[i][j], b[i][j])


def test_losses_match_oracle():
    from greedy_multimodal_learning_amd.losses import acc, blend_loss
    g = torch.Generator().manual_seed(0)
    outs = [torch.randn(6, 40, generator=g) for _ in range(2)]
    y = torch.randint(0, 40, (6,), generator=g)
    assert float(blend_loss(outs, y)) == pytest.approx(float(gating_ref.blend_loss(outs, y)), rel=1e-6)
    assert float(acc(outs, y)) == float(gating_ref.acc(outs, y))
    assert float(acc(outs[0], y[:2])) == float(gating_ref.acc(outs[0], y[:2]))


def test_grad_join_order_and_masked_pending():
    """gradsink.GradJoin (the block-input gradient join): every consumer but the last leaves its
    gradient pending and gets None; the last one's compute receives it; first_of_many() says when
    a consumer's contribution will be left pending (the block-output BN then hands a MaskedAddend
    instead of writing dres); the join resets for the next backward."""
    import torch
    from greedy_multimodal_learning_amd.gradsink import GradJoin, MaskedAddend
    jn = GradJoin()
    assert not jn.masked_ok
    jn.register()
    jn.register()
    for _ in range(2):  # two backward passes through the same join
        assert jn.first_of_many()
        dy, mask = torch.ones(2, 8), torch.full((2,), 0xA5, dtype=torch.uint8)
        assert jn.contribute(lambda add: MaskedAddend(dy, mask) if add is None else None) is None
        assert not jn.first_of_many()
        seen = []
        out = jn.contribute(lambda add: seen.append(add) or "dx")
        assert out == "dx" and isinstance(seen[0], MaskedAddend) and seen[0].dy is dy and seen[0].mask is mask
        assert jn.pending is None and jn.done == 0
    single = GradJoin()
    single.register()
    assert not single.first_of_many()  # a lone consumer is always the last
    assert single.contribute(lambda add: add) is None
