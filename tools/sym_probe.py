#!/usr/bin/env python3
"""Probe of the per-view gradient asymmetry.

mirror: a mirror-symmetric MMTM_MVCNN (net_view_1 := net_view_0, fc_skeleton := fc_visual,
        the skeleton half of every fc_squeeze := its visual half) fed the SAME image in both
        views computes the same function for both branches, so every view-0 gradient must
        equal its view-1 twin.  Run through the benchmarked bf16 BalancedStep (graphs, device
        gate) and report per-tensor max |g0 - g1| / max |g0|.
swap:   the C2 bf16 step vs the fp32 oracle, once as is and once with the two views swapped
        (inputs, trunk weights, fc_visual <-> fc_skeleton, fc_squeeze column halves): if the
        large main-gradient error follows the weights it is data-dependent, if it stays at
        index 0 it is a bug in the view-0 path.

usage: python tools/sym_probe.py mirror|swap [--batch B] [--size H]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def mirror_state(sd):
    out = dict(sd)
    for k, v in sd.items():
        if k.startswith("net_view_1."):
            out[k] = sd["net_view_0." + k[len("net_view_1."):]].clone()
        if ".fc_skeleton." in k:
            out[k] = sd[k.replace(".fc_skeleton.", ".fc_visual.")].clone()
        if k.endswith("fc_squeeze.weight"):
            w = v.clone()
            C = w.shape[1] // 2
            w[:, C:] = w[:, :C]
            out[k] = w
    return out


def swap_state(sd):
    out = dict(sd)
    for k, v in sd.items():
        if k.startswith("net_view_0."):
            out[k] = sd["net_view_1." + k[len("net_view_0."):]].clone()
        elif k.startswith("net_view_1."):
            out[k] = sd["net_view_0." + k[len("net_view_1."):]].clone()
        elif ".fc_skeleton." in k:
            out[k] = sd[k.replace(".fc_skeleton.", ".fc_visual.")].clone()
        elif ".fc_visual." in k:
            out[k] = sd[k.replace(".fc_visual.", ".fc_skeleton.")].clone()
        elif k.endswith("fc_squeeze.weight"):
            C = v.shape[1] // 2
            out[k] = torch.cat([v[:, C:], v[:, :C]], 1).clone()
    return out


def hip_step(sd, buf, y, dev, dtype=torch.bfloat16, steps=2):
    from greedy_multimodal_learning_amd.callbacks import Bias_Mitigation_Strong
    from greedy_multimodal_learning_amd.engine import BalancedStep
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN
    model = MMTM_MVCNN()
    model.load_state_dict(sd, strict=False)
    model = model.to(dev)
    gate = Bias_Mitigation_Strong(epsilon=0.01, curation_windowsize=5, branchnames=["net_view_0", "net_view_1"],
                                  starting_epoch=2)
    step = BalancedStep(model, lr=0.0, gate=gate, graphs=True, compute_dtype=dtype)
    step.on_epoch_begin(1)
    x = buf.to(dev).to(dtype).permute(1, 0, 4, 2, 3)
    for _ in range(steps):
        step(x, y.to(dev))
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().float().cpu().clone() for n, p in model.named_parameters()}
    sums = step.norms.sums(grad_scale=1.0, lr=0.0).cpu().numpy()
    return grads, sums


def oracle(sd, buf, y):
    from oracle import gating_ref, model_ref
    o = model_ref.MMTM_MVCNN_Ref()
    o.load_state_dict(sd, strict=False)
    xo = buf.float().permute(1, 0, 4, 2, 3).contiguous()
    _, oo, _, _ = o(xo)
    loss = gating_ref.blend_loss(oo, y)
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in o.named_parameters()}
    s = gating_ref.group_sums([(n, p, p.grad) for n, p in o.named_parameters()])
    flat = [v for i in range(2) for v in (s["wn_main"][i], s["gn_main"][i])] + \
           [v for i in range(2) for v in (s["wn_bypass"][i], s["gn_bypass"][i])]
    return grads, np.asarray(flat, np.float64)


def base_state(seed):
    from greedy_multimodal_learning_amd.model import MMTM_MVCNN
    from oracle import weights
    m = weights.apply_to_module(MMTM_MVCNN(), seed=seed)
    return {k: v.detach().clone() for k, v in m.state_dict().items()}


def cmd_mirror(a, dev):
    sd = mirror_state(base_state(a.seed))
    g = torch.Generator().manual_seed(2024)
    one = torch.randn(1, a.batch, a.size, a.size, 3, generator=g).bfloat16()
    buf = torch.cat([one, one], 0)
    y = torch.randint(0, 40, (a.batch,), generator=g)
    for dt in ([torch.bfloat16, torch.float32] if a.fp32 else [torch.bfloat16]):
        grads, sums = hip_step(sd, buf, y, dev, dtype=dt)
        worst = []
        for n, g0 in grads.items():
            if not n.startswith("net_view_0."):
                continue
            g1 = grads["net_view_1." + n[len("net_view_0."):]]
            d = float((g0 - g1).abs().max()) / (float(g0.abs().max()) + 1e-30)
            worst.append((d, n))
        for n, g0 in grads.items():
            if ".fc_visual." in n:
                g1 = grads[n.replace(".fc_visual.", ".fc_skeleton.")]
                worst.append((float((g0 - g1).abs().max()) / (float(g0.abs().max()) + 1e-30), n))
        worst.sort(reverse=True)
        nz = sum(1 for d, _ in worst if d > 0)
        print(f"[mirror {dt}] B={a.batch} H={a.size}: {nz}/{len(worst)} view-0 tensors differ from view 1; "
              f"gn main0 {sums[1]:.9e} main1 {sums[3]:.9e} bypass0 {sums[5]:.9e} bypass1 {sums[7]:.9e}")
        for d, n in worst[:12]:
            print(f"   {d:.3e}  {n}")


def cmd_swap(a, dev):
    torch.set_num_threads(max(1, min(32, torch.get_num_threads())))
    sd0 = base_state(a.seed)
    g = torch.Generator().manual_seed(2024)
    buf = torch.randn(2, a.batch, a.size, a.size, 3, generator=g).bfloat16()
    y = torch.randint(0, 40, (a.batch,), generator=g)
    for tag, sd, b in (("orig", sd0, buf), ("swapped", swap_state(sd0), buf.flip(0).contiguous())):
        hg, hs = hip_step(sd, b, y, dev)
        og, os_ = oracle(sd, b, y)
        e = np.abs(hs[1::2] - os_[1::2]) / os_[1::2]
        print(f"[swap {tag}] grad-sum rel err main0 {e[0]:.3e} main1 {e[1]:.3e} bypass0 {e[2]:.3e} "
              f"bypass1 {e[3]:.3e}; oracle gn main0 {os_[1]:.6e} main1 {os_[3]:.6e}", flush=True)
        rows = []
        for n in og:
            r = og[n].reshape(-1).double()
            h = hg[n].reshape(-1).double() if hg[n].shape == og[n].shape else \
                hg[n].contiguous().reshape(-1).double()
            rel = float((h - r).norm() / (r.norm() + 1e-30))
            rows.append((rel, n, float(r.norm())))
        rows.sort(reverse=True)
        for rel, n, nr in rows[:10]:
            print(f"   {rel:.3e}  |g|={nr:.3e}  {n}")
        for pre in ("net_view_0.", "net_view_1."):
            for tail in ("conv1.weight", "layer1.0.conv1.weight", "layer2.0.conv1.weight", "layer3.0.conv1.weight",
                         "layer4.0.conv1.weight", "layer4.1.conv2.weight", "fc.weight"):
                n = pre + tail
                r = og[n].reshape(-1).double()
                h = hg[n].contiguous().reshape(-1).double()
                print(f"      {n:40s} rel {float((h - r).norm() / r.norm()):.3e} |g| {float(r.norm()):.3e}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["mirror", "swap"])
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--size", type=int, default=224)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--fp32", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    from greedy_multimodal_learning_amd import build
    build.build()
    {"mirror": cmd_mirror, "swap": cmd_swap}[a.mode](a, dev)


if __name__ == "__main__":
    main()
