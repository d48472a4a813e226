"""Where does the resident-weight stem kernel differ from the im2col kernel? (diagnostic)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from greedy_multimodal_learning_amd import _lib as L  # noqa: E402
from greedy_multimodal_learning_amd import conv as G  # noqa: E402

lib = L.load()
N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
g = torch.Generator(device="cuda").manual_seed(1)
x = torch.randn(N, 3, 224, 224, device="cuda", generator=g)
w = torch.randn(64, 3, 7, 7, device="cuda", generator=g) / 12
P, Q, Sp, Hp, Wp = G._stem_geom(224, 224, 7, 7, 3)
xp, wp = G.stem_pack(x, w, 3)
lib.gm_conv_set_stem(0)
y0 = G.stem_fwd(xp, wp, P, Q)
lib.gm_conv_set_stem(int(os.environ.get("STEM", "1")))
y1 = G.stem_fwd(xp, wp, P, Q)
torch.cuda.synchronize()
d = (y1.float() - y0.float()).abs()  # [N,64,P,Q]
bad = d > 1e-2 * y0.float().abs().max()
print("N", N, "bad", int(bad.sum()), "of", bad.numel(), "max diff", float(d.max()))
if bad.any():
    idx = bad.nonzero()
    print("images", sorted(set(idx[:, 0].tolist()))[:20])
    print("channels", sorted(set(idx[:, 1].tolist()))[:64])
    print("rows", sorted(set(idx[:, 2].tolist()))[:40])
    print("cols", sorted(set(idx[:, 3].tolist()))[:40])
    rowsets = sorted(set((idx[:, 0] * P + idx[:, 2]).tolist()))
    print("bad output rows (b*P+p)", len(rowsets), rowsets[:40])

# timing of the selected variant vs the im2col kernel
for v in (0, int(os.environ.get("STEM", "1"))):
    lib.gm_conv_set_stem(v)
    for _ in range(3):
        G.stem_fwd(xp, wp, P, Q)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        G.stem_fwd(xp, wp, P, Q)
    e1.record()
    torch.cuda.synchronize()
    print(f"stem variant {v}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us")
