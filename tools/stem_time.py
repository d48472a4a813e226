"""Time the stem convolution launches (forward, weight gradient) of the view-batched trunk
alone, as tools/trunk_table.py does (HIP events, operand sets rotating past the Infinity
Cache): python tools/stem_time.py [build]."""
import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import trunk_table as T
from greedy_multimodal_learning_amd import build
if len(sys.argv) > 1 and sys.argv[1] == "build":
    build.build()
dev = torch.device("cuda:0")
ops = T.conv_ops(64, dev, 320e6)
for name, op, cnt, fl, nb, fn in ops:
    if name == "conv1":
        print(name, op, f"{T._time(fn, 10) * 1e6:.1f} us", flush=True)
