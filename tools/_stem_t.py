import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import trunk_table as T
from greedy_multimodal_learning_amd import build
if len(sys.argv) > 1 and sys.argv[1] == "build":
    build.build()
dev = torch.device("cuda:0")
ops = T.conv_ops(64, dev, 320e6)
name, op, cnt, fl, nb, fn = ops[0]
print(name, op, f"{T._time(fn, 10) * 1e6:.1f} us", flush=True)
