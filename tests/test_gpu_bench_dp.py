"""`python bench.py --gpus 2` without a launcher runs two ranks (VERDICT r03 missing #1):
on a one-GPU box both ranks share cuda:0 over gloo (the rehearsal knobs
GM_BENCH_DIST_BACKEND / GM_BENCH_SAME_DEVICE; the driver's 8-GPU node uses RCCL, one GPU
per rank) and rank 0 prints the line with n_gpus = 2."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus2_spawns_two_ranks():
    env = dict(os.environ, GM_BENCH_DIST_BACKEND="gloo", GM_BENCH_SAME_DEVICE="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "2",
                        "--batch", "8", "--profile"], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    assert lines[0]["n_gpus"] == 2 and lines[0]["value"] > 0
