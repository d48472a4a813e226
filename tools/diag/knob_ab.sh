#!/bin/bash
# Step-level A/B of kernel planning knobs: bench.py ms/step per env variant, two
# interleaved rounds (the isolated-kernel tuning in tools/conv_ab.py does not see the
# other trunk's kernels sharing the CUs).  usage: knob_ab.sh 'ENV=V[+ENV=V]' ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 1 2; do
  for v in base "$@"; do
    e=""; [ "$v" != base ] && e="${v//+/ }"
    ms=$(env $e timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || exit 1
    echo "round $r $v: $ms"
  done
done
