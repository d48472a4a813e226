#!/bin/bash
# per-shape conv bench under several env settings: bash tools/gpu_envs.sh "A=1 B=2" "C=3" ...
set -o pipefail
mkdir -p gpurun_out
i=0
for E in "$@"; do
  echo "== $E"
  env $E timeout -k 10 200 python tools/conv_bench.py > gpurun_out/envs_$i.log 2>&1 || exit 2
  grep -E "wgrad|total" gpurun_out/envs_$i.log | awk '{printf "%s %s %s | ", $1, $2, $3} END {print ""}'
  i=$((i+1))
done
