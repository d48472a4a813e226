#!/bin/bash
# Interleaved A/B of environment knobs on the default bench (run on the GPU box):
#   bash tools/ab_env.sh ROUNDS 'VAR=VAL[,VAR=VAL]' ...   ('-' = the defaults)
# each setting runs bench.py --no-cpu-baseline --steps 40 once per round, in order;
# prints one ms_per_step line per run -> gpurun_out/ab_env.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
rounds=$1; shift
: > gpurun_out/ab_env.txt
for r in $(seq 1 "$rounds"); do
  for s in "$@"; do
    envs=()
    [ "$s" != "-" ] && IFS=, read -ra envs <<< "$s"
    out=$(env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 2>gpurun_out/ab_env_err.log) || { echo "FAILED: $s"; exit 1; }
    echo "round $r  $s  $(grep -o '"ms_per_step": [0-9.]*' <<< "$out") $(grep -o '"frac": [0-9.]*' <<< "$out" | head -1)" | tee -a gpurun_out/ab_env.txt
  done
done
