#!/bin/bash
# bench.py under several env settings: bash tools/gpu_bench_envs.sh "A=1 B=2" "C=3" ...
set -o pipefail
mkdir -p gpurun_out
i=0
for E in "$@"; do
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/benv_$i.log 2>&1 || exit 2
  echo "== $E : $(tail -1 gpurun_out/benv_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["achieved"])')"
  i=$((i+1))
done
