#!/bin/bash
# bench ms/step under env-var variants: tools/gpu_variants.sh tag "VAR=a" "VAR=b" ...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
cd /root/repo
for v in "$@"; do
  echo "== $v" >> gpurun_out/${tag}_variants.log
  env $v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/${tag}_tmp.log 2>&1 || { cat gpurun_out/${tag}_tmp.log >> gpurun_out/${tag}_variants.log; exit 3; }
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/${tag}_tmp.log >> gpurun_out/${tag}_variants.log
done
echo done
