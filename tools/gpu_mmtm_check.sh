#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_mmtm.py tests/test_gpu_kernels.py tests/test_gpu_mmtm_n.py -q -x -p no:cacheprovider --timeout 200 > gpurun_out/mm_tests.log 2>&1
rc=$?; tail -2 gpurun_out/mm_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/mm_tests.log | head -20; exit 1; }
for E in GM_X=0 GM_MMTM_RED_WGS=512 GM_MMTM_RED_WGS=2048; do
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bm.log 2>&1 || exit 2
  echo "$E $(tail -1 gpurun_out/bm.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline_mmtm"]["achieved"], d["roofline_mmtm"]["avg_launch_us"])')"
done
