#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_bn.py tests/test_gpu_pool.py tests/test_gpu_model.py -q -x -p no:cacheprovider --timeout 200 > gpurun_out/bnc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/bnc_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/bnc_tests.log | head -20; exit 1; }
timeout -k 10 300 python tools/bn_micro.py || exit 2
bash tools/gpu_bench_envs.sh GM_X=0 || exit 3
