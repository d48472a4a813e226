#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_conv.py -q -x -p no:cacheprovider --timeout 200 > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/ab_tests.log | head -20; exit 1; }
bash tools/gpu_envs.sh GM_WGRAD_V=1 GM_WGRAD_V=3 "GM_WGRAD_V=3 GM_WGRAD_ST=2" "GM_WGRAD_V=3 GM_WGRAD_ST=4" "GM_WGRAD_V=3 GM_WGRAD_WGS=256" "GM_WGRAD_V=3 GM_WGRAD_WGS=1024"
