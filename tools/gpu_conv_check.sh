#!/bin/bash
# conv parity tests, per-shape fwd/dgrad timing, bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_conv.py tests/test_gpu_model.py -q -x -p no:cacheprovider --timeout 200 > gpurun_out/cc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/cc_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/cc_tests.log | head -20; exit 1; }
bash tools/gpu_fwd_envs.sh GM_X=0 || exit 2
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 3
tail -1 gpurun_out/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["ms_per_step"], d["roofline"]["achieved"])'
