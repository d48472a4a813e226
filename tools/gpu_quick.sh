#!/bin/bash
# quick GPU iteration: selected tests + micro benches + bench (each step time-limited)
set -o pipefail
mkdir -p gpurun_out
T=${TESTS:-"tests/test_gpu_bn.py tests/test_gpu_conv.py tests/test_gpu_model.py"}
timeout -k 10 600 python -m pytest $T -q -p no:cacheprovider -x --timeout 300 > gpurun_out/quick_tests.log 2>&1
echo "tests exit=$?" >> gpurun_out/quick_tests.log
tail -3 gpurun_out/quick_tests.log
grep -q "tests exit=0" gpurun_out/quick_tests.log || exit 1
if [ -n "$MICRO" ]; then
  timeout -k 10 300 python $MICRO > gpurun_out/micro.log 2>&1 || exit 2
  cat gpurun_out/micro.log
fi
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 4
tail -1 gpurun_out/bench.log | cut -c1-300
