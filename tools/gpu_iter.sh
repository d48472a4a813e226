#!/bin/bash
# GPU iteration: tests (selected), conv/bn micro-benchmarks, full bench
set -o pipefail
mkdir -p gpurun_out
T=${TESTS:-"tests/test_gpu_bn.py tests/test_gpu_pool.py tests/test_gpu_conv.py tests/test_gpu_mmtm_n.py tests/test_gpu_model.py"}
timeout -k 10 600 python -m pytest $T -q -p no:cacheprovider --timeout 300 > gpurun_out/iter_tests.log 2>&1
rc=$?
tail -3 gpurun_out/iter_tests.log
[ $rc -eq 0 ] || exit 1
GM_CONV_STAGES=2 timeout -k 10 300 python tools/conv_bench.py > gpurun_out/conv_bench_s2.log 2>&1 || exit 2
tail -1 gpurun_out/conv_bench_s2.log
timeout -k 10 300 python tools/conv_bench.py > gpurun_out/conv_bench_s3.log 2>&1 || exit 3
cat gpurun_out/conv_bench_s3.log
timeout -k 10 300 python tools/bn_bench.py > gpurun_out/bn_bench.log 2>&1 || exit 4
cat gpurun_out/bn_bench.log
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 5
tail -1 gpurun_out/bench.log | cut -c1-300
