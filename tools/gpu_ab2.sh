#!/bin/bash
# A/B of one env knob: conv tests, per-shape conv bench with and without the knob, then bench.py
# usage: bash tools/gpu_ab2.sh "ENV=val" [shapes...]
set -o pipefail
mkdir -p gpurun_out
KNOB="$1"; shift
timeout -k 10 300 python -m pytest tests/test_gpu_conv.py tests/test_gpu_model.py -q -x -p no:cacheprovider --timeout 200 > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit 1
env $KNOB timeout -k 10 300 python tools/conv_bench.py "$@" > gpurun_out/ab_a.log 2>&1 || exit 2
timeout -k 10 300 python tools/conv_bench.py "$@" > gpurun_out/ab_b.log 2>&1 || exit 3
paste <(awk '{print $1, $2, $3}' gpurun_out/ab_a.log) <(awk '{print $3, $4}' gpurun_out/ab_b.log)
tail -1 gpurun_out/ab_a.log; tail -1 gpurun_out/ab_b.log
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 4
tail -1 gpurun_out/bench.log | cut -c1-250
