#!/bin/bash
# tests that touch the engine/MMTM + eager and graph bench + rocprof of the graph bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q ${PYTEST_K:+-k "$PYTEST_K"} -p no:cacheprovider --timeout 300 > gpurun_out/iter_tests.log 2>&1
rc=$?
tail -5 gpurun_out/iter_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py --no-cpu-baseline --eager > gpurun_out/bench_eager.log 2>&1 || exit 4
tail -1 gpurun_out/bench_eager.log | cut -c1-250
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 5
tail -1 gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp && cd /root/repo
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit 6
python3 tools/summarize_stats.py gpurun_out/prof/bench_kernel_stats.csv 13
