#!/bin/bash
# bench + rocprof kernel stats of the bench (no tests)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 4
tail -1 gpurun_out/bench.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd /root/repo
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit 5
python3 tools/summarize_stats.py gpurun_out/prof/bench_kernel_stats.csv 13
