#!/bin/bash
# one GPU session: tests, smoke, bench, rocprof kernel stats
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/gpu_tests.log 2>&1
echo "tests exit=$?" >> gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 3
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp && cd /root/repo
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit 5
echo done
