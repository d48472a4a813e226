#!/bin/bash
# quick GPU iteration: selected gpu tests, bench, rocprof kernel trace
# usage: tools/gpu_quick2.sh tag "pytest selection args"
set -o pipefail
tag=${1:-q}
sel=${2:-tests}
mkdir -p gpurun_out
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest $sel -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?
echo "tests exit=$rc" >> gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || exit 2
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${tag}_bench.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o bench \
    -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 || exit 6
echo done
