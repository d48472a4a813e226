#!/bin/bash
# GPU session: gpu tests, smoke, bench (view streams on / off), rocprof kernel stats.
# usage: tools/gpu_ab.sh [tag]
set -o pipefail
tag=${1:-ab}
mkdir -p gpurun_out
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?
echo "tests exit=$rc" >> gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${tag}_bench.log 2>&1 || exit 4
GM_VIEW_STREAMS=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${tag}_bench_nostreams.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o bench \
    -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${tag}_prof.log 2>&1 || exit 6
echo done
