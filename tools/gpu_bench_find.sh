set -o pipefail
cd /root/repo
timeout -k 10 900 python bench.py --no-cpu-baseline --miopen-find --warmup 8 > gpurun_out/bench_find.log 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp && cd /root/repo
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_find -o bench -- python bench.py --steps 10 --warmup 8 --no-cpu-baseline --miopen-find > gpurun_out/prof_find.log 2>&1 || exit 5
