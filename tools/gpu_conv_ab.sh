set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_conv.py tests/test_gpu_model.py -q -p no:cacheprovider --timeout 200 > gpurun_out/conv_tests.log 2>&1
rc=$?; tail -2 gpurun_out/conv_tests.log; [ $rc -eq 0 ] || exit 1
GM_CONV_LEAN=0 timeout -k 10 300 python tools/conv_bench.py > gpurun_out/conv_bench_old.log 2>&1 || exit 2
timeout -k 10 300 python tools/conv_bench.py > gpurun_out/conv_bench_new.log 2>&1 || exit 3
paste <(awk '{print $1, $2, $3}' gpurun_out/conv_bench_old.log) <(awk '{print $3, $4, $5, $6}' gpurun_out/conv_bench_new.log)
tail -1 gpurun_out/conv_bench_old.log; tail -1 gpurun_out/conv_bench_new.log
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 4
tail -1 gpurun_out/bench.log | cut -c1-200
