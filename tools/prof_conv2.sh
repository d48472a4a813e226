set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd /root/repo
mkdir -p gpurun_out/pmc
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d /tmp/pmc3 -o tcc -- python tools/conv_bench.py l2 l3 > gpurun_out/pmc/tcc.log 2>&1 || exit 5
python tools/summarize_pmc.py /tmp/pmc3 gpurun_out/pmc/tcc.txt
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pmc4 -o fetch -- python tools/conv_bench.py l2 l3 > gpurun_out/pmc/fetch.log 2>&1 || exit 6
python tools/summarize_pmc.py /tmp/pmc4 gpurun_out/pmc/fetch.txt
timeout -k 10 300 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d /tmp/pmc5 -o tcp -- python tools/conv_bench.py l2 > gpurun_out/pmc/tcp.log 2>&1 || exit 7
python tools/summarize_pmc.py /tmp/pmc5 gpurun_out/pmc/tcp.txt
