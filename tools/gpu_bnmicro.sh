set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/bn_micro.py > gpurun_out/bn_micro.log 2>&1 || exit 2
cat gpurun_out/bn_micro.log
cd /tmp && export TMPDIR=/tmp && cd /root/repo
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/bnt -o bn -- python3 tools/bn_micro.py > gpurun_out/bn_trace.log 2>&1 || exit 3
python3 tools/trace_summary.py $(ls /tmp/bnt/*/*kernel_trace.csv /tmp/bnt/*kernel_trace.csv 2>/dev/null | head -1) k_bn > gpurun_out/bn_trace.txt
cat gpurun_out/bn_trace.txt
