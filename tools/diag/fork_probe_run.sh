set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out/fp
timeout -k 10 120 python3 tools/diag/graph_fork_probe.py 10 0 --big
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fp/s -o t -- python3 tools/diag/graph_fork_probe.py 30 40000 > /dev/null 2>&1 || exit 3
python3 tools/diag/trace_branches.py gpurun_out/fp/s/t_kernel_trace.csv
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fp/b -o t -- python3 tools/diag/graph_fork_probe.py 10 0 --big > /dev/null 2>&1 || exit 4
python3 tools/diag/trace_branches.py gpurun_out/fp/b/t_kernel_trace.csv
rm -rf gpurun_out/fp
