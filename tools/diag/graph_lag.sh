#!/bin/bash
# Where the two view branches of the captured step start relative to each other, under
# several runtime settings: kernel trace of a short bench per variant, summarised by
# tools/step_listing.py (concurrency profile + the first launches of the median step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/lag
run() {  # name, env assignments...
  local n="$1"; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline $BENCHX > "gpurun_out/lag/$n.bench" 2>&1 || return 1
  echo "$n: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/lag/$n.bench)"
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "gpurun_out/lag/$n" -o t \
    -- python3 bench.py --steps 8 --warmup 3 --profile $BENCHX > "gpurun_out/lag/$n.prof.log" 2>&1 || return 1
  python3 tools/step_listing.py "gpurun_out/lag/$n/t_kernel_trace.csv" --list > "gpurun_out/lag/$n.txt" || return 1
  head -3 "gpurun_out/lag/$n.txt"
  rm -rf "gpurun_out/lag/$n"
}
for v in "$@"; do
  case "$v" in
    base) run base GM_X=0 || exit 1 ;;
    hwq8) run hwq8 GPU_MAX_HW_QUEUES=8 || exit 1 ;;
    eager) BENCHX=--eager run eager GM_X=0 || exit 1 ;;
    il0) run il0 GM_VIEW_INTERLEAVE=0 || exit 1 ;;
    nopkt) run nopkt DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit 1 ;;
    env:*) kv="${v#env:}"; run "$(echo "$kv" | tr -c 'A-Za-z0-9_\n' '_')" "${kv//+/ }" || exit 1 ;;
    *) echo "unknown $v"; exit 2 ;;
  esac
done
