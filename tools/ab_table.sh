#!/bin/bash
# tools/trunk_table.py under two environment settings (run on the GPU box):
#   bash tools/ab_table.sh ONLY 'VAR=VAL' 'VAR=VAL'   -> gpurun_out/ab_table_<n>.md
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
only=$1; shift
i=0
for s in "$@"; do
  i=$((i + 1))
  env "$s" timeout -k 10 300 python tools/trunk_table.py --only "$only" > gpurun_out/ab_table_$i.md 2>&1 || exit 1
  echo "== $s"; grep -E "^\| |family" gpurun_out/ab_table_$i.md | grep -E "wgrad|family"
done
