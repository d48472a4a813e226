#!/bin/bash
set -o pipefail
export CB_OPS=fwd,dgrad CB_NOMIO=1
i=0
for E in "$@"; do
  echo "== $E"
  env $E timeout -k 10 200 python tools/conv_bench.py > gpurun_out/fenvs_$i.log 2>&1 || exit 2
  grep -E "fwd|dgrad" gpurun_out/fenvs_$i.log | awk '{printf "%s %s %s | ", $1, $2, $3} END {print ""}'
  i=$((i+1))
done
