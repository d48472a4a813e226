#!/bin/bash
# usage (GPU box, repo root): build two libraries here, copy them to gpurun_lib_new.so / gpurun_lib_old.so, then
#   bash tools/diag/ab_lib.sh ROUNDS [bench args]  -> ms/step per round and library (default: C2, 40 steps)
# alternate two prebuilt libraries: bench each in turn (new, old) x ROUNDS
set -o pipefail
R=${1:-3}
shift
ARGS="${*:---steps 40}"
for i in $(seq 1 $R); do
  for v in new old; do
    cp gpurun_lib_$v.so greedy_multimodal_learning_amd/libgreedymml_hip.so
    echo "round $i $v"
    timeout -k 10 240 python -u bench.py --no-cpu-baseline $ARGS | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms_per_step', d['ms_per_step'])" || exit 1
  done
done
cp gpurun_lib_new.so greedy_multimodal_learning_amd/libgreedymml_hip.so
