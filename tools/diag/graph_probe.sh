#!/bin/bash
mkdir -p gpurun_out
for p in conv conv_bwd bn pool mmtm norms model_fwd model_step; do
  timeout -k 10 120 python tools/diag/graph_probe.py $p > gpurun_out/probe_$p.log 2>&1
  echo "$p rc=$?"
  tail -3 gpurun_out/probe_$p.log | grep -v "^$" | head -3
done
