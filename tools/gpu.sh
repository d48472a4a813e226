#!/bin/bash
# The one GPU-session driver (run on the box through gpurun from the repo root):
#
#   gpurun --timeout 1200 -- bash tools/gpu.sh STEP [STEP ...]
#
# Steps (run in order, each under its own time limit; the first failure ends the call):
#   tests        pytest -m gpu (one process, per-test timeout)       -> gpurun_out/gpu_tests.log
#   tests:EXPR   the same, restricted with -k EXPR
#   smoke        __graft_entry__.smoke()                              -> gpurun_out/smoke.log
#   bench        python bench.py (defaults, incl. cpu_baseline)       -> gpurun_out/bench.log
#   benchq       python bench.py --no-cpu-baseline                    -> gpurun_out/benchq.log
#   bench:ARGS   python bench.py ARGS (commas become spaces)          -> gpurun_out/bench_ARGS.log
#   prof         rocprofv3 --kernel-trace --stats of a short bench    -> gpurun_out/prof/
#   profw:W      the same for bench.py --workload W (C4, C5)           -> gpurun_out/prof_W/
#   prof:V=X,..  the same with environment variables set               -> gpurun_out/prof_V_X/
#   pmc:NAME     one rocprofv3 --pmc pass over a short bench (sets below) -> gpurun_out/pmc_NAME/
#   table        tools/trunk_table.py: per-shape trunk launch table    -> gpurun_out/trunk_table.md
#   pmct:NAME    one rocprofv3 --pmc pass over tools/trunk_table.py, summarised per (kernel, grid)
#                                                                     -> gpurun_out/pmct_NAME.txt
#   pmcg:NAME    one rocprofv3 --pmc pass over tools/traffic_probe.py (the fused norms+SGD pass)
#                                                                     -> gpurun_out/pmcg_NAME.txt
#   trunkpmc     three rocprofv3 --pmc passes over tools/trunk_pmc.py (FETCH, WRITE, MFMA/LDS set),
#                per-op table + conv-family traffic json         -> gpurun_out/trunk_pmc.md, trunk_pmc.json
#   mmtmpmc      two rocprofv3 --pmc passes (FETCH, WRITE) over tools/mmtm_probe.py (the MMTM squeeze
#                at B=256 rotating over 411 MB)                   -> gpurun_out/traffic_mmtm.json
#   pmcone:SET:ARGS one rocprofv3 --pmc pass (counter set SET above) over tools/conv_one.py ARGS
#                (commas become spaces), summarised per kernel  -> gpurun_out/pmcone_SET.txt
#   rp:FILE[,ARGS] rocprofv3 --kernel-trace --stats of python FILE ARGS -> gpurun_out/rp_FILE/
#   py:FILE[,ARGS] python FILE ARGS (a tools/ script; commas become spaces) -> gpurun_out/py_FILE.log
#   env:V=X,..   export the variables for the following steps (bench:* logs get the tag _V_X); env: clears
set -o pipefail
mkdir -p gpurun_out
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
PROFCMD="python3 bench.py --steps 10 --warmup 3 --profile"

declare -A PMC
PMC[mfma]="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS"
PMC[lds]="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES"
PMC[fetch]="FETCH_SIZE"
PMC[write]="WRITE_SIZE"
PMC[opmfma]="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES"
PMC[stall]="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU"
PMC[l2]="TCC_HIT_sum TCC_MISS_sum"
PMC[lds2]="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAVES"

for s in "$@"; do
  echo "=== $s $(date +%T)"
  case "$s" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 -rA \
        --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 11; }
      tail -3 gpurun_out/gpu_tests.log ;;
    tests:*)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 -rA \
        --timeout-method thread -k "${s#tests:}" > "gpurun_out/gpu_tests_k_$(echo "${s#tests:}" | tr -c 'A-Za-z0-9\n' '_' | cut -c1-40).log" 2>&1 \
        || { tail -40 "gpurun_out/gpu_tests_k_$(echo "${s#tests:}" | tr -c 'A-Za-z0-9\n' '_' | cut -c1-40).log"; exit 12; }
      tail -3 "gpurun_out/gpu_tests_k_$(echo "${s#tests:}" | tr -c 'A-Za-z0-9\n' '_' | cut -c1-40).log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
        || { tail -30 gpurun_out/smoke.log; exit 13; }
      tail -2 gpurun_out/smoke.log ;;
    bench)
      timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 14; }
      tail -1 gpurun_out/bench.log | cut -c1-400 ;;
    benchq)
      timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/benchq.log 2>&1 \
        || { tail -30 gpurun_out/benchq.log; exit 15; }
      tail -1 gpurun_out/benchq.log | cut -c1-400 ;;
    env:*)
      for v in $ENVSET; do unset "${v%%=*}"; done
      ENVSET="${s#env:}"; ENVSET="${ENVSET//,/ }"; TAG=""
      [ -n "$ENVSET" ] && { export $ENVSET; TAG="_$(echo "$ENVSET" | tr -c 'A-Za-z0-9\n' '_')"; } ;;
    bench:*)
      a="${s#bench:}"; f="gpurun_out/bench_$(echo "$a" | tr -c 'A-Za-z0-9_=.\n-' '_')$TAG.log"
      timeout -k 10 600 python -u bench.py ${a//,/ } > "$f" 2>&1 || { tail -30 "$f"; exit 16; }
      tail -1 "$f" | cut -c1-400 ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
        -- $PROFCMD > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 17; }
      python3 tools/summarize_stats.py gpurun_out/prof/bench_kernel_stats.csv 13 | head -40 ;;
    prof:*)
      e="${s#prof:}"; d="gpurun_out/prof_$(echo "$e" | tr -c 'A-Za-z0-9\n' '_')"
      export ${e//,/ }
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o bench \
        -- $PROFCMD > "$d.log" 2>&1 || { tail -30 "$d.log"; exit 17; }
      for v in ${e//,/ }; do unset "${v%%=*}"; done
      python3 tools/summarize_stats.py "$d/bench_kernel_stats.csv" 13 | head -40 ;;
    profw:*)
      w="${s#profw:}"; d="gpurun_out/prof_$w"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o bench \
        -- python3 bench.py --workload "$w" --steps 10 --warmup 3 --profile > "$d.log" 2>&1 || { tail -30 "$d.log"; exit 27; }
      python3 tools/summarize_stats.py "$d/bench_kernel_stats.csv" 13 | head -40 ;;
    pmc:*)
      n="${s#pmc:}"
      timeout -s KILL 300 rocprofv3 --pmc ${PMC[$n]} --output-format csv -d "gpurun_out/pmc_$n" -o pmc \
        -- $PROFCMD > "gpurun_out/pmc_$n.log" 2>&1 || { tail -30 "gpurun_out/pmc_$n.log"; exit 18; } ;;
    table)
      timeout -k 10 600 python -u tools/trunk_table.py --md gpurun_out/trunk_table.md > gpurun_out/trunk_table.log 2>&1 \
        || { tail -30 gpurun_out/trunk_table.log; exit 20; }
      tail -4 gpurun_out/trunk_table.md ;;
    pmct:*)
      n="${s#pmct:}"
      timeout -s KILL 300 rocprofv3 --pmc ${PMC[$n]} --output-format csv -d "gpurun_out/pmct_$n" -o pmc \
        -- python3 tools/trunk_table.py --reps 4 > "gpurun_out/pmct_$n.log" 2>&1 || { tail -30 "gpurun_out/pmct_$n.log"; exit 21; }
      python3 tools/pmc_table.py "gpurun_out/pmct_$n" > "gpurun_out/pmct_$n.txt" && rm -rf "gpurun_out/pmct_$n"
      head -5 "gpurun_out/pmct_$n.txt" ;;
    pmcg:*)
      n="${s#pmcg:}"
      timeout -s KILL 300 rocprofv3 --pmc ${PMC[$n]} --output-format csv -d "gpurun_out/pmcg_$n" -o pmc \
        -- python3 tools/traffic_probe.py > "gpurun_out/pmcg_$n.log" 2>&1 || { tail -30 "gpurun_out/pmcg_$n.log"; exit 22; }
      python3 tools/pmc_table.py "gpurun_out/pmcg_$n" > "gpurun_out/pmcg_$n.txt" && rm -rf "gpurun_out/pmcg_$n"
      grep group_sumsq "gpurun_out/pmcg_$n.txt" ;;
    trunkpmc)
      for n in fetch write opmfma; do
        timeout -s KILL 300 rocprofv3 --pmc ${PMC[$n]} --output-format csv -d "gpurun_out/tp_$n" -o pmc \
          -- python3 tools/trunk_pmc.py run > "gpurun_out/tp_$n.log" 2>&1 || { tail -30 "gpurun_out/tp_$n.log"; exit 23; }
      done
      python3 tools/trunk_pmc.py report gpurun_out/tp_fetch gpurun_out/tp_write gpurun_out/tp_opmfma \
        --json gpurun_out/trunk_pmc.json > gpurun_out/trunk_pmc.md && rm -rf gpurun_out/tp_fetch gpurun_out/tp_write gpurun_out/tp_opmfma
      tail -3 gpurun_out/trunk_pmc.md ;;
    mmtmpmc)
      for n in fetch write; do
        timeout -s KILL 120 rocprofv3 --pmc ${PMC[$n]} --output-format csv -d "gpurun_out/mp_$n" -o pmc \
          -- python3 tools/mmtm_probe.py run > "gpurun_out/mp_$n.log" 2>&1 || { tail -30 "gpurun_out/mp_$n.log"; exit 24; }
      done
      python3 tools/mmtm_probe.py report gpurun_out/mp_fetch gpurun_out/mp_write --json gpurun_out/traffic_mmtm.json \
        > gpurun_out/mmtm_pmc.log && rm -rf gpurun_out/mp_fetch gpurun_out/mp_write
      tail -4 gpurun_out/traffic_mmtm.json ;;
    pmcone:*)
      r="${s#pmcone:}"; n="${r%%:*}"; args="${r#*:}"; d="gpurun_out/pmcone_${n}_$(echo "$args" | tr -c 'A-Za-z0-9\n' '_')"
      timeout -s KILL 120 rocprofv3 --pmc ${PMC[$n]} --output-format csv -d "$d" -o pmc \
        -- python3 tools/conv_one.py ${args//,/ } > "$d.log" 2>&1 || { tail -30 "$d.log"; exit 25; }
      python3 tools/pmc_table.py "$d" | grep -v spin_kernel > "$d.txt" && rm -rf "$d"
      cat "$d.txt" ;;
    rp:*)
      a="${s#rp:}"; f="${a%%,*}"; args=""; [ "$f" != "$a" ] && args="${a#*,}"
      d="gpurun_out/rp_$(basename "$f" .py)"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o rp \
        -- python3 "$f" ${args//,/ } > "$d.log" 2>&1 || { tail -30 "$d.log"; exit 26; }
      tail -5 "$d.log"; python3 tools/summarize_stats.py "$d/rp_kernel_stats.csv" 1 | head -12 ;;
    py:*)
      a="${s#py:}"; f="${a%%,*}"; args=""; [ "$f" != "$a" ] && args="${a#*,}"
      lg="gpurun_out/py_$(basename "$f" .py)$(echo "$args" | tr -c 'A-Za-z0-9\n' '_' | cut -c1-60).log"
      timeout -k 10 600 python -u "$f" ${args//,/ } > "$lg" 2>&1 || { tail -30 "$lg"; exit 19; }
      tail -20 "$lg" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== all done $(date +%T)"
