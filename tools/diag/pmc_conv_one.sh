set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for p in 0 5 6; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc1_p$p -o pmc -- python3 tools/conv_one.py --shape l2 --pipe $p > gpurun_out/pmc1_p$p.log 2>&1 || exit 5
  python3 tools/pmc_table.py gpurun_out/pmc1_p$p > gpurun_out/pmc1_p$p.txt && rm -rf gpurun_out/pmc1_p$p
  grep conv_igemm gpurun_out/pmc1_p$p.txt
done
for p in 0 5 6; do timeout -k 10 60 python3 tools/conv_one.py --shape l2 --pipe $p; done
