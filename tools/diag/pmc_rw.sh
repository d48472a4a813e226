# SQ counters of the resident-weight layer-1 kernel (k_conv_rw) and the im2col kernel on l1 fwd
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rw in 1 0; do
  GM_CONV_RW=$rw timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcrw_$rw -o pmc -- python3 tools/conv_one.py --shape l1 > gpurun_out/pmcrw_$rw.log 2>&1 || exit 5
  python3 tools/pmc_table.py gpurun_out/pmcrw_$rw > gpurun_out/pmcrw_$rw.txt && rm -rf gpurun_out/pmcrw_$rw
  grep conv gpurun_out/pmcrw_$rw.txt
  GM_CONV_RW=$rw timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM --output-format csv -d gpurun_out/pmcrw2_$rw -o pmc -- python3 tools/conv_one.py --shape l1 > gpurun_out/pmcrw2_$rw.log 2>&1 || exit 6
  python3 tools/pmc_table.py gpurun_out/pmcrw2_$rw > gpurun_out/pmcrw2_$rw.txt && rm -rf gpurun_out/pmcrw2_$rw
  grep conv gpurun_out/pmcrw2_$rw.txt
done
