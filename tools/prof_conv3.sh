set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd /root/repo
mkdir -p gpurun_out/pmc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM --output-format csv -d /tmp/pmc6 -o sq -- python tools/conv_bench.py l1 l2 > gpurun_out/pmc/sq.log 2>&1 || exit 5
python tools/summarize_pmc.py /tmp/pmc6 gpurun_out/pmc/sq.txt
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM --output-format csv -d /tmp/pmc7 -o sq2 -- python tools/conv_bench.py l1 l2 > gpurun_out/pmc/sq2.log 2>&1 || exit 6
python tools/summarize_pmc.py /tmp/pmc7 gpurun_out/pmc/sq2.txt
cat gpurun_out/pmc/sq.txt gpurun_out/pmc/sq2.txt
