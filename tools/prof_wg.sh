set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd /root/repo
mkdir -p gpurun_out/pmc
export CB_OPS=wgrad CB_NOMIO=1 GM_WGRAD_ST=2
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM --output-format csv -d /tmp/pmcw1 -o sq -- python tools/conv_bench.py l2 l4 > gpurun_out/pmc/w1.log 2>&1 || exit 5
python tools/summarize_pmc.py /tmp/pmcw1 gpurun_out/pmc/w1.txt
timeout -k 10 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d /tmp/pmcw2 -o sq2 -- python tools/conv_bench.py l2 l4 > gpurun_out/pmc/w2.log 2>&1 || exit 6
python tools/summarize_pmc.py /tmp/pmcw2 gpurun_out/pmc/w2.txt
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d /tmp/pmcw3 -o sq3 -- python tools/conv_bench.py l2 l4 > gpurun_out/pmc/w3.log 2>&1 || exit 7
python tools/summarize_pmc.py /tmp/pmcw3 gpurun_out/pmc/w3.txt
cat gpurun_out/pmc/w1.txt gpurun_out/pmc/w2.txt gpurun_out/pmc/w3.txt | grep -v -i "elementwise\|distribution\|copy" 
