set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd /root/repo
mkdir -p gpurun_out/pmc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d /tmp/pmc1 -o conv_sq -- python tools/conv_bench.py l2 l1 > gpurun_out/pmc/conv_sq.log 2>&1 || exit 5
python tools/summarize_pmc.py /tmp/pmc1 gpurun_out/pmc/conv_sq.txt
timeout -k 10 300 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d /tmp/pmc2 -o conv_sq2 -- python tools/conv_bench.py l2 > gpurun_out/pmc/conv_sq2.log 2>&1 || exit 6
python tools/summarize_pmc.py /tmp/pmc2 gpurun_out/pmc/conv_sq2.txt
