set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd /root/repo
mkdir -p gpurun_out/pmc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pf -o f -- python3 tools/traffic_probe.py > gpurun_out/pmc/tf.log 2>&1 || exit 5
python3 tools/summarize_pmc.py /tmp/pf gpurun_out/pmc/traffic_fetch.txt
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pw -o w -- python3 tools/traffic_probe.py > gpurun_out/pmc/tw.log 2>&1 || exit 6
python3 tools/summarize_pmc.py /tmp/pw gpurun_out/pmc/traffic_write.txt
grep -A2 "group_sumsq" gpurun_out/pmc/traffic_fetch.txt gpurun_out/pmc/traffic_write.txt
