# weight-gradient workgroup target (split count) probe: GM_WGRAD_WGS = 256 / 512 (default) / 1024
set -o pipefail
for w in 512 256 1024 384; do
  echo "== GM_WGRAD_WGS=$w"
  GM_WGRAD_WGS=$w timeout -k 10 300 python -u tools/conv_ab.py --pipes h --wgrad --rounds 3 > gpurun_out/wg_$w.log 2>&1 || exit 5
  grep "wgrad\|family" gpurun_out/wg_$w.log
done
