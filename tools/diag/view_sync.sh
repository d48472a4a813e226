# A/B of the view-stream synchronisation granularity (GM_VIEW_SYNC layer / block), C2 bench
set -o pipefail
for r in 1 2; do
  for v in layer block; do
    echo -n "GM_VIEW_SYNC=$v: "
    GM_VIEW_SYNC=$v timeout -k 10 300 python bench.py --no-cpu-baseline --profile --steps 30 || exit 5
  done
done
