# A/B of which view runs on the side stream and which is captured first (C2 bench)
set -o pipefail
for r in 1 2; do
  for cfg in "0 0" "1 0" "0 1" "1 1"; do
    set -- $cfg
    echo -n "swap=$1 main_first=$2: "
    GM_VIEW_SWAP=$1 GM_VIEW_MAIN_FIRST=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 | python3 -c "import sys,json; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])" || exit 5
  done
done
