# resident-weight layer-1 kernel vs the im2col kernel (GM_CONV_RW), tools/conv_one.py
set -o pipefail
for op in fwd dgrad; do
  for rw in ${RWS:-0 1}; do
    echo -n "rw=$rw "
    GM_CONV_RW=$rw timeout -k 10 120 python tools/conv_one.py --shape l1 --op $op --reps 50 2>&1 | grep -v amdgpu.ids || exit 5
  done
done
