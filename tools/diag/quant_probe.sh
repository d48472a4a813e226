# tile-quantization probe: time one conv shape at batches whose tile counts straddle
# multiples of the CU count (tools/conv_one.py)
set -o pipefail
for s in l2 l3 l4 l1; do
  for b in 32 48 64 80 84 96 128; do
    timeout -k 10 120 python tools/conv_one.py --shape $s --op fwd --batch $b --reps 50 2>&1 | grep -v amdgpu.ids || exit 5
  done
done
