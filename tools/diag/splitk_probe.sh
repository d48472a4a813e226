# split-K configuration probe on the layer-3/4 convolutions (tools/conv_one.py): default
# target (384 workgroups), and 200 / 256 / 512 workgroup targets, forward and dgrad
set -o pipefail
for sh in l3 l4 l4.0.c1 l3.0.c1; do
  for op in fwd dgrad; do
    for t in 384 200 256 512 0; do
      echo -n "target $t: "
      GM_CONV_SPLITK=$t timeout -k 10 60 python3 tools/conv_one.py --shape $sh --op $op || exit 5
    done
  done
done
