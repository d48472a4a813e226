set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for i in 1 2 3; do
 for f in "" "--curate-all"; do
  out=$(timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 $f) || exit 1
  echo "run $i [$f] $(grep -o '"ms_per_step": [0-9.]*' <<< "$out") $(grep -o '"curation_steps_timed": [0-9]*' <<< "$out")"
 done
done
