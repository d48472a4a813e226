set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "stem or pool or vtrunk" > gpurun_out/t.log 2>&1
timeout -k 10 200 python -u tools/trunk_table.py --only bn > gpurun_out/tt.log 2>&1
timeout -k 10 120 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline > gpurun_out/b1.log 2>&1
