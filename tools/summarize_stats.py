"""Summarise a rocprofv3 kernel_stats.csv per step: total and top kernels."""
import csv
import sys

path, nsteps = sys.argv[1], int(sys.argv[2])
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"kernel time per step: {tot / nsteps / 1e6:.3f} ms")
for r in rows[:30]:
    print(f"{r['Name'][:100]:100s} calls/step={int(r['Calls']) / nsteps:6.1f} avg_us={float(r['AverageNs']) / 1e3:8.2f} "
          f"ms/step={float(r['TotalDurationNs']) / nsteps / 1e6:.3f}")
