"""Print the top kernels of a rocprofv3 kernel_stats.csv per step: kstats.py FILE STEPS [N]."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 20
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print(f"{float(r['TotalDurationNs']) / steps / 1e6:8.3f} ms/step {int(r['Calls']):5d} "
          f"{float(r['AverageNs']) / 1e3:9.1f} us  {r['Name'][:100]}")
print(f"total {sum(float(r['TotalDurationNs']) for r in rows) / steps / 1e6:.3f} ms/step")
