"""Per-kernel ms/step side by side from several rocprofv3 kernel_stats.csv files (same STEPS each):
    python tools/cmp_kstats.py STEPS a.csv b.csv ..."""
import csv
import re
import sys

steps = float(sys.argv[1])
tabs = []
for f in sys.argv[2:]:
    t = {}
    for r in csv.DictReader(open(f)):
        m = re.search(r"::([A-Za-z0-9_]+(<[^(]*>)?)\(", r["Name"])
        k = (m.group(1) if m else r["Name"][:50])[:70]
        t[k] = t.get(k, 0.0) + float(r["TotalDurationNs"]) / steps / 1e6
    tabs.append(t)
keys = sorted(set().union(*tabs), key=lambda k: -max(t.get(k, 0.0) for t in tabs))
for k in keys[:30]:
    print(" ".join(f"{t.get(k, 0.0):8.3f}" for t in tabs), " ", k)
print(" ".join(f"{sum(t.values()):8.3f}" for t in tabs), "   total")
