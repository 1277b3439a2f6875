"""Per-kernel SQ counter ratios from tools/gpu_pmc_sq.sh (SQ_* quad-cycle units cancel in ratios).
    python tools/sq_summary.py <pmc_dir>
wait = SQ_WAIT_ANY / SQ_WAVE_CYCLES, lds_wait = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES,
valu = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES, lds = SQ_ACTIVE_INST_LDS / SQ_WAVE_CYCLES,
bank = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE."""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def main():
    f = glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True)[0]
    agg = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(f)):
        agg[short(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    rows = []
    for k, c in agg.items():
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        if wc <= 0:
            continue
        rows.append((wc, k, c["SQ_WAIT_ANY"] / wc, c["SQ_WAIT_INST_LDS"] / wc, c["SQ_ACTIVE_INST_VALU"] / wc,
                     c["SQ_ACTIVE_INST_LDS"] / wc,
                     c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"] if c.get("SQ_LDS_IDX_ACTIVE") else 0.0))
    rows.sort(reverse=True)
    print(f"{'kernel':34s} {'wave_cyc':>10s} {'wait':>6s} {'ldswait':>7s} {'valu':>6s} {'lds':>6s} {'bank':>6s}")
    for wc, k, w, lw, v, l, b in rows[:24]:
        print(f"{k:34s} {wc:10.3g} {w:6.3f} {lw:7.3f} {v:6.3f} {l:6.3f} {b:6.3f}")


if __name__ == "__main__":
    main()
