"""Per-kernel MFMA-pipe utilisation and effective clock from one rocprofv3 --pmc pass of
SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE (tools/gpu_pmc_mfma.sh).

    python tools/mfma_summary.py <pmc_dir> > summary.json

Per dispatch (MI355X_MICROARCH.md, PMC units / DVFS notes):
  cycles      = GRBM_GUI_ACTIVE / 8            (rocprofv3 sums the 8 XCDs)
  clock_ghz   = cycles / dispatch duration
  mfma_busy   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles)
              (the counter is summed over SIMDs; 16 cycles per v_mfma_f32_16x16x32_bf16,
              so FLOPs / 1024 is the expected count for a pure 16x16x32 kernel)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402

SIMDS = 256 * 4


def main():
    f = glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {sys.argv[1]}")
    disp = defaultdict(dict)
    for r in csv.DictReader(open(f[0])):
        d = disp[r["Dispatch_Id"]]
        d["k"] = short(r["Kernel_Name"])
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    agg = defaultdict(lambda: {"launches": 0, "ns": 0, "busy": 0.0, "gui": 0.0})
    for d in disp.values():
        if "SQ_VALU_MFMA_BUSY_CYCLES" not in d or "GRBM_GUI_ACTIVE" not in d:
            continue
        a = agg[d["k"]]
        a["launches"] += 1
        a["ns"] += d["ns"]
        a["busy"] += d["SQ_VALU_MFMA_BUSY_CYCLES"]
        a["gui"] += d["GRBM_GUI_ACTIVE"]
    out = {}
    for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["busy"]):
        cyc = a["gui"] / 8.0
        out[k] = {"launches": a["launches"], "us_per_launch": a["ns"] / a["launches"] / 1e3,
                  "clock_ghz": cyc / a["ns"] if a["ns"] else None,
                  "mfma_busy_cycles_per_launch": a["busy"] / a["launches"],
                  "mfma_busy_frac": a["busy"] / (SIMDS * cyc) if cyc else None}
    json.dump({"counters": ["SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"], "simds": SIMDS, "kernels": out},
              sys.stdout, indent=1)


if __name__ == "__main__":
    main()
