"""Kernel-boundary gaps of the bench step from a rocprofv3 kernel trace: per step (delimited by the pack
launch that opens it), the idle time of the union of both streams and the launch stream's kernel-to-kernel
gaps grouped by (previous -> next) kernel.

    python tools/gaps.py gpurun_out/prof_<tag> [--steps 2] [--top 12]
"""
import argparse
import collections
import csv
import glob
import os


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].split("<")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    f = a.path if a.path.endswith(".csv") else glob.glob(os.path.join(a.path, "**", "*kernel_trace.csv"),
                                                          recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "pack_many" in r["Kernel_Name"]]
    steps = list(zip(marks, marks[1:]))[-a.steps - 1:-1] or list(zip(marks, marks[1:]))
    for s0, s1 in steps:
        seg = rows[s0:s1 + 1]
        span = int(seg[-1]["Start_Timestamp"]) - int(seg[0]["Start_Timestamp"])
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in seg[:-1])
        busy, cs, ce = 0, None, None
        for s, e in iv:
            if ce is None or s > ce:
                if ce is not None:
                    busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        main = [r for r in seg if r["Stream_Id"] == seg[0]["Stream_Id"]]
        agg = collections.defaultdict(list)
        for p, r in zip(main, main[1:]):
            agg[short(p["Kernel_Name"]) + " -> " + short(r["Kernel_Name"])].append(
                (int(r["Start_Timestamp"]) - int(p["End_Timestamp"])) / 1e3)
        tot = sum(max(0.0, g) for v in agg.values() for g in v)
        print(f"step: span {span / 1e3:.1f} us, union idle {(span - busy) / 1e3:.1f} us, launch-stream gaps "
              f"{tot:.1f} us over {sum(len(v) for v in agg.values())} boundaries")
        for k, v in sorted(agg.items(), key=lambda x: -sum(x[1]))[:a.top]:
            print(f"   {sum(v):7.1f} us  n={len(v):3d} avg {sum(v) / len(v):5.1f}  {k}")


if __name__ == "__main__":
    main()
