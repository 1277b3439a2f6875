"""Aggregate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per kernel (per launch means).

    python tools/pmc_summary.py <fetch_dir> <write_dir> [base,size,batch,dtype] > summary.json

FETCH_SIZE/WRITE_SIZE are reported by rocprofv3 in KiB.  gfx950 correction
(MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts exactly half the bytes of
wide (16 B/lane) coalesced reads -> doubled here; WRITE_SIZE is exact for
16 B/lane stores.  Our kernels' bulk traffic is 16 B/lane loads and stores.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(\w+_kernel|colsum_stage\d|\w+Kernel|multi_tensor_apply_kernel|copyBuffer\w*)", name)
    k = m.group(1) if m else name[:60]
    if k == "conv3x3_fwd_kernel" and re.search(r"conv3x3_fwd_kernel<[^,>]*, ?true", name):
        k += ".dgrad"  # the data-gradient launches of the same kernel (template tag DG)
    return k


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(list)
    rows = csv.DictReader(open(f[0]))
    if "Counter_Name" not in (rows.fieldnames or []):
        raise SystemExit(f"unexpected columns in {f[0]}: {rows.fieldnames}")
    for r in rows:
        if r.get("Counter_Name") != counter:
            continue
        per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return per


def main():
    fd, wd = sys.argv[1], sys.argv[2]
    fe, wr = load(fd, "FETCH_SIZE"), load(wd, "WRITE_SIZE")
    out = {}
    for k in sorted(set(fe) | set(wr)):
        f = fe.get(k, [])
        w = wr.get(k, [])
        fb = 2.0 * 1024.0 * sum(f) / len(f) if f else None
        wb = 1024.0 * sum(w) / len(w) if w else None
        out[k] = {"launches": max(len(f), len(w)), "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                  "hbm_bytes_per_launch": (fb or 0.0) + (wb or 0.0)}
    wl = [int(x) if x.isdigit() else x for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else None
    json.dump({"workload": wl, "correction": "FETCH_SIZE(KiB)*1024*2 + WRITE_SIZE(KiB)*1024", "kernels": out},
              sys.stdout, indent=1)


if __name__ == "__main__":
    main()
