"""Timeline of one steady training step from a rocprofv3 kernel_trace.csv: every launch with its
stream, start offset and duration, and which other-stream launch it overlapped.  Diagnostic only.

    python tools/trace_steps.py gpurun_out/prof_X/run_kernel_trace.csv [step_from_end=3] [min_us=20]
"""
import csv
import re
import sys


def short(name):
    m = re.search(r"::([A-Za-z0-9_]+)(<[^(]*>)?\(", name)
    base = m.group(1) if m else name[:40]
    tmpl = m.group(2) or "" if m else ""
    if "conv3x3_fwd_kernel" in base:
        # conv3x3_fwd_kernel<T, DG, TO, BT, BNB, PF, CT>: DG = data gradient, BNB = fused BN-backward apply,
        # PF = LDS-DMA-staged untransformed forward, CT = half-width tail co-block
        args = [t.strip() for t in tmpl.strip("<>").split(",")]
        flag = lambda i: len(args) > i and args[i] in ("true", "1")  # noqa: E731
        base = ("dgrad" + ("_bnb" if flag(4) else "")) if flag(1) else ("fwd" + ("_pf" if flag(5) else ""))
        if flag(6):
            base += "_ct"
        return base
    return base.replace("_kernel", "")


def main():
    path = sys.argv[1]
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 20.0
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [int(r["Start_Timestamp"]) for r in rows if "pack_many" in r["Kernel_Name"]]
    a, b = starts[-back - 1], starts[-back]
    st = [r for r in rows if a <= int(r["Start_Timestamp"]) < b]
    streams = sorted({r["Stream_Id"] for r in st})
    busy = {s: 0 for s in streams}
    print(f"step {(b - a) / 1e3:.0f} us; streams {streams}")
    for r in st:
        s0, s1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        d = (s1 - s0) / 1e3
        busy[r["Stream_Id"]] += d
        if d < min_us:
            continue
        other = [short(o["Kernel_Name"]) for o in st if o["Stream_Id"] != r["Stream_Id"]
                 and int(o["Start_Timestamp"]) < s1 and int(o["End_Timestamp"]) > s0]
        ind = "    " * streams.index(r["Stream_Id"])
        print(f"{(s0 - a) / 1e3:8.0f} {ind}{short(r['Kernel_Name']):24s} {d:7.1f}  || {','.join(sorted(set(other)))}")
    print("busy per stream (us):", {k: round(v) for k, v in busy.items()})


if __name__ == "__main__":
    main()
