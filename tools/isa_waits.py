"""Find kernels whose global / buffer loads wait for themselves: compile csrc/*.hip to gfx950 assembly and
count, per kernel, the loads followed within three instructions by `s_waitcnt vmcnt(0)`.  A bounds-checked
load with a dependent instruction inside its branch (a conversion, a scale) or a load the compiler sank into
the branch of its select is issued and waited for one at a time; prefetches written that way prefetch nothing.

    python tools/isa_waits.py [--min 3] [csrc/head.hip ...]

Prints: file, kernel, loads, loads waited for immediately, and the instruction after each such wait (the
dependent op that forced it).  CPU only (hipcc --cuda-device-only -S)."""
import argparse
import collections
import glob
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "enhanced-unet_amd", "csrc")


def scan(asm_lines):
    cur, stats = None, {}
    for i, line in enumerate(asm_lines):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur = m.group(1)
            stats[cur] = [0, 0, collections.Counter()]
            continue
        if cur and ("global_load" in line or "buffer_load" in line):
            stats[cur][0] += 1
            for j in range(i + 1, min(i + 4, len(asm_lines))):
                if "s_waitcnt vmcnt(0)" in asm_lines[j]:
                    stats[cur][1] += 1
                    nxt = asm_lines[j + 1].split() if j + 1 < len(asm_lines) else ["?"]
                    stats[cur][2][nxt[0] if nxt else "?"] += 1
                    break
                if "global_load" in asm_lines[j] or "buffer_load" in asm_lines[j]:
                    break
    return stats


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="*")
    ap.add_argument("--min", type=int, default=3, help="report kernels with at least this many waited loads")
    a = ap.parse_args()
    files = a.files or sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    with tempfile.TemporaryDirectory() as td:
        for f in files:
            out = os.path.join(td, os.path.basename(f) + ".s")
            subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I", os.path.join(ROOT, "include"),
                            "-I", CSRC, "-S", "--cuda-device-only", f, "-o", out], check=True, capture_output=True)
            for k, (n, w, nxt) in scan(open(out).read().split("\n")).items():
                if w >= a.min:
                    print(f"{os.path.basename(f)}  {k[:90]}  loads {n}  waited {w}  then {dict(nxt.most_common(3))}")


if __name__ == "__main__":
    main()
