"""Per-layer SQ counter ratios for the conv3x3 kernels, from rocprofv3 --pmc passes over
tools/conv_bench.py (tools/gpu_sq_layers.sh).

    python tools/sq_layers.py <pmc_dir> [<pmc_dir> ...] > summary.txt

conv_bench launches, per layer in its fixed order, (1 + reps) forwards, (1 + reps) data gradients,
(1 + reps) weight gradients and (1 + reps) split reductions; the i-th launch of a kernel therefore
belongs to layer i // (1 + reps).  Counters of one dispatch from several passes are joined by
(kernel, ordinal).  SQ_* quad-cycle units cancel in the ratios:
  wait    = SQ_WAIT_ANY / SQ_WAVE_CYCLES        (wave parked: s_waitcnt / barrier)
  issue   = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   (ready but not issued: pipe busy / dependency)
  active  = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  ldsw    = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES   (LDS issue stall, part of issue)
  vmem    = SQ_ACTIVE_INST_VMEM / SQ_WAVE_CYCLES
  valu    = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
  lds     = SQ_ACTIVE_INST_LDS / SQ_WAVE_CYCLES
  bank    = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  mfma    = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 4 SIMDs x 256 CUs)
  coexec  = SQ_VALU_MFMA_COEXEC_CYCLES / SQ_VALU_MFMA_BUSY_CYCLES
  valu/mfma, lds/mfma = SQ_INSTS_VALU / SQ_INSTS_MFMA, SQ_INSTS_LDS / SQ_INSTS_MFMA (issued per MFMA)
"""
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_bench import layers  # noqa: E402
from pmc_summary import short  # noqa: E402

KINDS = {"conv3x3_fwd_kernel": "fwd", "conv3x3_fwd_kernel.dgrad": "dgrad", "conv3x3_wgrad_bf16_kernel": "wgrad",
         "conv3x3_wgrad_f32_kernel": "wgrad"}


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(lambda: defaultdict(float))  # dispatch id -> counter -> value
    names = {}
    for r in csv.DictReader(open(f[0])):
        did = int(r["Dispatch_Id"])
        per[did][r["Counter_Name"]] += float(r["Counter_Value"])
        per[did]["us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        names[did] = short(r["Kernel_Name"])
    # ordinal of each dispatch among the launches of its kernel
    seen = defaultdict(int)
    out = {}
    for did in sorted(per):
        k = names[did]
        out[(k, seen[k])] = per[did]
        seen[k] += 1
    return out


def main():
    reps = int(os.environ.get("SQ_REPS", "1"))
    base = int(os.environ.get("SQ_BASE", "64"))
    merged = defaultdict(dict)
    for d in sys.argv[1:]:
        for key, c in load(d).items():
            merged[key].update(c)
    if os.environ.get("SQ_BY_KERNEL") == "1":  # any program: one row per kernel name, all launches summed
        agg = defaultdict(lambda: defaultdict(float))
        for (k, i), c in merged.items():
            for n, v in c.items():
                agg[k][n] += v
        rows = sorted(((k, "all", c) for k, c in agg.items()), key=lambda r: -r[2].get("SQ_WAVE_CYCLES", 0.0))[:24]
        return emit(rows, 30)
    lay = [n for n, *_ in layers(base)]
    rows = []
    for (k, i), c in merged.items():
        kind = KINDS.get(k)
        if kind is None or i % (1 + reps) == 0:  # skip the warm-up launch
            continue
        li = i // (1 + reps)
        if li >= len(lay):
            continue
        rows.append((lay[li], kind, c))
    order = {n: j for j, n in enumerate(lay)}
    rows.sort(key=lambda r: (["fwd", "dgrad", "wgrad"].index(r[1]), order[r[0]]))
    emit(rows, 8)


def emit(rows, w):
    def rat(c, a, b, s=1.0):
        return c[a] / (c[b] * s) if c.get(a) is not None and c.get(b) else float("nan")

    hdr = ("layer", "pass", "us", "wait", "issue", "active", "ldsw", "vmem", "valu", "lds", "bank", "mfma", "coexec",
           "valu/mf", "lds/mf")
    print("%-*s %-6s" % (w, hdr[0], hdr[1]) + "".join("%8s" % h for h in hdr[2:]))
    for name, kind, c in rows:
        vals = [c.get("us", float("nan")), rat(c, "SQ_WAIT_ANY", "SQ_WAVE_CYCLES"), rat(c, "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES"),
                rat(c, "SQ_ACTIVE_INST_ANY", "SQ_WAVE_CYCLES"), rat(c, "SQ_WAIT_INST_LDS", "SQ_WAVE_CYCLES"),
                rat(c, "SQ_ACTIVE_INST_VMEM", "SQ_WAVE_CYCLES"), rat(c, "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES"),
                rat(c, "SQ_ACTIVE_INST_LDS", "SQ_WAVE_CYCLES"), rat(c, "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"),
                rat(c, "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", 4 * 256 / 8),
                rat(c, "SQ_VALU_MFMA_COEXEC_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES"),
                rat(c, "SQ_INSTS_VALU", "SQ_INSTS_MFMA"), rat(c, "SQ_INSTS_LDS", "SQ_INSTS_MFMA")]
        print("%-*s %-6s" % (w, name[:w], kind) + "".join("%8.3f" % v for v in vals))


if __name__ == "__main__":
    main()
