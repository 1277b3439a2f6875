"""bench.py with UNetEngine class attributes overridden, for schedule A/Bs on the GPU box:

    python tools/bench_knob.py wg3_early_last=0 [knob=value ...] -- [bench.py arguments]

Values are Python literals (0/1/True/False).  Runs bench.py in this process (runpy), nothing else."""
import ast
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]

from eunet import engine  # noqa: E402

args = sys.argv[1:]
sep = args.index("--") if "--" in args else len(args)
for kv in args[:sep]:
    k, v = kv.split("=", 1)
    if not hasattr(engine.UNetEngine, k):
        raise SystemExit(f"unknown UNetEngine attribute {k}")
    setattr(engine.UNetEngine, k, type(getattr(engine.UNetEngine, k))(ast.literal_eval(v)))
sys.argv = [os.path.join(ROOT, "bench.py")] + args[sep + 1:]
runpy.run_path(sys.argv[0], run_name="__main__")
