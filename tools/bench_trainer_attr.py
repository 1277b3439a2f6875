"""bench.py with Trainer instance attributes overridden, for A/Bs on the GPU box:

    python tools/bench_trainer_attr.py native_clip_adamw=0 [attr=value ...] -- [bench.py arguments]

Values are Python literals.  Runs bench.py in this process (runpy), nothing else."""
import ast
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]

from eunet import train_eval  # noqa: E402

args = sys.argv[1:]
sep = args.index("--") if "--" in args else len(args)
over = {}
for kv in args[:sep]:
    k, v = kv.split("=", 1)
    over[k] = ast.literal_eval(v)
_init = train_eval.Trainer.__init__


def _patched(self, *a, **kw):
    _init(self, *a, **kw)
    for k, v in over.items():
        if not hasattr(self, k):
            raise SystemExit(f"unknown Trainer attribute {k}")
        setattr(self, k, type(getattr(self, k))(v))


train_eval.Trainer.__init__ = _patched
sys.argv = [os.path.join(ROOT, "bench.py")] + args[sep + 1:]
runpy.run_path(sys.argv[0], run_name="__main__")
