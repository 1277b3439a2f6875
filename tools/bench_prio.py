"""bench.py with HIP stream priorities set, for a scheduling A/B on the GPU box:

    python tools/bench_prio.py main|side|none -- [bench.py arguments]

main: the step runs on a high-priority stream (the weight-gradient side stream stays normal);
side: the side stream is high priority.  Runs bench.py in this process (runpy), nothing else."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]

import torch  # noqa: E402

from eunet import engine  # noqa: E402

args = sys.argv[1:]
sep = args.index("--") if "--" in args else len(args)
mode = args[0] if sep > 0 else "none"
lo, hi = torch.cuda.Stream.priority_range()  # (least, greatest)
print(f"bench_prio: mode {mode}, priority range least {lo} greatest {hi}", file=sys.stderr)
if mode == "main":
    torch.cuda.set_stream(torch.cuda.Stream(device=0, priority=hi))
elif mode == "side":
    engine._SIDE[0] = torch.cuda.Stream(device=0, priority=hi)
elif mode != "none":
    raise SystemExit("mode: main | side | none")
sys.argv = [os.path.join(ROOT, "bench.py")] + args[sep + 1:]
runpy.run_path(sys.argv[0], run_name="__main__")
