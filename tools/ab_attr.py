"""Run bench.py's main() with UNetEngine schedule attributes overridden (same-box A/B of engine
choices without environment knobs in the product):

    python tools/ab_attr.py fuse_bn_apply=0 wg3_late=1 -- --steps 30 --warmup 5 --no-cpu-baseline ...
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]

argv = sys.argv[1:]
sep = argv.index("--") if "--" in argv else len(argv)
sets, rest = argv[:sep], argv[sep + 1:]
from eunet import ops  # noqa: E402
from eunet.engine import UNetEngine  # noqa: E402
for kv in sets:
    k, v = kv.split("=")
    if k.startswith("ops."):  # module switches of eunet.ops (e.g. ops.USE_DISPATCHER=0)
        setattr(ops, k[4:], bool(int(v)))
    elif k.startswith("dual."):  # DualEngine attributes (e.g. dual.narrow_mfma=0)
        from eunet.dual import DualEngine
        setattr(DualEngine, k[5:], bool(int(v)))
    elif v.startswith("{"):  # a per-block knob: fuse_bn_apply={enc4,dec4}
        setattr(UNetEngine, k, frozenset(x for x in v.strip("{}").split(",") if x))
    else:
        setattr(UNetEngine, k, bool(int(v)))
import bench  # noqa: E402
sys.argv = ["bench.py"] + rest
bench.main()
