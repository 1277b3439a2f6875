"""bench.py's driver contract on the GPU box: `bench.py --gpus 2` starts two ranks by itself (the
driver's command shape), each timing the per-rank workload with max-over-ranks timing and rank 0 printing
one JSON line that reports the real process-group size (BASELINE configs[3]: train_eval.py:337-343 per
rank).  gloo carries the collectives so that two ranks can share the one GPU of the box."""
import json
import math
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*extra, env=None, timeout=240):
    e = dict(os.environ, **(env or {}))
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), *extra]
    return subprocess.run(cmd, cwd=ROOT, env=e, capture_output=True, text=True, timeout=timeout)


@pytest.mark.gpu
def test_bench_gpus2_runs_two_ranks():
    r = _bench("--gpus", "2", "--size", "256", "--batch", "1", "--steps", "2", "--warmup", "1",
               "--no-cpu-baseline", "--dice-size", "0", "--no-fp32-leg", env={"EUNET_DIST_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["world"]["size"] == 2 and d["world"]["backend"] == "gloo"
    assert d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 2
    assert d["steps"] == 2 and d["value"] > 0
    # value = images of all ranks / the max-over-ranks time
    assert abs(d["value"] - 2 * 1 * 2 / (d["ms_per_step"] * 2e-3)) / d["value"] < 1e-2
    # per rank: its own step time, the communication its backward left exposed, the bucket count
    pr = d["world"]["per_rank"]
    assert [r["rank"] for r in pr] == [0, 1], pr
    for r in pr:
        assert r["steps"] == 2 and r["buckets"] >= 1, r
        for k in ("ms_per_step", "exposed_comm_ms", "last_bucket_ms"):
            assert isinstance(r[k], float) and math.isfinite(r[k]) and r[k] >= 0.0, (k, r)
    assert max(r["ms_per_step"] for r in pr) <= d["ms_per_step"] * 1.01


def test_bench_rejects_world_size_mismatch():
    """Under a launcher whose WORLD_SIZE differs from --gpus, bench.py exits non-zero before any GPU
    work (CPU-only: the check precedes device selection)."""
    r = _bench("--gpus", "2", env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr
