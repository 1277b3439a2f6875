"""Host time of back-to-back Trainer.step calls without synchronisation, eager vs StepGraph replay,
at the reference's training tile (3-ch 640x480, batch 2, bf16): does a replay return while the
previous one still runs?  Diagnostic only.

    python tools/graph_probe.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "enhanced-unet_amd")]

import torch  # noqa: E402


def main():
    from eunet.models import get_model
    from eunet.train_eval import Trainer
    out = {}
    for graph in (False, True):
        torch.manual_seed(0)
        tr = Trainer(get_model("enhanced_unet", num_classes=3, dtype="bf16").to("cuda"), "cuda", "enhanced_unet")
        tr.step_graph = graph
        x = torch.rand(2, 3, 480, 640, device="cuda")
        m = torch.randint(0, 3, (2, 480, 640), device="cuda")
        for _ in range(4):
            tr.step(x, m, sync_loss=False)
        torch.cuda.synchronize()
        calls = []
        t0 = time.perf_counter()
        for _ in range(12):
            a = time.perf_counter()
            tr.step(x, m, sync_loss=False)
            calls.append(round((time.perf_counter() - a) * 1e3, 3))
        t_issue = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        # a host-side sleep between calls: does the device keep running the queued replays?
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(6):
            tr.step(x, m, sync_loss=False)
            time.sleep(0.004)
        torch.cuda.synchronize()
        t_sleep = (time.perf_counter() - t1) / 6
        out["graph" if graph else "eager"] = {"call_ms": calls, "issue_ms_total": round(t_issue * 1e3, 2),
                                              "wall_ms_total": round(t_all * 1e3, 2),
                                              "ms_per_step_with_4ms_host_gap": round(t_sleep * 1e3, 3)}
        print(json.dumps(out["graph" if graph else "eager"]), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
