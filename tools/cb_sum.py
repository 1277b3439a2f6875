"""Summarise tools/conv_bench.py JSON lines from stdin: per-layer ms of one pass and the sum.
    python tools/conv_bench.py ... | python tools/cb_sum.py wgrad_ms"""
import json
import sys

key = sys.argv[1] if len(sys.argv) > 1 else "wgrad_ms"
rows = [json.loads(l) for l in sys.stdin if l.startswith('{"layer')]
print(" ".join(f"{d['layer']}={d[key]:.3f}" for d in rows), f"sum={sum(d[key] for d in rows):.3f}")
