"""Live per-kernel timing with HIP events on the launch stream (used by bench.py).

When a KernelTimer is active, ops.* launches of the named kernel families are
bracketed by events recorded on torch's current stream -- the same stream the
C-ABI launches on -- and credited with their algorithmic FLOPs / bytes.
"""
from __future__ import annotations

import os

import torch

_active = None


class KernelTimer:
    def __init__(self):
        self.records = {}  # family -> list of (ev0, ev1, flops, bytes)

    def __enter__(self):
        global _active
        _active = self
        self.origin = torch.cuda.Event(enable_timing=True)  # common time origin for interval unions
        self.origin.record()
        return self

    def __exit__(self, *exc):
        global _active
        _active = None

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for fam, recs in self.records.items():
            ms = sum(a.elapsed_time(b) for a, b, _, _ in recs)
            out[fam] = dict(launches=len(recs), ms=ms, flops=sum(r[2] for r in recs),
                            bytes=sum(r[3] for r in recs))
        return out

    def union_ms(self, families):
        """Wall time (ms) during which at least one launch of `families` ran: the union of their
        event intervals across streams (launches of one family on two streams overlap, so the
        summed spans of summary() count shared time twice)."""
        torch.cuda.synchronize()
        return _union([(self.origin.elapsed_time(a), self.origin.elapsed_time(b))
                       for fam in families for a, b, _, _ in self.records.get(fam, ())])


def _union(iv):
    tot, cur0, cur1 = 0.0, None, None
    for a, b in sorted(iv):
        if cur1 is None or a > cur1:
            if cur1 is not None:
                tot += cur1 - cur0
            cur0, cur1 = a, b
        else:
            cur1 = max(cur1, b)
    if cur1 is not None:
        tot += cur1 - cur0
    return tot


class BusyTimer:
    """Every launching C-ABI call (eunet._lib.call) bracketed by events on torch's current stream while
    active: busy_ms() = the union of all those intervals over both streams, i.e. the time some library
    kernel ran.  Kernels PyTorch launches itself (a few copies / fills per step) count as idle.  The
    events cost GPU time of their own, so bench.py runs this in an extra, untimed pass."""

    def __init__(self):
        self.iv = []

    def __enter__(self):
        from . import _lib
        self.origin = torch.cuda.Event(enable_timing=True)
        self.origin.record()
        _lib.BUSY_HOOK = self
        return self

    def __exit__(self, *exc):
        from . import _lib
        _lib.BUSY_HOOK = None
        self.last = torch.cuda.Event(enable_timing=True)
        self.last.record()

    def begin(self):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def end(self, e0):
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        self.iv.append((e0, e1))

    def busy_ms(self):
        torch.cuda.synchronize()
        return _union([(self.origin.elapsed_time(a), self.origin.elapsed_time(b)) for a, b in self.iv])

    def span_ms(self):
        torch.cuda.synchronize()
        return self.origin.elapsed_time(self.last)


_OFF = os.environ.get("EUNET_KPROF", "1") == "0"  # diagnostic: measure the event overhead itself
_scope = None  # while set: every timed conv3x3 launch is credited to this family too (scope())


class scope:
    """Credit every conv3x3 launch timed inside the block to `family` as well (None: no-op).  The engine
    wraps the encoder blocks' forward and backward in it, so bench.py can report the north-star's "3x3
    encoder convs" over forward, data and weight gradients (the weight gradients issued on the side stream
    from inside the block included)."""
    __slots__ = ("family", "prev")

    def __init__(self, family):
        self.family = family

    def __enter__(self):
        global _scope
        self.prev = _scope
        if self.family is not None:
            _scope = self.family
        return self

    def __exit__(self, *exc):
        global _scope
        _scope = self.prev
        return False


def timed(family: str, flops: float, nbytes: float = 0.0, sub: str | None = None):
    """Context manager used around a launch; no-op when no timer is active.
    sub: a second family the same events are credited to (a subset of `family`)."""
    t = _active
    if t is None or _OFF:
        return _Null
    return _Rec(t, family, flops, nbytes, sub, _scope if family.startswith("conv3x3") else None)


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


_Null = _NullCtx()


class _Rec:
    __slots__ = ("t", "fam", "flops", "nbytes", "e0", "sub", "scope")

    def __init__(self, t, fam, flops, nbytes, sub=None, scope=None):
        self.t, self.fam, self.flops, self.nbytes, self.sub, self.scope = t, fam, flops, nbytes, sub, scope

    def __enter__(self):
        self.e0 = torch.cuda.Event(enable_timing=True)
        self.e0.record()
        return self

    def __exit__(self, *exc):
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        self.t.records.setdefault(self.fam, []).append((self.e0, e1, self.flops, self.nbytes))
        if self.sub is not None:
            self.t.records.setdefault(self.sub, []).append((self.e0, e1, self.flops, self.nbytes))
        if self.scope is not None:
            self.t.records.setdefault(self.scope, []).append((self.e0, e1, self.flops, self.nbytes))
        return False
