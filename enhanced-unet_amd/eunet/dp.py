"""Data-parallel training: one process per GPU, bucketed gradient all-reduce.

The reference is single-process (no torch.distributed anywhere);
the build shards the minibatch across ranks (weak scaling: each rank trains
its own B samples) and has exactly one exchange step per iteration: the
gradient all-reduce (backend 'nccl' == RCCL over xGMI on MI355X; 'gloo' for
the CPU tests).  BatchNorm stays per replica, as under DDP without SyncBN;
running statistics are broadcast from rank 0 before each forward
(DDP broadcast_buffers semantics) as ONE collective on a persistent flat buffer: at
construction every floating-point module buffer is re-pointed at a slice of that buffer
(the HIP kernels update running statistics through those views), so the per-step sync
is a single async broadcast with no host-side concatenation or scatter copies.

Overlap: parameter gradients are written by the HIP backward straight into a
flat fp32 buffer laid out in backward-production order (head, dec1, dec2 ...
enc1).  The engine reports each finished block to the sink; a bucket whose
parameters are all written is all-reduced asynchronously right away, so RCCL
runs under the remaining backward kernels.  Buckets default to 8 MiB: few,
large collectives for the point-to-point xGMI mesh.
"""
from __future__ import annotations

from typing import Dict, List

import torch
import torch.distributed as dist

from .engine import BLOCKS


def backward_order(model) -> List[str]:
    custom = getattr(model, "backward_param_order", None)
    if custom is not None and custom() is not None:  # dual-branch model (eunet.dual)
        return custom()
    names = [n for n, _ in model.named_parameters()]
    order = [n for n in names if n.startswith("enhance.")]
    order += [n for n in names if n.startswith("model.dec1.")]
    for blk in ("dec2", "dec3", "dec4", "enc4", "enc3", "enc2", "enc1"):
        pre = f"model.{blk}."
        blk_names = [n for n in names if n.startswith(pre)]
        # conv b / BN b finish first, then BN a / conv a (engine._block_bwd order)
        blk_names.sort(key=lambda n: {"4": 0, "3": 1, "1": 2, "0": 3}[n[len(pre)]])
        order += blk_names
    assert sorted(order) == sorted(names), "backward order must cover every parameter"
    return order


class BucketSink:
    def __init__(self, dp: "DataParallel"):
        self.dp = dp
        self.done = set()
        self.launched = [False] * len(dp.buckets)
        self.works = []
        self.grads: Dict[str, torch.Tensor] = {}
        self.last_issue = None  # DataParallel.timing: event at the last bucket's issue (on the issuing stream)

    def slot(self, name, shape):
        off, numel = self.dp.offsets[name]
        t = self.dp.flat[off:off + numel].view(shape)
        self.grads[name] = t
        return t

    def ready(self, names):
        self.done.update(names)
        for i, (lo, hi, members) in enumerate(self.dp.buckets):
            if not self.launched[i] and all(m in self.done for m in members):
                self.launched[i] = True
                if self.dp.timing and all(self.launched):
                    self.last_issue = torch.cuda.Event(enable_timing=True)
                    self.last_issue.record()
                self.works.append(dist.all_reduce(self.dp.flat[lo:hi], group=self.dp.group, async_op=True))

    def finish(self):
        self.ready([])  # launch anything still pending
        for i, lo_hi in enumerate(self.dp.buckets):
            if not self.launched[i]:
                raise RuntimeError(f"bucket {i} never completed: missing gradients")
        e0 = None
        if self.dp.timing:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()  # the launch stream is done with the backward's own kernels here
        for w in self.works:
            w.wait()
        self.dp.flat.mul_(1.0 / self.dp.world)
        if e0 is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self.dp._timings.append((self.last_issue, e0, e1))
        return self.grads


class DataParallel:
    def __init__(self, model, bucket_mb: float = 8.0, group=None, broadcast_buffers: bool = True):
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed must be initialised (one process per GPU)")
        self.model = model
        self.group = group
        self.world = dist.get_world_size(group)
        self.broadcast_buffers = broadcast_buffers
        params = dict(model.named_parameters())
        self.order = backward_order(model)
        dev = next(model.parameters()).device
        total = sum(params[n].numel() for n in self.order)
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
        self.offsets = {}
        self.buckets = []
        cap = max(1, int(bucket_mb * (1 << 20) / 4))
        off, lo, members = 0, 0, []
        for n in self.order:
            k = params[n].numel()
            self.offsets[n] = (off, k)
            members.append(n)
            off += k
            if off - lo >= cap:
                self.buckets.append((lo, off, members))
                lo, members = off, []
        if members:
            self.buckets.append((lo, off, members))
        with torch.no_grad():  # identical initial replicas
            for n in self.order:
                dist.broadcast(params[n].data, src=0, group=group)
        self.flat_buffers, self._buffer_views = self._flatten_buffers(model)
        self._sync_buffers()
        # timing (bench.py): per step, HIP events at the last bucket's issue and around the sink's final wait
        self.timing = False
        self._timings = []
        model.grad_sink_factory = lambda: BucketSink(self)

    def start_timing(self):
        self._timings = []
        self.timing = True

    def stop_timing(self):
        """Per-step means over the steps since start_timing(): exposed_ms = the launch stream's time from the
        end of its backward kernels to the gradients being reduced and scaled (waiting for the side stream's
        last weight gradients, the outstanding bucket all-reduces and the 1/N scale: the communication the
        backward did not hide); last_bucket_ms = the last bucket from its issue to that point (its
        all-reduce and anything queued before it)."""
        self.timing = False
        torch.cuda.synchronize()
        ts, self._timings = self._timings, []
        if not ts:
            return {"buckets": len(self.buckets), "steps": 0}
        exposed = sum(e0.elapsed_time(e1) for _, e0, e1 in ts) / len(ts)
        last = [li.elapsed_time(e1) for li, _, e1 in ts if li is not None]
        return {"buckets": len(self.buckets), "bucket_mb": round(self.flat.numel() * 4 / 2 ** 20, 2), "steps": len(ts),
                "exposed_comm_ms": round(exposed, 4),
                "last_bucket_ms": round(sum(last) / len(last), 4) if last else None}

    @staticmethod
    def _flatten_buffers(model):
        """Re-point every floating-point buffer (BN running_mean / running_var) at a slice of one
        flat tensor; returns (flat, [(module, name, data_ptr)]) ((None, []) without such buffers)."""
        entries = [(mod, name, b) for mod in model.modules() for name, b in mod._buffers.items()
                   if b is not None and b.dtype.is_floating_point]
        if not entries:
            return None, []
        dt, dev = entries[0][2].dtype, entries[0][2].device
        if any(b.dtype != dt or b.device != dev for _, _, b in entries):
            raise RuntimeError("DataParallel: floating-point buffers must share one dtype and device")
        flat = torch.empty(sum(b.numel() for _, _, b in entries), dtype=dt, device=dev)
        off, views = 0, []
        with torch.no_grad():
            for mod, name, b in entries:
                view = flat[off:off + b.numel()].view_as(b)
                view.copy_(b)
                mod._buffers[name] = view
                views.append((mod, name, view.data_ptr()))
                off += b.numel()
        return flat, views

    def _check_buffer_views(self):
        """The broadcast updates flat_buffers; a module._apply (model.to / .float / .cuda ...) after
        construction replaces the registered buffers with tensors the broadcast no longer reaches,
        and the replicas' running statistics would drift apart silently.  Raise instead."""
        for mod, name, ptr in self._buffer_views:
            b = mod._buffers.get(name)
            if b is None or b.data_ptr() != ptr:
                raise RuntimeError(f"DataParallel: buffer {type(mod).__name__}.{name} no longer aliases the flat "
                                   "broadcast buffer (the model was moved or cast after DataParallel was built); "
                                   "construct DataParallel after the last .to() / dtype change")

    def _sync_buffers(self):
        if self.flat_buffers is None or self.world == 1:
            return
        dist.broadcast(self.flat_buffers, src=0, group=self.group)  # nccl: stream-ordered, no host wait

    def before_forward(self):
        if self.broadcast_buffers:
            self._check_buffer_views()
            self._sync_buffers()

    def after_backward(self):
        pass  # the sink already waited for every bucket

    def allreduce_grads_(self, params=None):
        """Non-overlapped path for models without the HIP engine (used by tests)."""
        ps = [p for p in (params or self.model.parameters()) if p.grad is not None]
        flat = torch.cat([p.grad.reshape(-1) for p in ps])
        dist.all_reduce(flat, group=self.group)
        flat.mul_(1.0 / self.world)
        off = 0
        for p in ps:
            p.grad.copy_(flat[off:off + p.numel()].view_as(p.grad))
            off += p.numel()


__all__ = ["DataParallel", "BucketSink", "backward_order", "BLOCKS"]
