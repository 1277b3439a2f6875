"""clip_grad_norm_ + AdamW as one native step (csrc/optim.hip) on a torch.optim.AdamW's own state.

Reference: train_eval.py:341-343 -- torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=1.0)
then optimizer.step() of the AdamW built at :120 (betas (0.9, 0.999), weight_decay 1e-4, the lr the
schedulers set in param_groups).  The optimizer object stays torch's: its param_groups carry the
learning rate, its state holds exp_avg / exp_avg_sq / step exactly as torch's fused AdamW lays them
out (fp32 step counter on the device), so state_dict / load_state_dict / the LR schedulers and a
later torch optimizer.step() all see the same state.  Three launches replace PyTorch's ~14 (per-
tensor norms, their norm, four elementwise kernels for the clip coefficient, the in-place scale, the
step counters, two fused-AdamW launches); p.grad is left clipped, as clip_grad_norm_ leaves it.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import call

KARG_MAX = 256  # EUNET_OPT_KARG_MAX


def supported(optimizer) -> bool:
    """One fused (or capturable) AdamW parameter group of contiguous fp32 CUDA tensors, no amsgrad /
    maximize.  A plain foreach AdamW (the reference's optim.AdamW(...), or the Trainer's fallback) keeps
    its step counters as CPU tensors, which the kernels cannot increment: torch's own step runs there."""
    if type(optimizer) is not torch.optim.AdamW or len(optimizer.param_groups) != 1:
        return False
    g = optimizer.param_groups[0]
    if g.get("amsgrad") or g.get("maximize") or g.get("differentiable"):
        return False
    if not (g.get("fused") or g.get("capturable")):
        return False
    return all(p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() for p in g["params"])


class ClipAdamW:
    """step(max_norm) == clip_grad_norm_(params, max_norm) + optimizer.step() for an AdamW that
    supported() accepts; returns the total gradient norm (a device scalar, as clip_grad_norm_)."""

    def __init__(self, optimizer):
        if not supported(optimizer):
            raise ValueError("ClipAdamW: needs one AdamW param group of contiguous fp32 CUDA tensors")
        self.optimizer = optimizer
        self._tables = {}  # key -> (device table, nblocks), most recently used last

    def _state(self, p):
        st = self.optimizer.state[p]
        if len(st) == 0:  # torch's fused AdamW initialisation (_init_group)
            st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            return st
        # state from torch's own step or load_state_dict: every tensor the kernels read or write must be
        # contiguous fp32 on the parameter's device (a CPU step counter would be a host address there)
        if st["step"].device != p.device or st["step"].dtype != torch.float32:
            st["step"] = st["step"].to(device=p.device, dtype=torch.float32)
        for k in ("exp_avg", "exp_avg_sq"):
            t = st[k]
            if t.device != p.device or t.dtype != torch.float32 or not t.is_contiguous() or t.shape != p.shape:
                raise ValueError(f"ClipAdamW: AdamW state {k!r} must be a contiguous fp32 tensor shaped and "
                                 f"placed like its parameter")
        return st

    def step(self, max_norm: float):
        g = self.optimizer.param_groups[0]
        ps = [p for p in g["params"] if p.grad is not None]  # torch skips parameters without a gradient
        if not ps:
            return torch.zeros((), device=g["params"][0].device)
        dev = ps[0].device
        rows, grads = [], []
        for p in ps:
            if p.grad.dtype != torch.float32 or not p.grad.is_contiguous():
                raise ValueError("ClipAdamW: gradients must be contiguous fp32")
            st = self._state(p)
            grads.append(p.grad.data_ptr())
            rows.append((p.data_ptr(), grads[-1], st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                         st["step"].data_ptr(), p.numel()))
        # the gradients travel as a kernel argument (<= KARG_MAX tensors): the table's key leaves them out
        karg = len(rows) <= KARG_MAX
        key = tuple(r[:1] + r[2:] for r in rows) if karg else tuple(rows)
        hit = self._tables.pop(key, None)
        if hit is None:  # new gradient storage (the caching allocator cycles through a few sets)
            n = len(rows)
            descs = (_lib.OptTensor * n)(*[_lib.OptTensor(*r) for r in rows])
            host = torch.empty(n * 7, dtype=torch.int64).pin_memory()
            nb = ctypes.c_int()
            call("eunet_opt_table", ctypes.cast(descs, ctypes.c_void_p), n, host.data_ptr(), ctypes.byref(nb))
            hit = (host.to(dev, non_blocking=True), nb.value)
            while len(self._tables) >= 4:
                self._tables.pop(next(iter(self._tables)))
        self._tables[key] = hit
        table, nblocks = hit
        partial = torch.empty(nblocks, dtype=torch.float64, device=dev)
        coef = torch.empty(1, dtype=torch.float32, device=dev)
        norm = torch.empty((), dtype=torch.float32, device=dev)
        b1, b2 = g["betas"]
        gptr = (ctypes.c_void_p * len(grads))(*grads) if karg else None
        call("eunet_clip_adamw", table.data_ptr(), len(rows), nblocks, gptr, float(max_norm), float(g["lr"]),
             float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]), partial.data_ptr(), coef.data_ptr(),
             norm.data_ptr(), ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
        return norm
