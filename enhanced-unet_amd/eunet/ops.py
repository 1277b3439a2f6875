"""Thin torch-tensor wrappers over the C-ABI (one function per entry point).

Tensors are device memory only (torch is the allocator); every call is
enqueued on torch's current HIP stream.  Activations are NHWC tensors
[N, H, W, Ctot]; a channel slice is expressed by (coff, c).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib, kprof
from ._lib import Act, call, c_int, c_size_t

DTYPES = {torch.float32: _lib.EUNET_F32, torch.bfloat16: _lib.EUNET_BF16}

# ---- torch.ops.eunet.* ---------------------------------------------------------------------------
# The network's device ops are registered with PyTorch's dispatcher (library "eunet", CUDA key), so they
# appear as eunet::<op> in torch.profiler traces and go through dispatcher hooks.  A
# decorated function keeps its Python signature: its arguments are flattened into the op schema
# (an Act becomes (tensor, coff, c)), the dispatcher calls the CUDA impl, which rebuilds the Acts and
# runs the original body (one C-ABI call).  Cost ~2 us of dispatcher per call (USE_DISPATCHER = False
# calls the bodies directly; tools/ab_attr.py ops.USE_DISPATCHER=0).
USE_DISPATCHER = True
_LIB = torch.library.Library("eunet", "DEF")
DISPATCHED: dict = {}


def _dispatched(kinds: str, returns_tensor: bool = False):
    """kinds: one token per parameter -- A (Act), T (tensor), i (int), f (float), b (bool), d (torch dtype),
    s (str); A! / T! mark the arguments the op writes, a trailing ? an optional (None-able) argument."""
    import inspect
    import string

    ks = kinds.split()

    def deco(fn):
        sig = inspect.signature(fn)
        names = list(sig.parameters)
        if len(names) != len(ks):
            raise _lib.EunetError(f"_dispatched({fn.__name__}): {len(names)} parameters, {len(ks)} kinds")
        letters = iter(string.ascii_lowercase)
        parts = []
        for nm, k in zip(names, ks):
            q = "?" if k.endswith("?") else ""
            base = k.rstrip("?")
            w = base.endswith("!")
            base = base.rstrip("!")
            if base in ("A", "T"):
                ty = f"Tensor({next(letters)}!){q}" if w else f"Tensor{q}"
                parts += [f"{ty} {nm}"] + ([f"int {nm}_coff", f"int {nm}_c"] if base == "A" else [])
            else:
                parts.append({"i": "int", "f": "float", "b": "bool", "d": "ScalarType", "s": "str"}[base] + f"{q} {nm}")
        _LIB.define(f"{fn.__name__}({', '.join(parts)}) -> {'Tensor' if returns_tensor else '()'}")

        def impl(*flat):
            args, j = [], 0
            for k in ks:
                if k.startswith("A"):
                    t, coff, c = flat[j:j + 3]
                    j += 3
                    args.append(None if t is None else act(t, coff, c))
                else:
                    args.append(flat[j])
                    j += 1
            return fn(*args)

        _LIB.impl(fn.__name__, impl, "CUDA")
        _LIB.impl(fn.__name__, impl, "CPU")  # raises EunetError in _ptr / act: no CPU fallback
        op = getattr(torch.ops.eunet, fn.__name__)

        defaults = [p.default for p in sig.parameters.values()]
        index = {nm: i for i, nm in enumerate(names)}
        isact = [k.startswith("A") for k in ks]

        def wrapper(*args, **kwargs):
            if not USE_DISPATCHER:
                return fn(*args, **kwargs)
            vals = list(args) + defaults[len(args):]
            for nm, v in kwargs.items():
                vals[index[nm]] = v
            flat = []
            for a, v in zip(isact, vals):
                if not a:
                    flat.append(v)
                elif v is None:
                    flat += (None, 0, 0)
                else:
                    flat += (v._keep, v.coff, v.c)
            return op(*flat)

        wrapper.__name__, wrapper.__doc__, wrapper.__wrapped__ = fn.__name__, fn.__doc__, fn
        DISPATCHED[fn.__name__] = op
        return wrapper

    return deco


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def stream_wait(frm: torch.cuda.Stream, to: torch.cuda.Stream):
    """`to` waits for the work enqueued on `frm` so far: eunet_stream_wait (a device-scope event release,
    where torch's Stream.wait_stream records a system-scope one)."""
    call("eunet_stream_wait", ctypes.c_void_p(frm.cuda_stream), ctypes.c_void_p(to.cuda_stream))


_guards = {}  # device index -> the fp64 [1] tensor eunet_set_update_guard points at (kept alive here)


def set_update_guard(device, guard):
    """eunet_set_update_guard: while guard (a device fp64 [1] tensor, or None) is nonzero, BN running
    statistics and the native clip + AdamW leave the persistent state untouched."""
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if guard is not None and (guard.dtype != torch.float64 or guard.device.type != "cuda" or guard.device.index != idx):
        raise ValueError("update guard: an fp64 tensor on the guarded device")
    if _guards.get(idx) is guard:
        return
    call("eunet_set_update_guard", idx, None if guard is None else ctypes.c_void_p(guard.data_ptr()))
    if guard is None:
        _guards.pop(idx, None)
    else:
        _guards[idx] = guard


def update_guard(device):
    """The tensor eunet_set_update_guard currently points at for device (None: no guard)."""
    dev = torch.device(device)
    return _guards.get(dev.index if dev.index is not None else torch.cuda.current_device())


def _ptr(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise _lib.EunetError("eunet ops need device tensors (no CPU fallback)")
    return ctypes.c_void_p(t.data_ptr())


def act(t: torch.Tensor, coff: int = 0, c: int | None = None) -> Act:
    """NHWC view of a contiguous [N,H,W,Ctot] tensor, channels [coff, coff+c)."""
    if t.dim() != 4 or not t.is_contiguous():
        raise _lib.EunetError(f"act(): need a contiguous NHWC tensor, got {tuple(t.shape)}")
    if not t.is_cuda:
        raise _lib.EunetError("act(): tensor must live on the GPU")
    n, h, w, ct = t.shape
    a = Act(t.data_ptr(), n, h, w, ct - coff if c is None else c, ct, coff, DTYPES[t.dtype])
    a._keep = t  # the view keeps its tensor (and device memory) alive
    return a


def _ref(a):
    return None if a is None else ctypes.byref(a)


@_dispatched("T T!")
def nchw_to_nhwc(x: torch.Tensor, out: torch.Tensor):
    call("eunet_nchw_to_nhwc", _ptr(x), ctypes.byref(act(out)), _stream())


def conv3x3_packed_bytes(cout, cin, dtype):
    b = c_size_t()
    call("eunet_conv3x3_packed_bytes", cout, cin, DTYPES[dtype], ctypes.byref(b))
    return b.value


@_dispatched("T d b", returns_tensor=True)
def conv3x3_pack(w: torch.Tensor, dtype, flip: bool) -> torch.Tensor:
    cout, cin = w.shape[0], w.shape[1]
    nbytes = conv3x3_packed_bytes(cin if flip else cout, cout if flip else cin, dtype)
    wp = torch.empty(nbytes // (2 if dtype == torch.bfloat16 else 4), dtype=dtype, device=w.device)
    call("eunet_conv3x3_pack", _ptr(w.contiguous()), cout, cin, int(flip), _ptr(wp), DTYPES[dtype], _stream())
    return wp


def conv3x3_pack_many(items, dtype):
    """[(w, flip), ...] -> packed tensors, one launch per PACK_MAX tensors (eunet_conv3x3_pack_many)."""
    out = []
    for lo in range(0, len(items), _lib.PACK_MAX):
        chunk = items[lo:lo + _lib.PACK_MAX]
        descs = (_lib.PackDesc * len(chunk))()
        keep = []
        for d, (w, flip) in zip(descs, chunk):
            cout, cin = w.shape[0], w.shape[1]
            nbytes = conv3x3_packed_bytes(cin if flip else cout, cout if flip else cin, dtype)
            wp = torch.empty(nbytes // (2 if dtype == torch.bfloat16 else 4), dtype=dtype, device=w.device)
            wc = w.contiguous()
            keep.append(wc)
            d.w, d.cout, d.cin, d.flip, d.wp = wc.data_ptr(), cout, cin, int(flip), wp.data_ptr()
            out.append(wp)
        call("eunet_conv3x3_pack_many", ctypes.cast(descs, ctypes.c_void_p), len(chunk), DTYPES[dtype], _stream())
    return out


def conv3x3_tiles(y_act: Act) -> int:
    t = c_int()
    call("eunet_conv3x3_tiles", ctypes.byref(y_act), ctypes.byref(t))
    return t.value


@_dispatched("A T A! T? T? T? T!? i s?")
def conv3x3_fwd(x: Act, wp, y: Act, bias=None, scale=None, shift=None, stats=None, nstride=0, sub=None):
    """nstride > 0: scale/shift are per-sample [N][nstride] (BN+ReLU+Dropout2d folded).
    sub: optional kprof sub-family the launch is also credited to (e.g. the encoder forward convs)."""
    flops = 2.0 * 9 * x.c * y.c * x.n * x.h * x.w
    esz = 2 if x.dtype == _lib.EUNET_BF16 else 4
    # algorithmic HBM bytes: read x once, write y once, read the packed weights once
    nbytes = float(esz * x.n * x.h * x.w * (x.c + y.c) + wp.numel() * wp.element_size())
    with kprof.timed("conv3x3_fwd", flops, nbytes, sub=sub):
        call("eunet_conv3x3_fwd", ctypes.byref(x), _ptr(scale), _ptr(shift), int(nstride), _ptr(wp), _ptr(bias),
             ctypes.byref(y), _ptr(stats), _stream())


@_dispatched("A T A! T?")
def conv3x3_dgrad(dy: Act, wp_t, gx: Act, gscale=None):
    """plain dgrad (the block-input gradient): gx = conv(dy, W'), wp_t packed with flip=True."""
    flops = 2.0 * 9 * dy.c * gx.c * dy.n * dy.h * dy.w
    esz = 2 if dy.dtype == _lib.EUNET_BF16 else 4
    nbytes = float(esz * dy.n * dy.h * dy.w * (dy.c + gx.c) + wp_t.numel() * wp_t.element_size())
    with kprof.timed("conv3x3_dgrad", flops, nbytes):
        call("eunet_conv3x3_dgrad", ctypes.byref(dy), _ptr(wp_t), ctypes.byref(gx), _ptr(gscale), _stream())


@_dispatched("A T A! A T T T T T! T?")
def conv3x3_dgrad_bnbwd(dy: Act, wp_t, gx: Act, y: Act, mean, invstd, scale, shift, part, gscale=None):
    """dgrad + the BN-backward partial sums of the layer it feeds (see eunet.h)."""
    flops = 2.0 * 9 * dy.c * gx.c * dy.n * dy.h * dy.w
    esz = 2 if dy.dtype == _lib.EUNET_BF16 else 4
    nbytes = float(esz * dy.n * dy.h * dy.w * (dy.c + 2 * gx.c) + wp_t.numel() * wp_t.element_size())
    with kprof.timed("conv3x3_dgrad", flops, nbytes):
        call("eunet_conv3x3_dgrad_bnbwd", ctypes.byref(dy), _ptr(wp_t), ctypes.byref(gx), ctypes.byref(y), _ptr(mean),
             _ptr(invstd), _ptr(scale), _ptr(shift), _ptr(gscale), _ptr(part), _stream())


def conv3x3_wgrad_splits(dy: Act, cin: int, dtype) -> int:
    s = c_int()
    call("eunet_conv3x3_wgrad_splits", ctypes.byref(dy), cin, DTYPES[dtype], ctypes.byref(s))
    return s.value


@_dispatched("A A T A!? T A! A? T? T? T? T? T!? T?")
def conv3x3_dgrad_fused(g: Act, y_in: Act, coef, gy_out: Act | None, wp_t, gx: Act, y_next: Act | None = None,
                        mean=None, invstd=None, scale=None, shift=None, part=None, gscale=None):
    """Data gradient with the BN backward of the differentiated layer fused into the operand staging
    (gy = coef-affine of (g, y_in), stored to gy_out for the weight gradient) and, optionally, the
    reduction half of the next BN backward over gx (include/eunet.h)."""
    flops = 2.0 * 9 * g.c * gx.c * g.n * g.h * g.w
    esz = 2 if g.dtype == _lib.EUNET_BF16 else 4
    # algorithmic HBM bytes: read g and y_in once, write gy_out and gx once, (read y_next), weights once
    nbytes = float(esz * g.n * g.h * g.w * (2 * g.c + (g.c if gy_out is not None else 0) + gx.c +
                                            (gx.c if y_next is not None else 0)) + wp_t.numel() * wp_t.element_size())
    with kprof.timed("conv3x3_dgrad", flops, nbytes):
        call("eunet_conv3x3_dgrad_fused", ctypes.byref(g), ctypes.byref(y_in), _ptr(coef), _ref(gy_out), _ptr(wp_t),
             ctypes.byref(gx), _ref(y_next), _ptr(mean), _ptr(invstd), _ptr(scale), _ptr(shift), _ptr(part),
             _ptr(gscale), _stream())


@_dispatched("A A T! T!? i T? T? i")
def conv3x3_wgrad(x: Act, dy: Act, dw_part, db_part, nsplit, scale=None, shift=None, nstride=0):
    flops = 2.0 * 9 * x.c * dy.c * x.n * x.h * x.w
    esz = 2 if x.dtype == _lib.EUNET_BF16 else 4
    # algorithmic HBM bytes: read x and dy once, write the fp32 split partials of dW (and db) once
    nbytes = float(esz * x.n * x.h * x.w * (x.c + dy.c) + 4 * nsplit * dy.c * (9 * x.c + 1))
    with kprof.timed("conv3x3_wgrad", flops, nbytes):
        call("eunet_conv3x3_wgrad", ctypes.byref(x), _ptr(scale), _ptr(shift), int(nstride), ctypes.byref(dy),
             _ptr(dw_part),
             _ptr(db_part), nsplit, _stream())


@_dispatched("T T? i i i i T! T!?")
def wgrad_reduce(dw_part, db_part, nsplit, cout, cin, taps, dw, db):
    call("eunet_wgrad_reduce", _ptr(dw_part), _ptr(db_part), nsplit, cout, cin, taps, _ptr(dw), _ptr(db),
         _stream())


@_dispatched("A T T? A! T!?")
def conv_small_fwd(x: Act, w, bias, y: Act, stats=None):
    call("eunet_conv_small_fwd", ctypes.byref(x), _ptr(w), _ptr(bias), ctypes.byref(y), _ptr(stats), _stream())


def conv3x3_fwd_narrow(x: Act, cin: int, wp, y: Act, bias=None, stats=None):
    """A few-channel conv (cin < 8) on the MFMA forward: x is a view of 8 channels whose channels >= cin
    are zero and wp packs the [cout][cin] weights (its padding is zero too).  Timed as the HBM-bound
    "conv_small" family with its true FLOPs, outside the conv3x3 MFMA roofline family."""
    flops = 2.0 * 9 * cin * y.c * x.n * x.h * x.w
    esz = 2 if x.dtype == _lib.EUNET_BF16 else 4
    nbytes = float(esz * x.n * x.h * x.w * (x.c + y.c))
    with kprof.timed("conv_small", flops, nbytes):
        call("eunet_conv3x3_fwd", ctypes.byref(x), None, None, 0, _ptr(wp), _ptr(bias), ctypes.byref(y),
             _ptr(stats), _stream())


def conv_small_wgrad_splits(dy: Act) -> int:
    s = c_int()
    call("eunet_conv_small_wgrad_splits", ctypes.byref(dy), ctypes.byref(s))
    return s.value


@_dispatched("A A T! T!? i")
def conv_small_wgrad(x: Act, dy: Act, dw_part, db_part, nsplit):
    call("eunet_conv_small_wgrad", ctypes.byref(x), ctypes.byref(dy), _ptr(dw_part), _ptr(db_part), nsplit,
         _stream())


@_dispatched("T i i T T f f T!? T!? T!? T!? T!? T!? T!?")
def bn_finalize(stats, tiles, c, gamma, beta, eps, momentum, run_mean, run_var, mean, invstd, scale, shift,
                num_batches_tracked=None):
    call("eunet_bn_finalize", _ptr(stats), tiles, c, _ptr(gamma), _ptr(beta), float(eps), float(momentum),
         _ptr(run_mean), _ptr(run_var), _ptr(mean), _ptr(invstd), _ptr(scale), _ptr(shift),
         _ptr(num_batches_tracked), _stream())


@_dispatched("T T T T f T! T!")
def bn_eval_affine(gamma, beta, run_mean, run_var, eps, scale, shift):
    call("eunet_bn_eval_affine", gamma.numel(), _ptr(gamma), _ptr(beta), _ptr(run_mean), _ptr(run_var),
         float(eps), _ptr(scale), _ptr(shift), _stream())


@_dispatched("A T T A!")
def bnrelu(y: Act, scale, shift, out: Act):
    call("eunet_bnrelu", ctypes.byref(y), _ptr(scale), _ptr(shift), ctypes.byref(out), _stream())


@_dispatched("A T T A!? A!")
def bnrelu_pool(y: Act, scale, shift, act_out: Act | None, pooled: Act):
    call("eunet_bnrelu_pool", ctypes.byref(y), _ptr(scale), _ptr(shift), _ref(act_out), ctypes.byref(pooled),
         _stream())


@_dispatched("A T T A!")
def bnrelu_upsample(y: Act, scale, shift, out: Act):
    call("eunet_bnrelu_upsample", ctypes.byref(y), _ptr(scale), _ptr(shift), ctypes.byref(out), _stream())


@_dispatched("A T T T T i T!")
def bnrelu_conv1x1(y: Act, scale, shift, w, b, k, z):
    call("eunet_bnrelu_conv1x1", ctypes.byref(y), _ptr(scale), _ptr(shift), _ptr(w), _ptr(b), k, _ptr(z),
         _stream())


def head_workspace_bytes(n, h, w, k, dtype=torch.float32):
    b = c_size_t()
    call("eunet_head_workspace_bytes", n, h, w, k, DTYPES[dtype], ctypes.byref(b))
    return b.value


@_dispatched("T i i i i T T T T T T b f f T!? T!? T!? T!? T!? T!? T! d")
def head_fwd(z, n, h, w, k, w1, b1, gamma, beta, w2, b2, training, eps, momentum, run_mean, run_var, mean,
             invstd, out2h, logits, ws, dtype=torch.float32):
    call("eunet_head_fwd", _ptr(z), n, h, w, k, _ptr(w1), _ptr(b1), _ptr(gamma), _ptr(beta), _ptr(w2), _ptr(b2),
         int(training), float(eps), float(momentum), _ptr(run_mean), _ptr(run_var), _ptr(mean), _ptr(invstd),
         _ptr(out2h), _ptr(logits), DTYPES[dtype], _ptr(ws), _stream())


@_dispatched("T i i i i T T T T T T T T? T? T! T! T! T! T! T! T! T! d")
def head_bwd(z, n, h, w, k, w1, b1, gamma, beta, w2, mean, invstd, g_logits, g_out2h, gz, gw1, gb1, ggamma,
             gbeta, gw2, gb2, ws, dtype=torch.float32):
    call("eunet_head_bwd", _ptr(z), n, h, w, k, _ptr(w1), _ptr(b1), _ptr(gamma), _ptr(beta), _ptr(w2),
         _ptr(mean), _ptr(invstd), _ptr(g_logits), _ptr(g_out2h), _ptr(gz), _ptr(gw1), _ptr(gb1), _ptr(ggamma),
         _ptr(gbeta), _ptr(gw2), _ptr(gb2), DTYPES[dtype], _ptr(ws), _stream())


def loss_reference_params() -> _lib.LossParams:
    p = _lib.LossParams()
    call("eunet_loss_reference_params", ctypes.byref(p))
    return p


def loss_sums_len(n, k):
    v = c_int()
    call("eunet_loss_sums_len", n, k, ctypes.byref(v))
    return v.value


def loss_workspace_bytes(n, k, h, w):
    b = c_size_t()
    call("eunet_loss_workspace_bytes", n, k, h, w, ctypes.byref(b))
    return b.value


def loss_fwd(logits, target, params, sums, loss, parts, ws):
    """params: _lib.LossParams or None (the reference Trainer's configuration)."""
    n, k, h, w = logits.shape
    call("eunet_loss_fwd", _ptr(logits), _ptr(target), n, k, h, w, _ref(params), _ptr(sums), _ptr(loss),
         _ptr(parts), _ptr(ws), _stream())


def loss_bwd(logits, target, params, sums, gloss, glogits):
    n, k, h, w = logits.shape
    call("eunet_loss_bwd", _ptr(logits), _ptr(target), n, k, h, w, _ref(params), _ptr(sums), _ptr(gloss),
         _ptr(glogits), _stream())


def bn_bwd_tiles(y: Act) -> int:
    t = c_int()
    call("eunet_bn_bwd_tiles", ctypes.byref(y), ctypes.byref(t))
    return t.value


@_dispatched("A A T T T T T!")
def bn_bwd_reduce(g: Act, y: Act, mean, invstd, scale, shift, part):
    call("eunet_bn_bwd_reduce", ctypes.byref(g), ctypes.byref(y), _ptr(mean), _ptr(invstd), _ptr(scale),
         _ptr(shift), _ptr(part), _stream())


@_dispatched("T i i T! i? T!?")
def colsum(part, rows, cols, out, split=None, out_hi=None):
    """Column sums of part [rows][cols] -> out (or out[:split] / out_hi[:cols - split])."""
    b = c_size_t()
    call("eunet_colsum_ws_bytes", rows, cols, ctypes.byref(b))
    ws = torch.empty(b.value, dtype=torch.uint8, device=part.device)
    if out_hi is None:
        call("eunet_colsum", _ptr(part), rows, cols, _ptr(out), _ptr(ws), _stream())
    else:
        call("eunet_colsum_split", _ptr(part), rows, cols, int(split), _ptr(out), _ptr(out_hi), _ptr(ws), _stream())


@_dispatched("A A T T T T T T A!")
def bn_bwd_apply(g: Act, y: Act, mean, invstd, scale, shift, dbeta, dgamma, gy: Act):
    """scale / shift: the BN's forward affine (they define the ReLU mask, see eunet.h)."""
    call("eunet_bn_bwd_apply", ctypes.byref(g), ctypes.byref(y), _ptr(mean), _ptr(invstd), _ptr(scale),
         _ptr(shift), _ptr(dbeta), _ptr(dgamma), ctypes.byref(gy), _stream())


@_dispatched("T T T T T T i T!")
def bn_bwd_coef(mean, invstd, scale, shift, dbeta, dgamma, count: int, coef):
    """coef [4][C] = (k1, kq, k2, k3) of gy = k1 g [y k1 + kq > 0] + k2 y + k3 (count = N*H*W)."""
    call("eunet_bn_bwd_coef", _ptr(mean), _ptr(invstd), _ptr(scale), _ptr(shift), _ptr(dbeta), _ptr(dgamma),
         int(count), int(mean.numel()), _ptr(coef), _stream())


@_dispatched("A A T A!")
def bn_bwd_apply_coef(g: Act, y: Act, coef, gy: Act):
    call("eunet_bn_bwd_apply_coef", ctypes.byref(g), ctypes.byref(y), _ptr(coef), ctypes.byref(gy), _stream())


@_dispatched("A A A? A!")
def pool_bwd_add(act_saved: Act, gpool: Act, gskip: Act | None, gout: Act):
    call("eunet_pool_bwd_add", ctypes.byref(act_saved), ctypes.byref(gpool), _ref(gskip), ctypes.byref(gout),
         _stream())


@_dispatched("A A!")
def upsample_bwd(ghi: Act, glo: Act):
    call("eunet_upsample_bwd", ctypes.byref(ghi), ctypes.byref(glo), _stream())


def pool_bwd_add_bnr_rows(gout: Act) -> int:
    r = c_int()
    call("eunet_pool_bwd_add_bnr_rows", ctypes.byref(gout), ctypes.byref(r))
    return r.value


@_dispatched("A A A? A!? A T T T T T!")
def pool_bwd_add_bnr(act_saved: Act, gpool: Act, gskip: Act | None, gout: Act | None, y: Act, mean, invstd, scale,
                     shift, part):
    """pool_bwd_add + the BN-backward partial sums of the block whose output gradient gout is (gout None: reduced
    only, bn_bwd_apply_pool recomputes it)."""
    call("eunet_pool_bwd_add_bnr", ctypes.byref(act_saved), ctypes.byref(gpool), _ref(gskip), _ref(gout),
         ctypes.byref(y), _ptr(mean), _ptr(invstd), _ptr(scale), _ptr(shift), _ptr(part), _stream())


@_dispatched("A A? A T T T T T T A!")
def bn_bwd_apply_pool(gpool: Act, gskip: Act | None, y: Act, mean, invstd, scale, shift, dbeta, dgamma, gy: Act):
    """bn_bwd_apply of gout = gskip + scatter(gpool) that pool_bwd_add_bnr reduced without storing (recomputed per
    2x2 window with its arithmetic and rounding: the same gy bit for bit)."""
    call("eunet_bn_bwd_apply_pool", ctypes.byref(gpool), _ref(gskip), ctypes.byref(y), _ptr(mean), _ptr(invstd),
         _ptr(scale), _ptr(shift), _ptr(dbeta), _ptr(dgamma), ctypes.byref(gy), _stream())


def upsample_bwd_bnr_rows(glo: Act) -> int:
    r = c_int()
    call("eunet_upsample_bwd_bnr_rows", ctypes.byref(glo), ctypes.byref(r))
    return r.value


@_dispatched("A A! A T T T T T!")
def upsample_bwd_bnr(ghi: Act, glo: Act, y: Act, mean, invstd, scale, shift, part):
    """upsample_bwd + the BN-backward partial sums of the block whose output gradient glo is."""
    call("eunet_upsample_bwd_bnr", ctypes.byref(ghi), ctypes.byref(glo), ctypes.byref(y), _ptr(mean), _ptr(invstd),
         _ptr(scale), _ptr(shift), _ptr(part), _stream())


def conv1x1_bwd_tiles(y: Act) -> int:
    t = c_int()
    call("eunet_conv1x1_bwd_tiles", ctypes.byref(y), ctypes.byref(t))
    return t.value


@_dispatched("A T T T i T A! T!?")
def conv1x1_bwd(y: Act, scale, shift, w, k, gz, gact: Act, part):
    call("eunet_conv1x1_bwd", ctypes.byref(y), _ptr(scale), _ptr(shift), _ptr(w), k, _ptr(gz),
         ctypes.byref(gact), _ptr(part), _stream())


@_dispatched("A T T T i T A!? T!? T T T!")
def conv1x1_bwd_bnr(y: Act, scale, shift, w, k, gz, gact: Act | None, part, mean, invstd, bn_part):
    """conv1x1_bwd + the BN-backward partial sums [tiles][2][C] of y's BatchNorm over gact (gact None: the
    gradient is reduced, not stored -- bn_bwd_apply_1x1 recomputes it)."""
    call("eunet_conv1x1_bwd_bnr", ctypes.byref(y), _ptr(scale), _ptr(shift), _ptr(w), k, _ptr(gz),
         _ref(gact), _ptr(part), _ptr(mean), _ptr(invstd), _ptr(bn_part), _stream())


@_dispatched("A T i T T T T T T T A!")
def bn_bwd_apply_1x1(y: Act, w, k, gz, mean, invstd, scale, shift, dbeta, dgamma, gy: Act):
    """bn_bwd_apply of the gradient W^T gz that conv1x1_bwd_bnr reduced without storing (recomputed per pixel
    with its arithmetic and rounding: the same gy bit for bit)."""
    call("eunet_bn_bwd_apply_1x1", ctypes.byref(y), _ptr(w), k, _ptr(gz), _ptr(mean), _ptr(invstd), _ptr(scale),
         _ptr(shift), _ptr(dbeta), _ptr(dgamma), ctypes.byref(gy), _stream())


# ---- evaluation path (evalpath.hip) ------------------------------------------------
def semantic_counts(pred, gt):
    """pred, gt int64 [n, ...] -> counts int64 [n, 3, 3] = (#pred==c, #gt==c, #both==c)."""
    n = pred.shape[0]
    hw = pred[0].numel()
    counts = torch.empty(n, 3, 3, dtype=torch.int64, device=pred.device)
    call("eunet_semantic_counts", _ptr(pred.contiguous()), _ptr(gt.contiguous()), n, hw, _ptr(counts), _stream())
    return counts


def binary_overlap(a, b):
    """int64 masks -> (inter, union, sum a, sum b) as python ints (nonzero = foreground)."""
    out = torch.empty(4, dtype=torch.int64, device=a.device)
    call("eunet_binary_overlap", _ptr(a.contiguous()), _ptr(b.contiguous()), a.numel(), _ptr(out), _stream())
    return tuple(int(v) for v in out.tolist())


def resize_bilinear(x, hout, wout, scale_h=None, scale_w=None, flip_h=False, flip_w=False, out=None):
    """x [..., H, W] fp32 -> [..., hout, wout]; scale_* = 1/scale_factor (F.interpolate with
    scale_factor) or None for in/out (F.interpolate with size)."""
    x = x.contiguous()
    hin, win = x.shape[-2:]
    planes = x.numel() // (hin * win)
    sh = float(scale_h) if scale_h is not None else hin / hout
    sw = float(scale_w) if scale_w is not None else win / wout
    y = out if out is not None else torch.empty(*x.shape[:-2], hout, wout, dtype=torch.float32, device=x.device)
    call("eunet_resize_bilinear", _ptr(x), planes, hin, win, _ptr(y), hout, wout, sh, sw, int(flip_h), int(flip_w),
         _stream())
    return y


def softmax_crop(logits, h, w, flip_h=False, flip_w=False, out=None):
    """logits [K, hp, wp] fp32 -> probs [K, h, w] (crop to the top-left h x w, optional flips)."""
    logits = logits.contiguous().float()
    k, hp, wp = logits.shape
    y = out if out is not None else torch.empty(k, h, w, dtype=torch.float32, device=logits.device)
    call("eunet_softmax_crop", _ptr(logits), k, hp, wp, h, w, int(flip_h), int(flip_w), _ptr(y), _stream())
    return y


def accumulate(acc, p, mode: int, count: float = 1.0):
    call("eunet_accumulate", _ptr(acc), _ptr(p.contiguous()), acc.numel(), int(mode), float(count), _stream())


def probs_to_mask(probs):
    """probs [K, h, w] fp32 -> int64 mask [h, w] (the reference's thresholded conversion)."""
    probs = probs.contiguous().float()
    k, h, w = probs.shape
    mask = torch.empty(h, w, dtype=torch.int64, device=probs.device)
    ws = torch.empty(2, dtype=torch.int64, device=probs.device)
    call("eunet_probs_to_mask", _ptr(probs), k, h, w, _ptr(mask), _ptr(ws), _stream())
    return mask


# ---- dual-branch fusion (fusion.hip) -------------------------------------------------
def fusion_tiles(n, h, w):
    t, gt = c_int(), c_int()
    call("eunet_fusion_tiles", n, h, w, ctypes.byref(t), ctypes.byref(gt))
    return t.value, gt.value


def gate_fwd(za, zb, k, w1, a, st1, aux_a, aux_b):
    n, h, w, _ = za.shape
    call("eunet_gate_fwd", _ptr(za), _ptr(zb), n, h, w, k, _ptr(w1), _ptr(a), _ptr(st1), _ptr(aux_a), _ptr(aux_b),
         _stream())


def gate_mid_fwd(za, zb, k, a, sc1, sh1, w2, b, st2):
    n, h, w, _ = za.shape
    call("eunet_gate_mid_fwd", _ptr(za), _ptr(zb), n, h, w, k, _ptr(a), _ptr(sc1), _ptr(sh1), _ptr(w2), _ptr(b),
         _ptr(st2), _stream())


def gate_out_fwd(za, zb, k, b, sc2, sh2, f2: Act):
    n, h, w, _ = za.shape
    call("eunet_gate_out_fwd", _ptr(za), _ptr(zb), n, h, w, k, _ptr(b), _ptr(sc2), _ptr(sh2), ctypes.byref(f2),
         _stream())


def fusion_out_fwd(za, zb, k, y3: Act, sc3, sh3, w11, b11, b, sc2, sh2, wr, br, out):
    call("eunet_fusion_out_fwd", _ptr(za), _ptr(zb), k, ctypes.byref(y3), _ptr(sc3), _ptr(sh3), _ptr(w11), _ptr(b11),
         _ptr(b), _ptr(sc2), _ptr(sh2), _ptr(wr), _ptr(br), _ptr(out), _stream())


def fusion_out_bwd(za, zb, k, gout, b, sc2, sh2, wr, gz, gf2res, part):
    n, h, w, _ = za.shape
    call("eunet_fusion_out_bwd", _ptr(za), _ptr(zb), n, h, w, k, _ptr(gout), _ptr(b), _ptr(sc2), _ptr(sh2),
         _ptr(wr), _ptr(gz), _ptr(gf2res), _ptr(part), _stream())


def gate_bwd1(za, zb, k, gf2conv: Act, gf2res, b, mean2, istd2, gam2, bet2, gffd, gbhat, part):
    call("eunet_gate_bwd1", _ptr(za), _ptr(zb), k, ctypes.byref(gf2conv), _ptr(gf2res), _ptr(b), _ptr(mean2),
         _ptr(istd2), _ptr(gam2), _ptr(bet2), _ptr(gffd), _ptr(gbhat), _ptr(part), _stream())


def gate_bwd2(n, h, w, k, gbhat, b, mean2, istd2, gam2, dbet2, dgam2, a, mean1, istd1, gam1, bet1, w2, gabn, part):
    call("eunet_gate_bwd2", n, h, w, k, _ptr(gbhat), _ptr(b), _ptr(mean2), _ptr(istd2), _ptr(gam2), _ptr(dbet2),
         _ptr(dgam2), _ptr(a), _ptr(mean1), _ptr(istd1), _ptr(gam1), _ptr(bet1), _ptr(w2), _ptr(gabn), _ptr(part),
         _stream())


def gate_bwd3(za, zb, k, gabn, a, mean1, istd1, gam1, dbet1, dgam1, w1, gffd, gaux_a, gaux_b, gz_a, gz_b, part):
    n, h, w, _ = za.shape
    call("eunet_gate_bwd3", _ptr(za), _ptr(zb), n, h, w, k, _ptr(gabn), _ptr(a), _ptr(mean1), _ptr(istd1),
         _ptr(gam1), _ptr(dbet1), _ptr(dgam1), _ptr(w1), _ptr(gffd), _ptr(gaux_a), _ptr(gaux_b), _ptr(gz_a),
         _ptr(gz_b), _ptr(part), _stream())


def dropout_affine(scale, shift, keep, p, nscale, nshift, gscale=None):
    n, c = keep.shape
    call("eunet_dropout_affine", _ptr(scale), _ptr(shift), _ptr(keep), n, c, float(p), _ptr(nscale), _ptr(nshift),
         _ptr(gscale), _stream())


def consistency_tiles(h, w):
    t = c_int()
    call("eunet_consistency_tiles", h, w, ctypes.byref(t))
    return t.value


def consistency_fwd(fused, b0, b1, c0, c1, part, loss):
    n, k, h, w = fused.shape
    call("eunet_consistency_fwd", _ptr(fused), _ptr(b0), _ptr(b1), n, k, h, w, float(c0), float(c1), _ptr(part),
         _ptr(loss), _stream())


def consistency_bwd(fused, b0, b1, c0, c1, gloss, gfused, g0, g1):
    n, k, h, w = fused.shape
    call("eunet_consistency_bwd", _ptr(fused), _ptr(b0), _ptr(b1), n, k, h, w, float(c0), float(c1), _ptr(gloss),
         _ptr(gfused), _ptr(g0), _ptr(g1), _stream())


# ---- device-side data path (datapath.hip) ---------------------------------------------
def upload(a, device):
    """Host numpy array -> device tensor without a host synchronisation: staged through the
    caching pinned-memory allocator and copied asynchronously on the current stream (a pageable
    copy would wait for the stream to drain first)."""
    import numpy as np
    t = torch.from_numpy(np.ascontiguousarray(a))
    if torch.device(device).type != "cuda":
        return t.to(device)
    return t.pin_memory().to(device, non_blocking=True)


def _poly_arrays(polys):
    import numpy as np
    pts = np.concatenate([np.asarray(p, np.int32).reshape(-1, 2) for p in polys])
    off = np.concatenate([[0], np.cumsum([len(p) for p in polys])]).astype(np.int32)
    return pts, off


def rasterize_polygons(polys, labels, h, w, device):
    """polys: list of int32 [n_i, 2] (x, y) arrays; labels: ints (1 live, 2 dead) -> int64 [h, w]."""
    mask = torch.empty(h, w, dtype=torch.int64, device=device)
    if not polys:
        call("eunet_rasterize_polygons", None, None, None, 0, h, w, _ptr(mask), _stream())
        return mask
    import numpy as np
    pts_h, off_h = _poly_arrays(polys)
    pts, off, lab = upload(pts_h, device), upload(off_h, device), upload(np.asarray(labels, np.int32), device)
    call("eunet_rasterize_polygons", _ptr(pts), _ptr(off), _ptr(lab), len(polys), h, w, _ptr(mask), _stream())
    return mask


def rasterize_instances(polys, h, w, device, flip_h: bool = False, flip_v: bool = False):
    """One uint8 [h, w] mask per polygon (stacked [n, h, w]), mirrored by the training flips."""
    if not polys:
        return torch.zeros(0, h, w, dtype=torch.uint8, device=device)
    pts_h, off_h = _poly_arrays(polys)
    pts, off = upload(pts_h, device), upload(off_h, device)
    masks = torch.empty(len(polys), h, w, dtype=torch.uint8, device=device)
    call("eunet_rasterize_instances", _ptr(pts), _ptr(off), len(polys), h, w, int(flip_h), int(flip_v), _ptr(masks),
         _stream())
    return masks


def flip_u8(img, mode: int):
    out = torch.empty_like(img)
    h, w, c = img.shape
    call("eunet_flip_u8", _ptr(img.contiguous()), _ptr(out), h, w, c, int(mode), _stream())
    return out


def flip_mask(mask, mode: int):
    out = torch.empty_like(mask)
    h, w = mask.shape
    call("eunet_flip_mask", _ptr(mask.contiguous()), _ptr(out), h, w, int(mode), _stream())
    return out


def augment_u8(img, alpha=None, beta=None, noise=None, lut=None):
    """In-place on a contiguous uint8 device tensor (reference order: alpha, beta, noise, LUT)."""
    flags = (1 if alpha is not None else 0) | (2 if beta is not None else 0) | \
        (4 if noise is not None else 0) | (8 if lut is not None else 0)
    call("eunet_augment_u8", _ptr(img), img.numel(), flags, float(alpha or 0.0), float(beta or 0.0),
         _ptr(noise), _ptr(lut), _stream())
    return img


def augment_ratio_u8(img, counts, u_alpha=None, u_beta=None):
    """In place: the reference's live-ratio-dependent brightness / contrast (dataset.py:225-257) with
    the ratio read from device counts (semantic_counts) and u_* the host's random.random() draws."""
    flags = (1 if u_alpha is not None else 0) | (2 if u_beta is not None else 0)
    if flags:
        call("eunet_augment_ratio_u8", _ptr(img), img.numel(), _ptr(counts), flags,
             0.0 if u_alpha is None else float(u_alpha), 0.0 if u_beta is None else float(u_beta), _stream())
    return img


def to_tensor(img):
    h, w, c = img.shape
    out = torch.empty(c, h, w, dtype=torch.float32, device=img.device)
    call("eunet_to_tensor", _ptr(img.contiguous()), h, w, c, _ptr(out), _stream())
    return out


def resize_u8(img, ho, wo):
    hi, wi, c = img.shape
    out = torch.empty(ho, wo, c, dtype=torch.uint8, device=img.device)
    call("eunet_resize_u8", _ptr(img.contiguous()), hi, wi, c, _ptr(out), ho, wo, _stream())
    return out


# ---- cv2 image operations (imgproc.hip) -------------------------------------------------
SHARPEN_3X3 = (-1.0, -1.0, -1.0, -1.0, 9.0, -1.0, -1.0, -1.0, -1.0)  # dataset.py:288-290, train_eval.py:388-390


def _size_out(fn, *args):
    n = ctypes.c_size_t(0)
    call(fn, *args, ctypes.byref(n))
    return int(n.value)


def rgb2lab_u8(img):
    out = torch.empty_like(img)
    call("eunet_rgb2lab_u8", _ptr(img.contiguous()), _ptr(out), img.shape[0] * img.shape[1], _stream())
    return out


def lab2rgb_u8(lab):
    out = torch.empty_like(lab)
    call("eunet_lab2rgb_u8", _ptr(lab.contiguous()), _ptr(out), lab.shape[0] * lab.shape[1], _stream())
    return out


def rgb2gray_u8(img):
    h, w, _ = img.shape
    out = torch.empty(h, w, dtype=torch.uint8, device=img.device)
    call("eunet_rgb2gray_u8", _ptr(img.contiguous()), _ptr(out), h * w, _stream())
    return out


def hsv_adjust_u8(img, sat=None, hue=None, val=None):
    """In place: S *= sat (dataset.py:259-264) or H += hue mod 180, V *= val (:295-300)."""
    mode = (1 if sat is not None else 0) | (2 if hue is not None else 0)
    if mode & 2 and val is None:
        raise ValueError("hsv_adjust_u8: hue and val go together")
    # explicit None tests: sat = 0.0 / val = 0.0 are real requests (desaturate / black), not "unset"
    call("eunet_hsv_adjust_u8", _ptr(img), img.shape[0] * img.shape[1], 1.0 if sat is None else float(sat),
         0.0 if hue is None else float(hue), 1.0 if val is None else float(val), mode, _stream())
    return img


def clahe_u8(src, clip_limit, grid=(8, 8), lab_to_rgb=False):
    """cv2.createCLAHE(clip_limit, grid).apply.  lab_to_rgb: src is a Lab image, its L channel is
    equalised and the RGB image is returned (the merge + LAB2RGB of dataset.py:70-71)."""
    h, w = src.shape[:2]
    luts = torch.empty(grid[0] * grid[1] * 256, dtype=torch.uint8, device=src.device)
    out = torch.empty(h, w, 3, dtype=torch.uint8, device=src.device) if lab_to_rgb else torch.empty_like(src)
    call("eunet_clahe_u8", _ptr(src.contiguous()), int(lab_to_rgb), h, w, float(clip_limit), grid[0], grid[1],
         _ptr(luts), _ptr(out), _stream())
    return out


def clahe_rgb_u8(img, clip_limit, grid=(8, 8)):
    """RGB -> Lab, CLAHE on L, -> RGB (dataset.py:63-71, 268-272; train_eval.py:380-385)."""
    return clahe_u8(rgb2lab_u8(img), clip_limit, grid, lab_to_rgb=True)


def filter3x3_u8(img, k9):
    h, w = img.shape[:2]
    c = img.shape[2] if img.dim() == 3 else 1
    kk = (ctypes.c_float * 9)(*[float(v) for v in k9])
    out = torch.empty_like(img)
    call("eunet_filter3x3_u8", _ptr(img.contiguous()), _ptr(out), h, w, c, ctypes.addressof(kk), _stream())
    return out


def sharpen_u8(img, strength):
    """cv2.filter2D(img, -1, [[-1,-1,-1],[-1,9,-1],[-1,-1,-1]] * strength)."""
    return filter3x3_u8(img, [v * strength for v in SHARPEN_3X3])


def unsharp_u8(img):
    h, w = img.shape[:2]
    c = img.shape[2] if img.dim() == 3 else 1
    out = torch.empty_like(img)
    call("eunet_unsharp_u8", _ptr(img.contiguous()), _ptr(out), h, w, c, _stream())
    return out


def edge_features_u8(gray):
    h, w = gray.shape
    ws = torch.empty(_size_out("eunet_edge_features_workspace_bytes", h, w), dtype=torch.uint8, device=gray.device)
    out = torch.empty_like(gray)
    call("eunet_edge_features_u8", _ptr(gray.contiguous()), h, w, _ptr(ws), _ptr(out), _stream())
    return out


def cell_preprocess_u8(img, live_mask, dead_mask=None):
    """dataset.py:58-131 (_apply_cell_specific_preprocessing) on an HWC uint8 device image.
    live_mask / dead_mask: int64 [h, w], nonzero where any live / dead instance covers the
    pixel (the np.maximum unions of :96-100); dead_mask None = no dead instance."""
    h, w, _ = img.shape
    img = img.contiguous()
    clahe = clahe_rgb_u8(img, 2.5)
    edges = edge_features_u8(rgb2gray_u8(img))
    if live_mask is not None:
        call("eunet_live_boost_u8", _ptr(clahe), _ptr(live_mask.contiguous()), h * w, _stream())
    dead_gray = clahe_u8(rgb2gray_u8(clahe), 3.0) if dead_mask is not None else None
    mixed = torch.empty_like(img)
    call("eunet_cell_mix_u8", _ptr(img), _ptr(clahe), _ptr(edges),
         _ptr(dead_mask.contiguous() if dead_mask is not None else None), _ptr(dead_gray), h * w, _ptr(mixed),
         _stream())
    return unsharp_u8(mixed)


def chw_to_u8(x):
    """train_eval.py:367-377: CHW float -> HWC uint8 (x * 255 if max(x) <= 1), on the device."""
    c, h, w = x.shape
    x = x.contiguous().float()
    ws = torch.empty(_size_out("eunet_chw_to_u8_workspace_bytes", c, h, w), dtype=torch.uint8, device=x.device)
    out = torch.empty(h, w, c, dtype=torch.uint8, device=x.device)
    call("eunet_chw_to_u8", _ptr(x), c, h, w, _ptr(ws), _ptr(out), _stream())
    return out
