"""Formula-defined deterministic parameters (test infrastructure).

Fixtures never ship a 31 MB weight blob: every tensor of a state_dict is a pure
function of (key, shape) so the reference (when fixtures are generated), the
oracle and the HIP product can all load *identical* weights.

value[i] = (2*u_i - 1) * scale,  u_i = mix32(i * 0x9E3779B1 + crc32(key)) / 2**32
scale    = 1/sqrt(fan_in) for conv weights/biases (the bound PyTorch's default
           conv init uses), 0.1 for BN affine offsets around (1, 0).
"""
from __future__ import annotations

import zlib

import numpy as np


def _mix32(h: np.ndarray) -> np.ndarray:
    h = h.astype(np.uint64) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x7FEB352D)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(15)
    h = (h * np.uint64(0x846CA68B)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    return h


def uniform01(key: str, n: int) -> np.ndarray:
    salt = np.uint64(zlib.crc32(key.encode()) & 0xFFFFFFFF)
    idx = np.arange(n, dtype=np.uint64)
    h = _mix32((idx * np.uint64(0x9E3779B1) + salt) & np.uint64(0xFFFFFFFF))
    return h.astype(np.float64) / 4294967296.0


def formula_tensor(key: str, shape, fan_in: int | None = None) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    u = uniform01(key, n).reshape(shape)
    leaf = key.rsplit(".", 1)[-1]
    if leaf in ("running_mean",):
        return np.zeros(shape)
    if leaf in ("running_var",):
        return np.ones(shape)
    if leaf == "num_batches_tracked":
        return np.zeros(shape)
    if fan_in is None:  # BatchNorm affine
        return (1.0 if leaf == "weight" else 0.0) + 0.1 * (2.0 * u - 1.0)
    return (2.0 * u - 1.0) / np.sqrt(fan_in)


def formula_state_dict(spec):
    """spec: iterable of (key, shape, fan_in_or_None) -> {key: float64 ndarray}."""
    return {k: formula_tensor(k, s, f) for k, s, f in spec}
