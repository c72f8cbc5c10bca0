"""Bit-level restatements of the numpy / OpenBLAS arithmetic the reference relies on.

TEST INFRASTRUCTURE (see oracle/__init__.py).  Each function states the numpy call it
stands for and how that was established in this container (numpy 2.2.6, OpenBLAS 0.3.29
DYNAMIC_ARCH selecting the SkylakeX kernels on an AVX-512 Xeon):

* ``sdot_skx``   == ``np.dot`` / ``np.linalg.norm`` on float32 vectors of length >= 32
  (OpenBLAS ``sdot_kernel_16``: four 16-lane FMA accumulators per 64 elements, folded
  to 8 lanes, AVX2 loop over 32-element chunks, ((a0+a1)+a2)+a3, 256->128 fold, two
  ``hadd``; scalar tail accumulated in double).  Verified 100 % on 3000 random vectors
  each at n = 32, 64, 96, 128, 130.
* ``sdot_tail``  == ``np.dot`` on float32 vectors shorter than 32 (products rounded to
  f32, summed in double, result rounded to f32).  Verified on 20 000 random 3-vectors.
* ``RAD2DEG_F32`` == numpy's float32 ``rad2deg`` constant ``f32(180) / f32(pi)``.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
RAD2DEG_F32 = np.float32(np.float32(180.0) / np.float32(np.pi))


def _fma32(a, b, c):
    """Single-rounding f32 fused multiply-add (product of two f32 is exact in f64)."""
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(F32)


def sdot_skx(x: np.ndarray, y: np.ndarray) -> np.float32:
    """OpenBLAS 0.3.29 SkylakeX ``sdot`` summation order (leading axis = vector)."""
    x = np.asarray(x, F32)
    y = np.asarray(y, F32)
    n = x.shape[-1]
    lead = x.shape[:-1]
    n64 = n & ~63
    n32 = n & ~31
    acc16 = [np.zeros(lead + (16,), F32) for _ in range(4)]
    i = 0
    while i < n64:
        for k in range(4):
            s = slice(i + 16 * k, i + 16 * k + 16)
            acc16[k] = _fma32(x[..., s], y[..., s], acc16[k])
        i += 64
    acc8 = [(a[..., :8] + a[..., 8:]).astype(F32) for a in acc16]
    while i < n32:
        for k in range(4):
            s = slice(i + 8 * k, i + 8 * k + 8)
            acc8[k] = _fma32(x[..., s], y[..., s], acc8[k])
        i += 32
    v = ((acc8[0] + acc8[1]).astype(F32) + acc8[2]).astype(F32)
    v = (v + acc8[3]).astype(F32)
    h = (v[..., :4] + v[..., 4:]).astype(F32)
    h01 = (h[..., 0] + h[..., 1]).astype(F32)
    h23 = (h[..., 2] + h[..., 3]).astype(F32)
    kern = (h01 + h23).astype(F32)
    tail = np.zeros(lead, np.float64)
    for j in range(n32, n):
        tail = tail + (x[..., j] * y[..., j]).astype(F32).astype(np.float64)
    return (kern.astype(np.float64) + tail).astype(F32)


def sdot_tail(x, y) -> np.float32:
    """``np.dot`` of short float32 vectors: f32 products, double sum, f32 result."""
    acc = 0.0
    for a, b in zip(np.asarray(x, F32), np.asarray(y, F32)):
        acc += float(F32(a * b))
    return F32(acc)


def sdot(x, y) -> np.float32:
    return sdot_skx(x, y) if len(x) >= 32 else sdot_tail(x, y)


def norm_f32(v) -> np.float32:
    """``np.linalg.norm`` of a float32 vector: sqrt(sdot(v, v)) in float32."""
    return np.sqrt(sdot(v, v)).astype(F32)
