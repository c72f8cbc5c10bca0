"""Restatement of the Harris feature path of image_stitching_harris.py -- TEST INFRASTRUCTURE.

==============================  ==================================================
oracle function                 reference (image_stitching_harris.py)
==============================  ==================================================
``gradients``                   conv2d :49-61 with Hx / Hy :150-158
``orientation``                 calc_orientation :63-70
``corners``                     HarrisCorner :135-185
``patch_descriptor``            gen_descriptor :72-133
``detect_and_describe``         compute_keypoints_and_descriptors_harris :187-214
==============================  ==================================================
"""
from __future__ import annotations

import numpy as np

from . import cv2_compat
from .numerics import F32, norm_f32


def gradients(gray: np.ndarray):
    """conv2d with the two 3x3 central-difference kernels, edge padding, float64.

    Only two taps are non-zero, so the correlation reduces exactly (integer inputs) to
    Ix = g[y, x-1] - g[y, x+1] and Iy = g[y-1, x] - g[y+1, x] with edge clamping.
    """
    p = np.pad(gray, 1, mode="edge").astype(np.float64)
    ix = p[1:-1, :-2] - p[1:-1, 2:]
    iy = p[:-2, 1:-1] - p[2:, 1:-1]
    return ix, iy


def response(ix, iy, k=0.05, block_size=21, gauss_sigma=2):
    sxx = cv2_compat.GaussianBlur(ix ** 2, (block_size, block_size), gauss_sigma)
    syy = cv2_compat.GaussianBlur(iy ** 2, (block_size, block_size), gauss_sigma)
    sxy = cv2_compat.GaussianBlur(ix * iy, (block_size, block_size), gauss_sigma)
    det = (sxx * syy) - (sxy ** 2)
    tr = sxx + syy
    return det - k * (tr ** 2)


def corners(img_bgr, max_points=200, k=0.05, block_size=21, gauss_sigma=2, thresh_ratio=0.02):
    """-> (list of (y, x, R) best-first, Ix, Iy)."""
    gray = cv2_compat.bgr_to_gray_u8(img_bgr).astype(F32)
    ix, iy = gradients(gray)
    R = response(ix, iy, k, block_size, gauss_sigma)
    thr = np.max(R) * thresh_ratio
    h, w = R.shape
    inner = R[1:-1, 1:-1]
    nmax = np.full(inner.shape, -np.inf)
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            nmax = np.maximum(nmax, R[1 + dy:h - 1 + dy, 1 + dx:w - 1 + dx])
    sel = (inner > thr) & (inner == nmax)
    ys, xs = np.nonzero(sel)
    vals = inner[ys, xs]
    order = np.argsort(-vals, kind="stable")[:max_points]
    cands = [(int(ys[i]) + 1, int(xs[i]) + 1, float(vals[i])) for i in order]
    return cands, ix, iy


def orientation(ix, iy):
    m = np.sqrt(ix ** 2 + iy ** 2)
    theta = np.arctan2(iy, ix) * 180 / np.pi
    theta = (theta + 360) % 360
    return m, theta


def _hist8(mag, ang, bins=8):
    """Sequential f32 histogram: h[b] = f32(double(h[b]) + mag) in row-major order."""
    h = np.zeros(bins, F32)
    idx = ((np.remainder(ang, 360) / 360) * bins).astype(np.int64) % bins
    for b, mv in zip(idx.ravel().tolist(), mag.ravel().tolist()):
        h[b] = F32(float(h[b]) + mv)
    return h


def patch_descriptor(y, x, m, theta):
    pm = np.pad(m, 8, mode="edge")
    pt = np.pad(theta, 8, mode="edge")
    patch_m = pm[y + 8:y + 24, x + 8:x + 24].copy()
    patch_t = pt[y + 8:y + 24, x + 8:x + 24].copy()
    patch_m = cv2_compat.GaussianBlur(patch_m, (9, 9), 1.5 * 3)
    main = _hist8(patch_m, patch_t)
    main_theta = (np.argmax(main) + 0.5) * (360 / 8)
    patch_t = patch_t - main_theta
    patch_t = (patch_t + 360) % 360
    desc = []
    for by in range(4):
        for bx in range(4):
            sl = (slice(4 * by, 4 * by + 4), slice(4 * bx, 4 * bx + 4))
            desc.append(_hist8(patch_m[sl], patch_t[sl]))
    d = np.concatenate(desc).astype(F32)
    d = (d / F32(norm_f32(d) + F32(1e-7))).astype(F32)
    d = np.clip(d, F32(0), F32(0.2))
    d = (d / F32(norm_f32(d) + F32(1e-7))).astype(F32)
    return d


def detect_and_describe(img_bgr, max_points=200):
    """-> (kps [(x, y)], descs float32 (N, 128)); corners within 8 px of the border dropped."""
    cands, ix, iy = corners(img_bgr, max_points=max_points)
    m, theta = orientation(ix, iy)
    h, w = img_bgr.shape[:2]
    kps, descs = [], []
    for (yy, xx, _) in cands:
        if yy < 8 or yy >= h - 8 or xx < 8 or xx >= w - 8:
            continue
        kps.append((xx, yy))
        descs.append(patch_descriptor(yy, xx, m, theta))
    return kps, np.array(descs, F32).reshape(-1, 128)
