"""Restatement of the per-pair loop and the warp/composite of the stitchers -- TEST INFRASTRUCTURE.

================================  ==========================================================
oracle function                   reference
================================  ==========================================================
``read_pano_data``                image_stitching_sift.py:12-46 (= image_stitching_harris.py:10-44)
``cylindrical``                   cylindrical_projection image_stitching_sift.py:117-136
``nn_match_sift``                 NN loop of compute_shift_sift image_stitching_sift.py:63-79
``nn_match_harris``               simple_match image_stitching_harris.py:219-240
``ransac``                        ransac image_stitching_sift.py:86-111 (= harris :242-271)
``pad_image``                     image_stitching_sift.py:139-153
``blend_two_images``              image_stitching_sift.py:156-202
``rectangle_crop``                image_stitching_sift.py:208-247
``stitch``                        run_panorama's numeric body image_stitching_sift.py:290-384
                                  (= image_stitching_harris.py:460-542)
================================  ==========================================================
"""
from __future__ import annotations

import math

import numpy as np

from . import cv2_compat, harris, sift
from .numerics import F32, sdot_skx


def read_pano_data(path):
    images, focals, pending = [], [], None
    with open(path, "r", encoding="utf-8") as f:
        for line in f.read().splitlines():
            low = line.strip().lower()
            if ".jpg" in low or ".png" in low:
                pending = line.strip()
            elif " " not in low and low:
                try:
                    v = float(low)
                except ValueError:
                    continue
                if pending is not None:
                    images.append(pending)
                    focals.append(v)
                    pending = None
    return images, focals


# ----------------------------------------------------------------------------- C1
def cylindrical_maps(h, w, focal):
    """Forward map of every source pixel: (x', y') in fp64 with half-even rounding."""
    cx, cy = w // 2, h // 2
    xd = np.arange(w) - cx
    xm = np.array([round(focal * math.atan(d / focal)) for d in xd.tolist()], np.int64) + cx
    den = np.sqrt(xd.astype(np.float64) ** 2 + focal ** 2)
    yd = (np.arange(h) - cy).astype(np.float64)
    ym = np.rint(focal * (yd[:, None] / den[None, :])).astype(np.int64) + cy
    return xm, ym


def cylindrical(img, focal):
    """Last writer (largest row-major source index) wins for colliding destinations."""
    h, w = img.shape[:2]
    xm, ym = cylindrical_maps(h, w, focal)
    xm2 = np.broadcast_to(xm[None, :], (h, w))
    ok = (xm2 >= 0) & (xm2 < w) & (ym >= 0) & (ym < h)
    src = np.arange(h * w).reshape(h, w)
    dst = ym * w + xm2
    win = np.full(h * w, -1, np.int64)
    np.maximum.at(win, dst[ok], src[ok])
    out = np.zeros_like(img)
    hit = win >= 0
    flat_in = img.reshape(h * w, -1)
    out.reshape(h * w, -1)[hit] = flat_in[win[hit]]
    return out


# ----------------------------------------------------------------------------- M1 / H4
def nn_match_sift(descA, descB, thresh=25000):
    """-> (best index per row, best distance); distances are exact integers here."""
    if len(descA) == 0 or len(descB) == 0:
        return np.full(len(descA), -1, np.int64), np.full(len(descA), np.inf)
    # row chunks of 2048 (the whole f64 matrix at 1080p, 25k x 25k, is 5 GB); exact integers in
    # any chunking
    b = descB.astype(np.float64)
    nb = (b * b).sum(1)
    js, ds = [], []
    for i0 in range(0, len(descA), 2048):
        a = descA[i0:i0 + 2048].astype(np.float64)
        d = (a * a).sum(1)[:, None] + nb[None, :] - 2 * a @ b.T
        j = np.argmin(d, axis=1)
        js.append(j)
        ds.append(d[np.arange(len(a)), j])
    return np.concatenate(js), np.concatenate(ds)


def sift_matches(kpsA, descA, kpsB, descB, thresh=25000):
    j, dist = nn_match_sift(descA, descB, thresh)
    out = []
    for i in range(len(descA)):
        if j[i] >= 0 and dist[i] < thresh:
            out.append(((float(kpsA[i]["x"]), float(kpsA[i]["y"])),
                        (float(kpsB[j[i]]["x"]), float(kpsB[j[i]]["y"]))))
    return out


def nn_match_harris(descA, descB):
    """f32 distances in OpenBLAS sdot order; strict '<' keeps the first minimum."""
    if len(descA) == 0 or len(descB) == 0:
        return np.full(len(descA), -1, np.int64), np.full(len(descA), np.inf, F32)
    diff = (descA[:, None, :] - descB[None, :, :]).astype(F32)
    dist = sdot_skx(diff, diff)
    j = np.argmin(dist, axis=1)
    return j, dist[np.arange(len(descA)), j]


def harris_matches(kpsA, descA, kpsB, descB, thresh=1.0):
    j, dist = nn_match_harris(descA, descB)
    return [(kpsA[i], kpsB[j[i]]) for i in range(len(descA)) if j[i] >= 0 and dist[i] < F32(thresh)]


# ----------------------------------------------------------------------------- R1
def ransac(matches, thresh=3):
    """Exhaustive translation vote; first maximum wins; returns ((dx, dy), pair)."""
    if not matches:
        return (0, 0), None
    mv = np.array([(a[0] - b[0], a[1] - b[1]) for a, b in matches], np.float64)
    ddx = mv[None, :, 0] - mv[:, None, 0]
    ddy = mv[None, :, 1] - mv[:, None, 1]
    votes = ((ddx ** 2 + ddy ** 2) < thresh).sum(1)
    i = int(np.argmax(votes))
    a, b = matches[i]
    return (a[0] - b[0], a[1] - b[1]), matches[i]


# ----------------------------------------------------------------------------- B1
def pad_image(img, mx, my):
    mx = int(round(mx))
    my = int(round(my))
    py = (my, 0) if my >= 0 else (0, -my)
    px = (mx, 0) if mx >= 0 else (0, -mx)
    return np.pad(img, (py, px, (0, 0)), "constant")


def blend_geometry(shift, ref, wA_img, hA_img, wB_img, hB_img):
    """The scalar part of blend_two_images: swap, pads, overlap range (Python doubles)."""
    dx, dy = shift
    swapped = dx < 0
    if swapped:
        dx, dy = -dx, -dy
        ref = (ref[1], ref[0])
        wA_img, hA_img, wB_img, hB_img = wB_img, hB_img, wA_img, hA_img
    padA_x = wB_img - wA_img + ref[0][0] - ref[1][0]
    padB_x = ref[0][0] - ref[1][0]
    overlap = ref[1][0] - ref[0][0] + wA_img
    return swapped, dx, dy, padA_x, padB_x, overlap


def blend_two_images(shift, ref, imgA, imgB):
    swapped, dx, dy, padA_x, padB_x, overlap = blend_geometry(
        shift, ref, imgA.shape[1], imgA.shape[0], imgB.shape[1], imgB.shape[0])
    if swapped:
        imgA, imgB = imgB, imgA
    sa = pad_image(imgA, -padA_x, -dy)
    sb = pad_image(imgB, padB_x, dy)
    H = max(sa.shape[0], sb.shape[0])
    W = max(sa.shape[1], sb.shape[1])
    ca = np.zeros((H, W, 3), F32)
    cb = np.zeros((H, W, 3), F32)
    ca[:sa.shape[0], :sa.shape[1]] = sa
    cb[:sb.shape[0], :sb.shape[1]] = sb
    fa = (ca != 0).any(axis=(0, 2))
    fb = (cb != 0).any(axis=(0, 2))
    both = fa & fb
    rank = np.cumsum(both) - both
    out = np.where(fa[None, :, None], ca, cb)
    for c in np.nonzero(both)[0].tolist():
        alpha = rank[c] / overlap if overlap != 0 else 0
        out[:, c, :] = F32(1 - alpha) * ca[:, c, :] + F32(alpha) * cb[:, c, :]
    return out.astype(np.uint8)


def rectangle_crop(img, black_threshold=0, extra_margin=15):
    h = img.shape[0]
    gray = cv2_compat.bgr_to_gray_u8(img)
    ys, xs = np.nonzero(gray > black_threshold)
    if ys.size == 0:
        return img
    y0, y1 = max(0, ys.min() + extra_margin), min(h - 1, ys.max() - extra_margin)
    x0, x1 = xs.min(), xs.max()
    if y0 > y1 or x0 > x1:
        return img
    return img[y0:y1 + 1, x0:x1 + 1]


# ----------------------------------------------------------------------------- driver
def drift_correct(shifts):
    """Spread the accumulated vertical drift evenly over the pairs (:336-365)."""
    total_dy = 0
    for _, dy in shifts:
        total_dy = total_dy + dy
    n = len(shifts) + 1
    avg = total_dy / (n - 1) if n > 1 else 0
    return [(dx, dy - avg) for dx, dy in shifts]


def compose(cyl, shifts, pairs):
    """Second loop of run_panorama: sequential pad + blend (:369-381)."""
    mosaic = cyl[0].copy()
    for i in range(1, len(cyl)):
        frame = cyl[i]
        diff = mosaic.shape[0] - frame.shape[0]
        if diff != 0:
            frame = pad_image(frame, 0, diff)
        mosaic = blend_two_images(shifts[i - 1], pairs[i - 1], mosaic, frame)
    return mosaic


def pair_shift_sift(kA, dA, kB, dB, ransac_thr=3, desc_thresh=25000):
    return ransac(sift_matches(kA, dA, kB, dB, desc_thresh), ransac_thr)


def pair_shift_harris(fA, fB, ransac_thr=3, desc_thresh=1.0):
    (kA, dA), (kB, dB) = fA, fB
    return ransac(harris_matches(kA, dA, kB, dB, desc_thresh), ransac_thr)


def stitch(frames, focals, method="sift", margin=15, features=None):
    """Whole numeric pipeline for one sequence -> (cropped panorama, shifts, pairs, mosaic).

    Features are computed once per frame (the reference recomputes interior frames for
    both of their pairs; the features are a pure function of the frame, so the per-pair
    results are identical).
    """
    cyl = [cylindrical(f, fl) for f, fl in zip(frames, focals)]
    feats = features
    if feats is None:
        if method == "sift":
            feats = [sift.detect_and_describe(c) for c in cyl]
        else:
            feats = [harris.detect_and_describe(c) for c in cyl]
    shifts, pairs = [], []
    for i in range(len(cyl) - 1):
        if method == "sift":
            mv, pr = pair_shift_sift(*feats[i], *feats[i + 1])
        else:
            mv, pr = pair_shift_harris(feats[i], feats[i + 1])
        shifts.append(mv)
        pairs.append(pr)
    corrected = drift_correct(shifts)
    mosaic = compose(cyl, corrected, pairs)
    return rectangle_crop(mosaic, 0, margin), shifts, pairs, mosaic
