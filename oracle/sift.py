"""Vectorised numpy restatement of /root/reference/sift_impl.py -- TEST INFRASTRUCTURE.

Every stage keeps the reference's arithmetic (numpy 2.x NEP-50 promotion, half-even
rounding, f32/f64 mix) while replacing its per-pixel Python loops with array code.  The
stage boundaries are the reference's, so tests can compare stage by stage:

==================================  =================================================
oracle function                     reference (sift_impl.py)
==================================  =================================================
``to_gray_f32``                     :27-29
``base_image``                      generate_base_image :45-56
``n_octaves``                       compute_number_of_octaves :59-63
``level_sigmas``                    generate_gaussian_kernels :66-79
``gaussian_pyramid``                generate_gaussian_images :82-97
``dog_pyramid``                     generate_DoG_images :100-111
``extremum_mask`` / ``candidates``  find_scale_space_extrema :117-140 +
                                    is_pixel_an_extremum :143-163
``localize``                        localize_extremum_via_quadratic_fit :169-211
                                    (+ gradient/Hessian :217-240)
``orientations``                    compute_keypoints_with_orientations :246-293
``sort_dedup``                      compare_keypoints / remove_duplicate_keypoints :299-327
``to_input_size``                   convert_keypoints_to_input_image_size :333-343
``unpack_octave``                   :349-358
``descriptors``                     generate_descriptors :361-526
``detect_and_describe``             compute_keypoints_and_descriptors :15-39
==================================  =================================================

Keypoints are carried as a structured numpy array ``KP_DTYPE`` (float32 fields, as
cv2.KeyPoint stores them) instead of KeyPoint objects.
"""
from __future__ import annotations

import math

import numpy as np

from . import cv2_compat
from .numerics import F32, RAD2DEG_F32, norm_f32, sdot_tail

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i8")])
FLOAT_TOL = 1e-7


# ----------------------------------------------------------------------------- pyramid
def to_gray_f32(image: np.ndarray) -> np.ndarray:
    if image.ndim == 3 and image.shape[2] == 3:
        image = cv2_compat.bgr_to_gray_u8(image)
    return image.astype(F32)


def base_image(gray: np.ndarray, sigma=1.6, assumed_blur=0.5) -> np.ndarray:
    up = cv2_compat.resize(gray, (0, 0), fx=2, fy=2, interpolation=cv2_compat.INTER_LINEAR)
    s = float(np.sqrt(max(sigma ** 2 - (2 * assumed_blur) ** 2, 0.01)))
    return cv2_compat.GaussianBlur(up, (0, 0), sigmaX=s, sigmaY=s)


def n_octaves(shape) -> int:
    return int(np.round(np.log(min(shape)) / np.log(2) - 1))


def level_sigmas(sigma=1.6, num_intervals=3) -> np.ndarray:
    """Incremental blur per level; level 0 is the octave base (sigma itself)."""
    k = 2 ** (1.0 / num_intervals)
    out = np.zeros(num_intervals + 3)
    out[0] = sigma
    for i in range(1, num_intervals + 3):
        prev = (k ** (i - 1)) * sigma
        out[i] = np.sqrt((k * prev) ** 2 - prev ** 2)
    return out


def gaussian_pyramid(base: np.ndarray, octaves: int, sigmas: np.ndarray):
    pyr = []
    img = base
    for _ in range(octaves):
        levels = [img]
        for s in sigmas[1:]:
            img = cv2_compat.GaussianBlur(img, (0, 0), sigmaX=s, sigmaY=s)
            levels.append(img)
        pyr.append(levels)
        src = levels[-3]
        img = cv2_compat.resize(src, (src.shape[1] // 2, src.shape[0] // 2),
                                interpolation=cv2_compat.INTER_NEAREST)
    return pyr


def dog_pyramid(gpyr):
    return [[(b - a).astype(F32) for a, b in zip(lv, lv[1:])] for lv in gpyr]


# ----------------------------------------------------------------------------- extrema
def extremum_mask(prev, curr, nxt, thresh, border):
    """Boolean mask of is_pixel_an_extremum over the interior [border, n-border)."""
    h, w = curr.shape
    ys = slice(border, h - border)
    xs = slice(border, w - border)
    v = curr[ys, xs]
    big = np.abs(v) > thresh
    pos = v > 0
    ge = np.ones_like(big)
    le = np.ones_like(big)
    for img in (prev, curr, nxt):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                if img is curr and dy == 0 and dx == 0:
                    continue
                nb = img[border + dy:h - border + dy, border + dx:w - border + dx]
                ge &= v >= nb
                le &= v <= nb
    m = np.zeros((h, w), bool)
    m[ys, xs] = big & np.where(pos, ge, le)
    return m


def candidates(dogs, num_intervals=3, border=5, contrast_threshold=0.04):
    """All (octave, layer, y, x) extrema in the reference's scan order."""
    thresh = np.floor(0.5 * contrast_threshold / num_intervals * 255)
    out = []
    for o, d in enumerate(dogs):
        for i in range(len(d) - 2):
            m = extremum_mask(d[i], d[i + 1], d[i + 2], thresh, border)
            ys, xs = np.nonzero(m)
            for y, x in zip(ys.tolist(), xs.tolist()):
                out.append((o, i + 1, y, x))
    return out


def _cube(d, layer, y, x):
    c = np.stack([d[layer - 1][y - 1:y + 2, x - 1:x + 2],
                  d[layer][y - 1:y + 2, x - 1:x + 2],
                  d[layer + 1][y - 1:y + 2, x - 1:x + 2]]).astype(F32)
    return (c / 255.0).astype(F32)


def _grad_hess(c):
    h = F32(0.5)
    q = F32(0.25)
    g = np.array([h * (c[1, 1, 2] - c[1, 1, 0]),
                  h * (c[1, 2, 1] - c[1, 0, 1]),
                  h * (c[2, 1, 1] - c[0, 1, 1])], F32)
    v2 = F32(2) * c[1, 1, 1]
    dxx = c[1, 1, 2] - v2 + c[1, 1, 0]
    dyy = c[1, 2, 1] - v2 + c[1, 0, 1]
    dss = c[2, 1, 1] - v2 + c[0, 1, 1]
    dxy = q * (c[1, 2, 2] - c[1, 2, 0] - c[1, 0, 2] + c[1, 0, 0])
    dxs = q * (c[2, 1, 2] - c[2, 1, 0] - c[0, 1, 2] + c[0, 1, 0])
    dys = q * (c[2, 2, 1] - c[2, 0, 1] - c[0, 2, 1] + c[0, 0, 1])
    H = np.array([[dxx, dxy, dxs], [dxy, dyy, dys], [dxs, dys, dss]], F32)
    return g, H


def localize(x, y, layer, octave, dog_oct, num_intervals=3, sigma=1.6,
             contrast_threshold=0.04, border=5, eigen_ratio=10, max_iter=5):
    """Quadratic-fit refinement; returns (kp record, layer) or None.

    Keeps the reference's quirk: after ``max_iter`` non-converged steps the last cube /
    gradient / Hessian are used with the moved x, y, layer (sift_impl.py:175-195).
    """
    hgt, wid = dog_oct[0].shape
    for _ in range(max_iter):
        c = _cube(dog_oct, layer, y, x)
        g, H = _grad_hess(c)
        upd = (-np.linalg.lstsq(H, g, rcond=None)[0]).astype(F32)
        if np.all(np.abs(upd) < 0.5):
            break
        x += int(np.round(upd[0]))
        y += int(np.round(upd[1]))
        layer += int(np.round(upd[2]))
        if y < border or y >= hgt - border or x < border or x >= wid - border \
                or layer < 1 or layer > num_intervals:
            return None
    val = F32(c[1, 1, 1] + F32(F32(0.5) * sdot_tail(g, upd)))
    if abs(val) * F32(num_intervals) < F32(contrast_threshold):
        return None
    tr = F32(H[0, 0] + H[1, 1])
    det = F32(np.linalg.det(H[:2, :2]))
    if det <= 0 or F32(eigen_ratio) * F32(tr * tr) >= F32((eigen_ratio + 1) ** 2) * det:
        return None
    scale_o = 2 ** octave
    kp = np.zeros((), KP_DTYPE)
    kp["x"] = F32((x + upd[0]) * F32(scale_o))
    kp["y"] = F32((y + upd[1]) * F32(scale_o))
    kp["octave"] = octave + layer * 256 + int(np.round(F32(F32(upd[2] + F32(0.5)) * F32(255)))) * 65536
    expo = F32(F32(layer + upd[2]) / F32(num_intervals))
    kp["size"] = F32(F32(F32(sigma) * F32(2 ** expo)) * F32(2 ** (octave + 1)))
    kp["response"] = abs(val)
    kp["angle"] = -1.0
    return kp, layer


# ----------------------------------------------------------------------------- orientation
def orientations(kp, octave, gimg, radius_factor=3, num_bins=36, peak_ratio=0.8,
                 scale_factor=1.5):
    """36-bin orientation histogram -> list of (angle) for each accepted peak."""
    size = float(kp["size"])
    scale = F32(F32(scale_factor * size) / F32(2 ** (octave + 1)))
    radius = int(np.round(F32(radius_factor) * scale))
    wfac = F32(F32(-0.5) / F32(scale * scale))
    cy = int(np.round(F32(F32(kp["y"]) / F32(2 ** octave))))
    cx = int(np.round(F32(F32(kp["x"]) / F32(2 ** octave))))
    dy, dx = np.mgrid[-radius:radius + 1, -radius:radius + 1]
    dy = dy.ravel()
    dx = dx.ravel()
    yy = cy + dy
    xx = cx + dx
    h, w = gimg.shape
    ok = (xx > 0) & (xx < w - 1) & (yy > 0) & (yy < h - 1)
    dy, dx, yy, xx = dy[ok], dx[ok], yy[ok], xx[ok]
    gx = gimg[yy, xx + 1] - gimg[yy, xx - 1]
    gy = gimg[yy - 1, xx] - gimg[yy + 1, xx]
    mag = np.sqrt(gx * gx + gy * gy)
    ang = np.remainder(np.arctan2(gy, gx) * RAD2DEG_F32, F32(360))
    wgt = np.exp(wfac * (dx * dx + dy * dy).astype(F32))
    idx = np.round(ang * F32(num_bins) / F32(360.0)).astype(np.int64) % num_bins
    hist = np.zeros(num_bins)
    np.add.at(hist, idx, (wgt * mag).astype(np.float64))
    sm = np.empty(num_bins)
    for i in range(num_bins):
        sm[i] = (6 * hist[i] + 4 * (hist[i - 1] + hist[(i + 1) % num_bins])
                 + hist[i - 2] + hist[(i + 2) % num_bins]) / 16.0
    mx = sm.max()
    angles = []
    for p in range(num_bins):
        l = sm[(p - 1) % num_bins]
        r = sm[(p + 1) % num_bins]
        if not (sm[p] > l and sm[p] > r):
            continue
        if sm[p] < peak_ratio * mx:
            continue
        interp = np.remainder(p + 0.5 * (l - r) / (l - 2 * sm[p] + r), num_bins)
        a = 360.0 - interp * 360.0 / num_bins
        if abs(a - 360.0) < FLOAT_TOL:
            a = 0
        angles.append(float(a))
    return angles


# ----------------------------------------------------------------------------- keypoints
def find_keypoints(gpyr, dogs, num_intervals=3, sigma=1.6, border=5, contrast_threshold=0.04):
    """find_scale_space_extrema: candidates -> localize -> orientations (scan order)."""
    out = []
    for (o, i, y, x) in candidates(dogs, num_intervals, border, contrast_threshold):
        r = localize(x, y, i, o, dogs[o], num_intervals, sigma, contrast_threshold, border)
        if r is None:
            continue
        kp, layer = r
        for a in orientations(kp, o, gpyr[o][layer]):
            k = kp.copy()
            k["angle"] = a
            out.append(k)
    return np.array(out, KP_DTYPE) if out else np.zeros(0, KP_DTYPE)


def sort_dedup(kps: np.ndarray) -> np.ndarray:
    """Stable sort on (x, y, -size, angle, -response), drop repeated (pt, size, angle)."""
    if len(kps) < 2:
        return kps
    order = sorted(range(len(kps)), key=lambda i: (float(kps[i]["x"]), float(kps[i]["y"]),
                                                    -float(kps[i]["size"]), float(kps[i]["angle"]),
                                                    -float(kps[i]["response"])))
    s = kps[np.array(order)]
    keep = [0]
    for i in range(1, len(s)):
        a, b = s[keep[-1]], s[i]
        if (a["x"], a["y"], a["size"], a["angle"]) != (b["x"], b["y"], b["size"], b["angle"]):
            keep.append(i)
    return s[np.array(keep)]


def to_input_size(kps: np.ndarray) -> np.ndarray:
    k = kps.copy()
    k["x"] = (k["x"].astype(np.float64) * 0.5).astype(F32)
    k["y"] = (k["y"].astype(np.float64) * 0.5).astype(F32)
    k["size"] = (k["size"].astype(np.float64) * 0.5).astype(F32)
    o = k["octave"]
    k["octave"] = (o & ~255) | ((o - 1) & 255)
    return k


def unpack_octave(octave_field: int):
    octave = octave_field & 255
    layer = (octave_field >> 8) & 255
    if octave >= 128:
        octave |= -128
    scale = 1 / F32(1 << octave) if octave >= 0 else F32(1 << -octave)
    return octave, layer, F32(scale)


# ----------------------------------------------------------------------------- descriptors
def descriptor(kp, gpyr, window_width=4, num_bins=8, scale_multiplier=3, max_value=0.2):
    octv, lyr, scl = unpack_octave(int(kp["octave"]))
    img = gpyr[octv + 1][lyr]
    rows, cols = img.shape
    px = int(np.round(np.float64(scl) * np.float64(kp["x"])))
    py = int(np.round(np.float64(scl) * np.float64(kp["y"])))
    angle = 360.0 - float(kp["angle"])
    rad = np.deg2rad(angle)
    cos_a, sin_a = np.cos(rad), np.sin(rad)
    hist_w = F32(F32(scale_multiplier * 0.5 * scl) * F32(kp["size"]))
    half = int(np.round(np.float64(hist_w) * np.sqrt(2) * (window_width + 1) * 0.5))
    half = min(half, int(np.sqrt(rows ** 2 + cols ** 2)))
    ys, xs = np.mgrid[-half:half + 1, -half:half + 1]
    ys = ys.ravel()
    xs = xs.ravel()
    rr = py + ys
    cc = px + xs
    ok = (rr > 0) & (rr < rows - 1) & (cc > 0) & (cc < cols - 1)
    if not ok.any():
        return np.zeros(128, F32)
    rr, cc, ys, xs = rr[ok], cc[ok], ys[ok], xs[ok]
    gx = img[rr, cc + 1] - img[rr, cc - 1]
    gy = img[rr - 1, cc] - img[rr + 1, cc]
    mag = np.sqrt(gx * gx + gy * gy)
    ori = np.remainder(np.arctan2(gy, gx) * RAD2DEG_F32, F32(360))
    rrot = xs * sin_a + ys * cos_a
    crot = xs * cos_a - ys * sin_a
    hw64 = np.float64(hist_w)
    rbin = (rrot / hw64) + 0.5 * window_width - 0.5
    cbin = (crot / hw64) + 0.5 * window_width - 0.5
    inb = (rbin > -1.0) & (rbin < window_width) & (cbin > -1.0) & (cbin < window_width)
    if not inb.any():
        return np.zeros(128, F32)
    rbin, cbin, mag, ori, rrot, crot = rbin[inb], cbin[inb], mag[inb], ori[inb], rrot[inb], crot[inb]
    wmul = -0.5 / ((0.5 * window_width) ** 2)
    wgt = np.exp(wmul * ((rrot / hw64) ** 2 + (crot / hw64) ** 2))
    wm = wgt * mag.astype(np.float64)
    ob = ((ori - F32(angle)) * F32(num_bins / 360.0)).astype(F32)
    ob = np.remainder(ob, F32(num_bins))
    r0 = np.floor(rbin).astype(np.int64)
    c0 = np.floor(cbin).astype(np.int64)
    o0 = np.floor(ob).astype(np.int64) % num_bins
    rf = rbin - r0
    cf = cbin - c0
    of = ob.astype(np.float64) - o0
    c1 = wm * rf
    c0w = wm - c1
    parts = ((c0w * (1 - cf), 0, 0), (c0w * cf, 0, 1), (c1 * (1 - cf), 1, 0), (c1 * cf, 1, 1))
    t = np.zeros((window_width + 2, window_width + 2, num_bins), F32)
    for val, dr, dc in parts:
        np.add.at(t, (r0 + dr + 1, c0 + dc + 1, o0 % num_bins), val * (1 - of))
        np.add.at(t, (r0 + dr + 1, c0 + dc + 1, (o0 + 1) % num_bins), val * of)
    v = t[1:-1, 1:-1, :].ravel().copy()
    thr = F32(norm_f32(v) * F32(max_value))
    v[v > thr] = thr
    nv = norm_f32(v)
    if nv < F32(FLOAT_TOL):
        nv = F32(FLOAT_TOL)
    v = (v / nv).astype(F32)
    v = np.round(F32(512) * v)
    return np.clip(v, 0, 255).astype(F32)


def descriptors(kps, gpyr):
    if len(kps) == 0:
        return np.zeros((0, 128), F32)
    return np.stack([descriptor(k, gpyr) for k in kps]).astype(F32)


# ----------------------------------------------------------------------------- driver
def detect_and_describe(image, sigma=1.6, num_intervals=3, assumed_blur=0.5, border=5,
                        return_stages=False):
    gray = to_gray_f32(image)
    base = base_image(gray, sigma, assumed_blur)
    no = n_octaves(base.shape)
    gp = gaussian_pyramid(base, no, level_sigmas(sigma, num_intervals))
    dp = dog_pyramid(gp)
    raw = find_keypoints(gp, dp, num_intervals, sigma, border)
    kps = to_input_size(sort_dedup(raw))
    desc = descriptors(kps, gp)
    if return_stages:
        return kps, desc, {"gauss": gp, "dog": dp, "raw": raw}
    return kps, desc
