"""Restatement of the visualiser's match + homography step -- TEST INFRASTRUCTURE ONLY.

Reference: sift_visualizeUI.py:247-266 -- FLANN kNN-2 (kd-trees=5, checks=50), the Lowe ratio
test ``m.distance < 0.7 * n.distance``, and ``cv2.findHomography(src, dst, cv2.RANSAC, 5.0)``
when ``len(good) > MIN_MATCH_COUNT`` (10).

OpenCV is not installed, and both of its pieces here are randomised (FLANN's kd-trees, the
RANSAC sampler), so the product path (csrc/homography.hip) fixes a deterministic
algorithm and this module restates exactly that algorithm in numpy:

``knn2``            exact brute-force two nearest neighbours, squared L2 (FLANN approximates)
``good_matches``    float32 sqrt(d1) < ratio * sqrt(d2) (the matcher's L2 distances, Python floats)
``sample``          splitmix64(seed ^ pair << 48 ^ hyp << 16 ^ draw) mod K, distinct indices
``good_sample``     cv2 HomographyEstimatorCallback::checkSubset: no collinear triple, equal
                    triangle orientations in source and destination
``dlt4``            the 4-point DLT with h33 = 1 (8 x 8, Gaussian elimination, partial pivot)
``find_homography`` score = #{err^2 <= thr^2}; first best; Hartley-normalised least-squares
                    refit over its inliers; the refit's inliers

Parity with cv2.findHomography is "unpinned" (cv2 refines with Levenberg-Marquardt on the
reprojection error); the tests pin the kernel to this module and both to known homographies.
"""
from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1


def splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def sample(seed: int, pair: int, hyp: int, K: int) -> list[int]:
    idx, draw = [], 0
    base = (seed ^ (pair << 48) ^ (hyp << 16)) & M64
    while len(idx) < 4:
        c = splitmix64(base ^ draw) % K
        draw += 1
        if c not in idx:
            idx.append(c)
    return idx


def knn2(desc_a: np.ndarray, desc_b: np.ndarray):
    """Exact kNN-2 on squared L2 (integer descriptors: exact in int64)."""
    a = desc_a.astype(np.int64)
    b = desc_b.astype(np.int64)
    d = (a * a).sum(1)[:, None] + (b * b).sum(1)[None, :] - 2 * a @ b.T
    order = np.argsort(d, axis=1, kind="stable")
    rows = np.arange(len(a))
    best = order[:, 0]
    d1 = d[rows, best]
    d2 = d[rows, order[:, 1]] if b.shape[0] > 1 else np.full(len(a), np.inf)
    return best.astype(np.int32), d1.astype(np.float32), np.asarray(d2, np.float32)


def good_matches(best, d1, d2, ratio=0.7, desc_thresh=0.0):
    """Indices i of the good matches in query order (the visualiser's ``good`` list)."""
    d1 = np.asarray(d1, np.float32)
    d2 = np.asarray(d2, np.float32)
    ok = np.asarray(best) >= 0
    if desc_thresh > 0:
        ok &= d1 < np.float32(desc_thresh)
    if ratio > 0:
        # sift_visualizeUI.py:252-257: m.distance < 0.7 * n.distance, the matcher's float32
        # L2 distances (sqrt of the squared distance) compared as Python floats
        ok &= np.sqrt(d1).astype(np.float64) < ratio * np.sqrt(d2).astype(np.float64)
    return np.nonzero(ok)[0]


def _cross(a, b, c):
    return (b[0] - a[0]) * (c[1] - a[1]) - (b[1] - a[1]) * (c[0] - a[0])


def good_sample(s, d) -> bool:
    for t in ((0, 1, 2), (1, 2, 3), (2, 3, 0), (3, 0, 1)):
        cs = _cross(s[t[0]], s[t[1]], s[t[2]])
        cd = _cross(d[t[0]], d[t[1]], d[t[2]])
        if abs(cs) < 1e-6 or abs(cd) < 1e-6:
            return False
        if (cs > 0) != (cd > 0):
            return False
    return True


def solve_gauss(A, b):
    """Gaussian elimination with partial pivoting; None when (numerically) singular."""
    A = np.array(A, np.float64)
    b = np.array(b, np.float64)
    n = len(b)
    amax = np.abs(A).max()
    if not amax > 0:
        return None
    for c in range(n):
        p = c + int(np.argmax(np.abs(A[c:, c])))
        if not abs(A[p, c]) > 1e-12 * amax:
            return None
        if p != c:
            A[[c, p]] = A[[p, c]]
            b[[c, p]] = b[[p, c]]
        for r in range(c + 1, n):
            f = A[r, c] / A[c, c]
            A[r, c:] -= f * A[c, c:]
            b[r] -= f * b[c]
    x = np.zeros(n)
    for r in range(n - 1, -1, -1):
        x[r] = (b[r] - A[r, r + 1:] @ x[r + 1:]) / A[r, r]
    return x


def dlt4(s, d):
    A = np.zeros((8, 8))
    b = np.zeros(8)
    for k in range(4):
        x, y = s[k]
        u, v = d[k]
        A[2 * k] = [x, y, 1, 0, 0, 0, -u * x, -u * y]
        A[2 * k + 1] = [0, 0, 0, x, y, 1, -v * x, -v * y]
        b[2 * k], b[2 * k + 1] = u, v
    h = solve_gauss(A, b)
    return None if h is None else np.append(h, 1.0)


def reproj_err2(H, S, D):
    w = H[6] * S[:, 0] + H[7] * S[:, 1] + H[8]
    u = (H[0] * S[:, 0] + H[1] * S[:, 1] + H[2]) / w
    v = (H[3] * S[:, 0] + H[4] * S[:, 1] + H[5]) / w
    return (u - D[:, 0]) ** 2 + (v - D[:, 1]) ** 2


def hypothesis_scores(S, D, n_hyp=2000, seed=0, pair=0, thr=5.0):
    """Inlier count of each hypothesis (-1: degenerate sample or singular system)."""
    K = len(S)
    thr2 = thr * thr
    scores = np.full(n_hyp, -1, np.int64)
    for h in range(n_hyp):
        idx = sample(seed, pair, h, K)
        s4, d4 = S[idx], D[idx]
        if not good_sample(s4, d4):
            continue
        H = dlt4(s4, d4)
        if H is None:
            continue
        scores[h] = int((reproj_err2(H, S, D) <= thr2).sum())
    return scores


def refit(H, S, D, thr=5.0):
    """Hartley-normalised linear least squares (h33' = 1) over the inliers of H."""
    m = reproj_err2(H, S, D) <= thr * thr
    s, d = S[m], D[m]
    ms, md = s.mean(0), d.mean(0)
    ds = np.sqrt(((s - ms) ** 2).sum(1)).mean()
    dd = np.sqrt(((d - md) ** 2).sum(1)).mean()
    ks = np.sqrt(2.0) / ds if ds > 0 else 1.0
    kd = np.sqrt(2.0) / dd if dd > 0 else 1.0
    x, y = ((s - ms) * ks).T
    u, v = ((d - md) * kd).T
    z, o = np.zeros_like(x), np.ones_like(x)
    r0 = np.stack([x, y, o, z, z, z, -u * x, -u * y, u], 1)
    r1 = np.stack([z, z, z, x, y, o, -v * x, -v * y, v], 1)
    M = r0.T @ r0 + r1.T @ r1
    h = solve_gauss(M[:8, :8], M[:8, 8])
    if h is None:
        return H
    Hn = np.append(h, 1.0).reshape(3, 3)
    Ts = np.array([[ks, 0, -ks * ms[0]], [0, ks, -ks * ms[1]], [0, 0, 1]])
    Ti = np.array([[1 / kd, 0, md[0]], [0, 1 / kd, md[1]], [0, 0, 1]])
    Hf = Ti @ Hn @ Ts
    if not abs(Hf[2, 2]) > 1e-300:
        return H
    return (Hf / Hf[2, 2]).reshape(-1)


def find_homography(S, D, thr=5.0, n_hyp=2000, seed=0, pair=0, min_good=10):
    """-> dict(H [9] or None, hyp, hyp_inliers, inliers, mask [K] bool, status)."""
    S = np.asarray(S, np.float64).reshape(-1, 2)
    D = np.asarray(D, np.float64).reshape(-1, 2)
    K = len(S)
    out = dict(H=None, hyp=-1, hyp_inliers=0, inliers=0, mask=np.zeros(K, bool), n_matches=K,
               status="nomatch")
    if K <= min_good or K < 4:
        return out
    scores = hypothesis_scores(S, D, n_hyp, seed, pair, thr)
    hv = int(scores.max())
    out["hyp_inliers"] = max(hv, 0)
    if hv < 4:
        return out
    hi = int(np.argmax(scores))                      # first best
    idx = sample(seed, pair, hi, K)
    H = refit(dlt4(S[idx], D[idx]), S, D, thr)
    mask = reproj_err2(H, S, D) <= thr * thr
    out.update(H=H, hyp=hi, inliers=int(mask.sum()), mask=mask, status="ok")
    return out


def perspective_transform(pts, H):
    """cv2.perspectiveTransform for an [N, 2] point list (sift_visualizeUI.py:268-273)."""
    H = np.asarray(H, np.float64).reshape(3, 3)
    p = np.asarray(pts, np.float64).reshape(-1, 2)
    q = np.c_[p, np.ones(len(p))] @ H.T
    return q[:, :2] / q[:, 2:3]
