"""The visualiser's match + homography step on the device.

Reference: sift_visualizeUI.py:240-273 -- SIFT on two gray images, FLANN kNN-2, the Lowe
ratio test at 0.7, and ``cv2.findHomography(src, dst, cv2.RANSAC, 5.0)`` when there are more
than MIN_MATCH_COUNT = 10 good matches; the homography maps the query frame's outline into the
train frame (``cv2.perspectiveTransform``).

Here the chain is pano_sift_u8 -> pano_match_u8 (exact kNN-2) -> pano_pair_homography
(deterministic RANSAC, csrc/homography.hip).  ``find_pair_homographies`` is the batched
device entry point (many pairs, one launch chain); ``match_homography`` is the two-image call
the visualiser makes.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import PanoError, ptr

MIN_MATCH_COUNT = 10          # sift_visualizeUI.py:259


@dataclass
class PairHomography:
    H: np.ndarray | None           # 3 x 3 (None when status != "ok")
    good: np.ndarray               # [G, 2] (queryIdx, trainIdx) of the good matches, query order
    distance: np.ndarray           # [G] L2 distance of each good match (DMatch.distance)
    mask: np.ndarray               # [G] bool, inliers of H
    inliers: int
    hyp_inliers: int
    status: str                    # "ok" | "nomatch" | "overflow"


_STATUS = {_lib.PANO_OK: "ok", _lib.PANO_E_NOMATCH: "nomatch", _lib.PANO_E_OVERFLOW: "overflow"}


def find_pair_homographies(st, feats, pairs, ratio=0.7, reproj_thr=5.0,
                           min_match_count=MIN_MATCH_COUNT, n_hyp=2000, seed=0, desc_thresh=0.0,
                           readback=True):
    """Match every (a, b) pair of ``feats`` (a Stitcher's SIFT features) and fit a homography
    per pair on the device.  Returns the device records (and, with ``readback``, a list of
    PairHomography)."""
    T = st.torch
    kps, desc, counts = feats
    if st.method != "sift":
        raise PanoError(_lib.PANO_E_UNSUPPORTED, "homographies are fitted on SIFT features")
    P = len(pairs)
    cap = desc.shape[1]
    hp = np.ascontiguousarray(np.array(pairs, np.int32).reshape(-1))
    best = st._get("hm_best", (P, cap), T.int32)
    d1 = st._get("hm_d1", (P, cap), T.float32)
    d2 = st._get("hm_d2", (P, cap), T.float32)
    lib, c = st.ctx.lib, st.ctx.h
    if desc.dtype == T.uint8:
        norms = getattr(feats, "norms", None)
        if norms is None:
            norms = st.desc_norms(desc)
        st.ctx.check(lib.pano_match_u8(c, ptr(desc), ptr(norms), ptr(counts), cap, _lib.i32p(hp), P,
                                       ptr(best), ptr(d1), ptr(d2)))
    else:
        st.ctx.check(lib.pano_match(c, ptr(desc), ptr(counts), cap, _lib.i32p(hp), P, 2,
                                    ptr(best), ptr(d1), ptr(d2)))
    recs = st._get("hm_recs", (P, _lib.HOMOGRAPHY_NP.itemsize), T.uint8)
    mask = st._get("hm_mask", (P, cap), T.uint8)
    st.ctx.check(lib.pano_pair_homography(c, ptr(kps), ptr(counts), cap, _lib.i32p(hp), P, ptr(best),
                                          ptr(d1), ptr(d2), float(desc_thresh), float(ratio),
                                          float(reproj_thr), int(n_hyp), ctypes.c_uint64(seed),
                                          int(min_match_count), ptr(recs), ptr(mask)))
    if not readback:
        return recs, mask, (best, d1, d2)
    st.ctx.sync()
    r = recs.cpu().numpy().view(_lib.HOMOGRAPHY_NP).reshape(-1)
    cnt = counts.cpu().numpy()
    best_h, d1_h, d2_h, mask_h = best.cpu().numpy(), d1.cpu().numpy(), d2.cpu().numpy(), mask.cpu().numpy()
    out = []
    for p, (a, b) in enumerate(pairs):
        na, nb = min(max(int(cnt[a]), 0), cap), min(max(int(cnt[b]), 0), cap)
        bp, p1, p2 = best_h[p, :na], d1_h[p, :na].astype(np.float64), d2_h[p, :na].astype(np.float64)
        # the kernel's predicate (pair_compact): a valid neighbour and the visualiser's
        # m.distance < ratio * n.distance on float32 L2 distances
        ok = (bp >= 0) & (bp < nb)
        if desc_thresh > 0:
            ok &= d1_h[p, :na] < np.float32(desc_thresh)
        if ratio > 0:
            ok &= np.sqrt(d1_h[p, :na]).astype(np.float64) < ratio * np.sqrt(d2_h[p, :na]).astype(np.float64)
        qi = np.nonzero(ok)[0]
        G = len(qi)
        if G != int(r["n_matches"][p]):
            raise PanoError(_lib.PANO_E_HIP, "pano_pair_homography: good-match count disagrees")
        status = _STATUS.get(int(r["status"][p]), "error")
        out.append(PairHomography(
            H=r["H"][p].reshape(3, 3).copy() if status == "ok" else None,
            good=np.stack([qi, bp[qi]], 1).astype(np.int32),
            distance=np.sqrt(p1[qi]).astype(np.float32),
            mask=mask_h[p, :G].astype(bool),
            inliers=int(r["inliers"][p]), hyp_inliers=int(r["hyp_inliers"][p]), status=status))
    return out


def perspective_transform(pts, H):
    """cv2.perspectiveTransform for a [N, 1, 2] or [N, 2] point list (host arithmetic)."""
    H = np.asarray(H, np.float64).reshape(3, 3)
    p = np.asarray(pts, np.float64).reshape(-1, 2)
    q = np.c_[p, np.ones(len(p))] @ H.T
    return (q[:, :2] / q[:, 2:3]).reshape(np.shape(pts))


def match_homography(img1, img2, ratio=0.7, reproj_thr=5.0, min_match_count=MIN_MATCH_COUNT,
                     n_hyp=2000, seed=0):
    """sift_visualizeUI.py:240-273 without the Qt widgets: (kp1, kp2, PairHomography, outline)
    where ``outline`` is the query frame's corners mapped into the train frame (None without
    a homography)."""
    from .keypoint import from_records
    from .sift_impl import _frame_u8, _stitcher
    a, b = _frame_u8(img1), _frame_u8(img2)
    st = _stitcher(1.6, 3, 0.5, 5)
    feats = st.features_of([a, b])
    res = find_pair_homographies(st, feats, [(0, 1)], ratio, reproj_thr, min_match_count, n_hyp, seed)[0]
    kps, _, counts = feats
    cnt = counts.cpu().numpy()
    kp = [from_records(kps[i, :int(cnt[i])].cpu().numpy().view(_lib.KP_NP).reshape(-1)) for i in (0, 1)]
    outline = None
    if res.H is not None:
        h, w = a.shape[:2]
        corners = np.float32([[0, 0], [0, h - 1], [w - 1, h - 1], [w - 1, 0]]).reshape(-1, 1, 2)
        outline = perspective_transform(corners, res.H)
    return kp[0], kp[1], res, outline
