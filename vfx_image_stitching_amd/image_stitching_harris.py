"""Drop-in for /root/reference/image_stitching_harris.py (Harris path on the GPU).

compute_keypoints_and_descriptors_harris (:187-214), simple_match (:219-240),
ransac (:242-271) and compute_shift_harris (:273-285) keep their signatures; the warp /
blend / crop helpers are shared with the SIFT shim (AST-identical in the reference).
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .stitching import (blend_two_images, cylindrical_projection, pad_image,  # noqa: F401
                        ransac, read_pano_data, rectangle_crop)
from .stitching import run_panorama as _run

_st = {}


def _stitcher(max_points=200):
    from .pipeline import Stitcher
    st = _st.get(max_points)
    if st is None:
        st = _st[max_points] = Stitcher("harris", max_points=max_points)
    return st


def compute_keypoints_and_descriptors_harris(img_bgr, max_points=200):
    st = _stitcher(max_points)
    xy, desc, counts = st.features(st.upload(np.ascontiguousarray(img_bgr, np.uint8)[None]))
    n = int(counts.cpu()[0])
    pts = xy[0, :n].cpu().numpy()
    kps = [(int(x), int(y)) for x, y in pts]
    return kps, desc[0, :n].cpu().numpy().astype(np.float32)


def simple_match(kpsA, descA, kpsB, descB, desc_thresh=1.0):
    """NN on the GPU with the OpenBLAS sdot distance order; strict '<' first minimum."""
    import torch
    st = _stitcher()
    if len(descA) == 0:
        return []
    nA, nB = len(descA), len(descB)
    cap = max(nA, nB, 1)
    d = np.zeros((2, cap, 128), np.float32)
    d[0, :nA] = descA
    d[1, :nB] = descB
    desc = torch.from_numpy(d).to(st.device)
    counts = torch.tensor([nA, nB], dtype=torch.int32, device=st.device)
    best = torch.empty((1, cap), dtype=torch.int32, device=st.device)
    d1 = torch.empty((1, cap), dtype=torch.float32, device=st.device)
    d2 = torch.empty_like(d1)
    hp = np.array([0, 1], np.int32)
    st.ctx.check(st.ctx.lib.pano_match(st.ctx.h, _lib.ptr(desc), _lib.ptr(counts), cap,
                                       _lib.i32p(hp), 1, 0, _lib.ptr(best), _lib.ptr(d1),
                                       _lib.ptr(d2)))
    b = best.cpu().numpy()[0]
    dist = d1.cpu().numpy()[0]
    return [(kpsA[i], kpsB[b[i]]) for i in range(nA) if b[i] >= 0 and dist[i] < np.float32(desc_thresh)]


def compute_shift_harris(imgA, imgB, ransac_thr, desc_thresh):
    st = _stitcher(200)
    st.ransac_thr = float(ransac_thr)
    st.desc_thresh = float(desc_thresh)
    # frames may differ in shape (each frame's corners are its own: :277-278)
    feats = st.features_of([np.asarray(imgA, np.uint8), np.asarray(imgB, np.uint8)])
    recs, _ = st.pair_records(feats, [(0, 1)])
    r = recs.cpu().numpy().view(_lib.PAIR_NP).reshape(-1)[0]
    if r["status"] != _lib.PANO_OK:
        return (0, 0), None
    return (int(r["dx"]), int(r["dy"])), ((int(r["xA"]), int(r["yA"])), (int(r["xB"]), int(r["yB"])))


def run_panorama(folder_path=".", pano_file=None, margin=15, **kw):
    return _run(folder_path, pano_file, margin, method="harris", **kw)
