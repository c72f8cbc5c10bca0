"""Drop-in for /root/reference/image_stitching_sift.py (per-pair loop + warp/blend on GPU).

Same function names and signatures; ``run_panorama`` takes its three interactive answers
as arguments.  compute_shift_sift (image_stitching_sift.py:52-83) extracts both frames'
features in one batched pano_sift_u8 launch (byte descriptors), matches with the exact i8
MFMA distance GEMM (pano_match_u8: v_mfma_i32_32x32x32_i8 on the descriptor bytes - 128,
integer distances, first-index ties) and votes the translation on the GPU.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .sift_impl import compute_keypoints_and_descriptors  # noqa: F401  (reference import)
from .stitching import (blend_two_images, cylindrical_projection, pad_image,  # noqa: F401
                        ransac, read_pano_data, rectangle_crop)
from .stitching import run_panorama as _run


def compute_shift_sift(imgA, imgB, ransac_thr=3, desc_thresh=25000):
    """Frames may differ in shape: the reference extracts each frame's features on its own
    (image_stitching_sift.py:59-60); so does features_of."""
    from .sift_impl import _frame_u8, _stitcher
    st = _stitcher(1.6, 3, 0.5, 5)
    st.ransac_thr = float(ransac_thr)
    st.desc_thresh = float(desc_thresh)
    feats = st.features_of([_frame_u8(imgA), _frame_u8(imgB)])
    recs, _ = st.pair_records(feats, [(0, 1)])
    r = recs.cpu().numpy().view(_lib.PAIR_NP).reshape(-1)[0]
    if r["status"] == _lib.PANO_E_OVERFLOW:
        raise _lib.PanoError(_lib.PANO_E_OVERFLOW, "keypoint capacity exceeded")
    if r["status"] != _lib.PANO_OK:
        return (0, 0), None
    return (float(r["dx"]), float(r["dy"])), ((float(r["xA"]), float(r["yA"])),
                                              (float(r["xB"]), float(r["yB"])))


def run_panorama(folder_path=".", pano_file=None, margin=15, **kw):
    return _run(folder_path, pano_file, margin, method="sift", **kw)
