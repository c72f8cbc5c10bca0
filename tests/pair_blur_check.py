"""Subprocess body of tests/test_gpu_parity.py::test_fused_pair_blur_bit_exact: the fused
level-pair blur (PANO_BLUR_PAIR, read once per process) against the oracle's pyramid."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from oracle import sift as osift  # noqa: E402
from oracle import stitch as ostitch  # noqa: E402
from vfx_image_stitching_amd import _lib, data  # noqa: E402
from vfx_image_stitching_amd.pipeline import Stitcher  # noqa: E402

names, frames, focals, _ = data.load_set("parrington")
cyl = np.stack([ostitch.cylindrical(frames[i], focals[i]) for i in range(2)])
st = Stitcher("sift")
dev = st.upload(cyl)
ctx = st.ctx
ctx.check(ctx.lib.pano_sift_pyramid(ctx.h, _lib.ptr(dev), 2, dev.shape[1], dev.shape[2], ctypes.byref(st.params)))
_, _, stg = osift.detect_and_describe(cyl[0], return_stages=True)
bad = []
for o in range(len(stg["gauss"])):
    h, w = ctypes.c_int32(), ctypes.c_int32()
    ctx.check(ctx.lib.pano_sift_level_shape(ctx.h, o, ctypes.byref(h), ctypes.byref(w), None))
    for dog, levels in ((0, stg["gauss"][o]), (1, stg["dog"][o])):
        for lv, ref in enumerate(levels):
            out = torch.empty((h.value, w.value), dtype=torch.float32, device=st.device)
            ctx.check(ctx.lib.pano_sift_copy_level(ctx.h, 0, o, lv, dog, _lib.ptr(out)))
            if not np.array_equal(out.cpu().numpy(), ref):
                bad.append((o, lv, dog))
print("pair blur", os.environ.get("PANO_BLUR_PAIR"), os.environ.get("PANO_BLUR_PAIR_TT"), "mismatches", bad)
sys.exit(1 if bad else 0)
