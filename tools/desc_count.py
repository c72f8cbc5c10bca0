#!/usr/bin/env python3
"""Lane occupancy of the descriptor's column walk (diagnostics build, PANO_DESC_COUNT=1):
    tools/ab_variant.sh dcount -DPANO_DESC_COUNT=1
    PANO_LIB=tools/ab/libpano_dcount.so python tools/desc_count.py [parrington|synthetic]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from vfx_image_stitching_amd import data  # noqa: E402
from vfx_image_stitching_amd.pipeline import Stitcher  # noqa: E402

work = sys.argv[1] if len(sys.argv) > 1 else "parrington"
if work == "synthetic":
    frames, focals, _ = data.synthetic_sequence(n_frames=144, h=1080, w=1920, start=0, count=19)
else:
    _, frames, focals, _ = data.load_set("parrington")
st = Stitcher("sift", cap=32768 if work == "synthetic" else 4096)
cyl, _ = st.cylindrical(st.upload(frames), focals)
st.features(cyl)
torch.cuda.synchronize()
fn = st.ctx.lib.pano_dbg_desc_count
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_uint64 * 8)()
fn(buf, 1)
st.features(cyl)
torch.cuda.synchronize()
fn(buf, 0)
cand, passed, blocks, steps, lanes, kps = list(buf)[:6]
print(f"{work}: keypoints {kps}, wave steps {steps}, active lanes per step {lanes / max(steps, 1):.1f}, "
      f"candidate lane-samples {cand}, passing {passed} ({passed / max(cand, 1):.1%}), "
      f"sample blocks executed {blocks}, lanes binning per executed block {passed / max(blocks, 1):.1f} of 64")
