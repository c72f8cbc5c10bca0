#!/usr/bin/env python3
"""Run the parrington SIFT pipeline N times (for rocprofv3 counter collection)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from vfx_image_stitching_amd import data  # noqa: E402
from vfx_image_stitching_amd.pipeline import Stitcher  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
names, frames, focals, margin = data.load_set("parrington")
st = Stitcher("sift", match=os.environ.get("PANO_MATCH"))     # None: the Stitcher default (u8)
d = st.upload(frames)
for _ in range(n):
    try:
        st.run(d, focals, margin=margin)
    except Exception as e:          # ablation builds (PANO_BLUR_DBG) produce garbage features
        print("run failed:", e)
        torch.cuda.synchronize()
torch.cuda.synchronize()
print("done")
