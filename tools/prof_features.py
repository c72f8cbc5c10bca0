#!/usr/bin/env python3
"""Run the SIFT stitch N times (for rocprofv3 counter collection).

    python tools/prof_features.py N [parrington|synthetic]
synthetic = BASELINE config 5's 1080p frames, 19 frames (the bench's N=1 weak workload)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from vfx_image_stitching_amd import data  # noqa: E402
from vfx_image_stitching_amd.pipeline import Stitcher  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
work = sys.argv[2] if len(sys.argv) > 2 else "parrington"
if work == "synthetic":
    frames, focals, _ = data.synthetic_sequence(n_frames=144, h=1080, w=1920, start=0, count=19)
    margin, cap = 15, 65536
else:
    names, frames, focals, margin = data.load_set(work)
    cap = 4096
st = Stitcher("sift", cap=cap, match=os.environ.get("PANO_MATCH"))  # None: the default (u8)
d = st.upload(frames)
for _ in range(n):
    try:
        st.run(d, focals, margin=margin)
    except Exception as e:          # ablation builds produce garbage features
        print("run failed:", e)
        torch.cuda.synchronize()
torch.cuda.synchronize()
print("done")
