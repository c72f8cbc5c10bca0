#!/usr/bin/env python3
"""Per-class kernel times of the SIFT feature stage alone (no matching, so timing ablation
builds whose features are garbage still run): parrington or synthetic 1080p, eager launches,
one HIP-event pair per launch of the chosen classes (pano_prof).

    PANO_LIB=tools/ab/libpano_<v>.so python tools/feat_time.py [parrington|synthetic] [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from vfx_image_stitching_amd import _lib, data  # noqa: E402
from vfx_image_stitching_amd.pipeline import Stitcher  # noqa: E402

work = sys.argv[1] if len(sys.argv) > 1 else "parrington"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
if work == "synthetic":
    frames, focals, _ = data.synthetic_sequence(n_frames=144, h=1080, w=1920, start=0, count=19)
else:
    _, frames, focals, _ = data.load_set("parrington")
st = Stitcher("sift", cap=32768 if work == "synthetic" else 4096)
cyl, _ = st.cylindrical(st.upload(frames), focals)
st.features(cyl)
torch.cuda.synchronize()
classes = ["blur_level", "extrema_localize", "orientation", "sort_dedup", "descriptor"]
out = {}
for k in classes:
    st.ctx.prof_enable(k)
    for _ in range(reps):
        st.features(cyl)
    torch.cuda.synchronize()
    r = st.ctx.prof_read(k)
    out[k] = round(r["total_ms"] / reps, 4)
st.ctx.prof_enable(-1)
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(reps):
    st.features(cyl)
ev1.record()
torch.cuda.synchronize()
out["features_ms"] = round(ev0.elapsed_time(ev1) / reps, 4)
print(os.path.basename(os.environ.get("PANO_LIB", "") or "base"), work, out)
