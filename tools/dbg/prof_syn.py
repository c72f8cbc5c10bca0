"""Run the synthetic 1080p stitch N times (rocprofv3 counter collection)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch
from vfx_image_stitching_amd import data
from vfx_image_stitching_amd.pipeline import Stitcher
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
frames, focals, _ = data.synthetic_sequence(n_frames=144, h=1080, w=1920, start=0, count=19)
st = Stitcher("sift", cap=65536)
d = st.upload(frames)
for _ in range(n):
    st.run(d, focals, margin=15)
torch.cuda.synchronize()
print("done")
