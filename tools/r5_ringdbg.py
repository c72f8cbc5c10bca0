import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vfx_image_stitching_amd import data
from vfx_image_stitching_amd.pipeline import Stitcher
_, frames, focals, _ = data.load_set("parrington")
st = Stitcher("sift", cap=4096)
cyl, _ = st.cylindrical(st.upload(frames[:1]), focals[:1])
st.features(cyl)
torch.cuda.synchronize()
print("done")
