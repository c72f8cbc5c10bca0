#!/usr/bin/env python3
"""Graph-replayed stitch steps only (what bench.py times), for a kernel trace of one step:
    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/step_timeline.py [workload]
    python3 tools/timeline.py DIR/run_kernel_trace.csv --step 10
"""
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402

from vfx_image_stitching_amd import data  # noqa: E402
from vfx_image_stitching_amd.pipeline import Stitcher  # noqa: E402

work = sys.argv[1] if len(sys.argv) > 1 else "parrington"
if work == "synthetic":
    frames, focals, _ = data.synthetic_sequence(n_frames=144, h=1080, w=1920, start=0, count=19)
    margin, cap = 15, 65536
else:
    _, frames, focals, margin = data.load_set(work)
    cap = 4096
st = Stitcher("sift", cap=cap)
dev = st.upload(frames)
for _ in range(20):
    st.run(dev, focals, margin=margin, graph=True)
torch.cuda.synchronize()
