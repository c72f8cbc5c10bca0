"""Phase clocks of plan_device (a PANO_PLAN_CLOCK=1 build: PANO_LIB=tools/ab/libpano_planclk.so):
s_memtime stamps of workgroup 0 at kernel entry, records staged, drift done, plan_core done,
the plan's status known, tables done, write-out begun -- 100 MHz ticks, printed as us deltas."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from vfx_image_stitching_amd import _lib, data  # noqa: E402
from vfx_image_stitching_amd.pipeline import Stitcher  # noqa: E402

names, frames, focals, margin = data.load_set("parrington")
st = Stitcher("sift")
dev = st.upload(frames)
for _ in range(3):
    st.run(dev, focals, margin=margin)
torch.cuda.synchronize()
res = st._buf["result"]
P = len(frames) - 1
off_plan = (P * 64 + 4 * 64 * 4 + 255) // 256 * 256
nb = int(st.ctx.lib.pano_plan_device_bytes())
clk = res[off_plan + nb - 64: off_plan + nb].cpu().numpy().view(np.int64)
print("plan_device phase clocks (s_memtime ticks from entry):", [int(c - clk[0]) for c in clk[:8]])
