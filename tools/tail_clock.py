#!/usr/bin/env python3
"""Per-level clock stamps of blur_tail (diagnostics build: tools/ab_variant.sh tailclk
-DPANO_TAIL_TIMING=1), parrington features, frame 0's workgroup.  s_memtime counts the
shader clock; the ratio of stamps to the event-timed kernel gives its rate.

    PANO_LIB=tools/ab/libpano_tailclk.so PANO_TAIL_SOLO=1 python tools/tail_clock.py
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from vfx_image_stitching_amd import _lib, data  # noqa: E402
from vfx_image_stitching_amd.pipeline import Stitcher  # noqa: E402

_, frames, focals, _ = data.load_set("parrington")
st = Stitcher("sift", cap=4096)
cyl, _ = st.cylindrical(st.upload(frames), focals)
lib = _lib.load()
buf = (ctypes.c_ulonglong * 64)()
for rep in range(4):
    st.features(cyl)
    torch.cuda.synchronize()
    assert lib.pano_dbg_tail_clock(buf) == 0
    v = list(buf)
    n = max(i for i in range(64) if v[i]) + 1
    d = [v[i] - v[i - 1] for i in range(1, n)]
    print(f"rep {rep}: total {v[n - 1] - v[0]} clk; per level: {d}")
st.ctx.prof_enable("blur_level")
for _ in range(5):
    st.features(cyl)
torch.cuda.synchronize()
print("blur class ms per features():", st.ctx.prof_read("blur_level")["total_ms"] / 5)
