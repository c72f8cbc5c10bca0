#!/usr/bin/env python3
"""Per-phase clock stamps of one blur_cascade workgroup (diagnostics build:
tools/ab_variant.sh casclk -DPANO_CAS_TIMING=<strip index + 1>): the cascade kernels of the
parrington features, then the stamps of the LAST cascade launch (octave 3's walker B by
default; PANO_CAS_STOP=<launches> stops the pyramid after that many by octave count).

    PANO_LIB=tools/ab/libpano_casclk.so PANO_BLUR_CASCADE=1 python tools/cas_clock.py
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from vfx_image_stitching_amd import _lib, data  # noqa: E402
from vfx_image_stitching_amd.pipeline import Stitcher  # noqa: E402

_, frames, focals, _ = data.load_set("parrington")
n = int(os.environ.get("CAS_FRAMES", "18"))
st = Stitcher("sift", cap=4096)
cyl, _ = st.cylindrical(st.upload(frames[:n]), focals[:n])
lib = _lib.load()
buf = (ctypes.c_ulonglong * (3 * 96 * 16))()
ctx = st.ctx
for rep in range(3):
    ctx.check(lib.pano_sift_pyramid(ctx.h, _lib.ptr(cyl), n, cyl.shape[1], cyl.shape[2], ctypes.byref(st.params)))
    torch.cuda.synchronize()
assert lib.pano_dbg_cas_clock(buf) == 0
v = np.array(list(buf), dtype=np.int64).reshape(3, 96, 16)
c = v[0]
steps = [i for i in range(96) if c[i, 0]]
print("steps stamped:", len(steps))
for i in steps[:40]:
    row = c[i]
    evs = [e for e in range(16) if row[e]]
    t0 = row[0]
    d = [int(row[e] - t0) for e in evs]
    ld = v[2, i]
    sw = v[1, i]
    print(f"step {i:3d}: compute {d}  load issue {int(ld[1]-ld[0]) if ld[0] else '-'} commit {int(ld[3]-ld[2]) if ld[2] else '-'} (commit starts at {int(ld[2]-t0) if ld[2] else '-'})  store {[int(sw[2*k+1]-sw[2*k]) for k in range(3) if sw[2*k]]}")
tot = [int(c[i, 15] - c[i, 0]) for i in steps if c[i, 15]]
print("mean clk per step:", np.mean(tot) if tot else None)
