#!/usr/bin/env python3
"""Per-wave clocks of the descriptor kernel (diagnostics build: tools/ab_variant.sh descclk
-DPANO_DESC_TIMING=1): each persistent wave records s_memrealtime (100 MHz) at entry and exit
and its keypoint count -- the drain (how long the last waves run after the median one).

    PANO_LIB=tools/ab/libpano_descclk.so python tools/desc_clock.py [parrington|synthetic]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vfx_image_stitching_amd import _lib, data  # noqa: E402
from vfx_image_stitching_amd.pipeline import Stitcher  # noqa: E402

WAVES = 16384
TICK_US = 0.01                          # s_memrealtime: 100 MHz

work = sys.argv[1] if len(sys.argv) > 1 else "parrington"
if work == "synthetic":
    frames, focals, _ = data.synthetic_sequence(n_frames=144, h=1080, w=1920, start=0, count=19)
    cap = 65536
else:
    _, frames, focals, _ = data.load_set(work)
    cap = 4096
st = Stitcher("sift", cap=cap)
cyl, _ = st.cylindrical(st.upload(frames), focals)
lib = _lib.load()
fn = lib.pano_dbg_desc_clock
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros((WAVES, 4), np.uint64)
for rep in range(4):
    torch.cuda.synchronize()
    assert fn(None, 1) == 0
    st.features(cyl)
    torch.cuda.synchronize()
    assert fn(buf.ctypes.data, 0) == 0
    v = buf[buf[:, 3] != 0].astype(np.int64)
    t0 = v[:, 0].min()
    ent = (v[:, 0] - t0) * TICK_US
    ext = (v[:, 1] - t0) * TICK_US
    nk = v[:, 2]
    busy = (v[:, 1] - v[:, 0]) * TICK_US
    print(f"rep {rep}: {len(v)} waves, {nk.sum()} keypoints ({nk.mean():.2f} per wave, max {nk.max()}); "
          f"span {ext.max():.1f} us; entry p50 / max {np.percentile(ent, 50):.1f} / {ent.max():.1f} us; "
          f"exit p10 / p50 / p90 / p99 / max {np.percentile(ext, 10):.1f} / {np.percentile(ext, 50):.1f} / "
          f"{np.percentile(ext, 90):.1f} / {np.percentile(ext, 99):.1f} / {ext.max():.1f} us; "
          f"wave busy mean {busy.mean():.1f} us; per keypoint {busy.sum() / max(1, nk.sum()):.2f} wave-us", flush=True)
    for x in range(1, 9):
        m = v[:, 3] == x
        if m.any():
            print(f"   xcd {x - 1}: waves {m.sum()}, keypoints {nk[m].sum()}, exit p50 {np.percentile(ext[m], 50):.1f}, "
                  f"last {ext[m].max():.1f} us", flush=True)
st.ctx.prof_enable("descriptor")
for _ in range(5):
    st.features(cyl)
torch.cuda.synchronize()
print("descriptor ms per features():", st.ctx.prof_read("descriptor")["total_ms"] / 5)
