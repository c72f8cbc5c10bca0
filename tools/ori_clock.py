#!/usr/bin/env python3
"""Per-wave phase clocks of the orientation kernel (diagnostics build:
tools/ab_variant.sh oriclk -DPANO_ORI_TIMING=1).  Each persistent wave records s_memrealtime
(100 MHz) at entry and exit, its candidate count, and per phase the summed time: claim + locate
+ candidate load, patch staging, the sample walk, and histogram / smoothing / peaks / emit.

    PANO_LIB=tools/ab/libpano_oriclk.so python tools/ori_clock.py [parrington|synthetic]
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
fn = lib.pano_dbg_ori_clock
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros((WAVES, 8), np.uint64)
for rep in range(4):
    torch.cuda.synchronize()
    assert fn(None, 1) == 0
    st.features(cyl)
    torch.cuda.synchronize()
    assert fn(buf.ctypes.data, 0) == 0
    v = buf[buf[:, 7] != 0].astype(np.int64)
    t0 = v[:, 0].min()
    ent = (v[:, 0] - t0) * TICK_US
    ext = (v[:, 1] - t0) * TICK_US
    nc = v[:, 2]
    ph = v[:, 3:7].sum(0) * TICK_US / max(1, nc.sum())
    busy = (v[:, 1] - v[:, 0]) * TICK_US
    print(f"rep {rep}: {len(v)} waves, {nc.sum()} candidates ({nc.mean():.2f} per wave, max {nc.max()}); "
          f"span {ext.max():.1f} us; entry p50 / p90 / max {np.percentile(ent, 50):.1f} / "
          f"{np.percentile(ent, 90):.1f} / {ent.max():.1f} us; exit p10 / p50 / p90 / max "
          f"{np.percentile(ext, 10):.1f} / {np.percentile(ext, 50):.1f} / {np.percentile(ext, 90):.1f} / "
          f"{ext.max():.1f} us; wave busy mean {busy.mean():.1f} us", flush=True)
    print(f"   per candidate (us): claim+locate+load {ph[0]:.2f}, staging {ph[1]:.2f}, walk {ph[2]:.2f}, "
          f"post+emit {ph[3]:.2f}; sum {ph.sum():.2f}", flush=True)
    for x in range(1, 9):
        m = v[:, 7] == x
        if m.any():
            print(f"   xcd {x - 1}: waves {m.sum()}, candidates {nc[m].sum()}, last exit {ext[m].max():.1f} us, "
                  f"entry max {ent[m].max():.1f} us", flush=True)
st.ctx.prof_enable("orientation")
for _ in range(5):
    st.features(cyl)
torch.cuda.synchronize()
print("orientation ms per features():", st.ctx.prof_read("orientation")["total_ms"] / 5)
