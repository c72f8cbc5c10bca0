#!/usr/bin/env python3
"""Where run()'s host time goes on the graph-replay fast path (parrington, SIFT): cProfile of
200 replayed stitches, sorted by own time, against the bare launch+wait library call."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from vfx_image_stitching_amd import _lib, data  # noqa: E402
from vfx_image_stitching_amd.pipeline import Stitcher  # noqa: E402

names, frames, focals, margin = data.load_set("parrington")
st = Stitcher("sift")
d = st.upload(frames)
for _ in range(3):
    st.run(d, focals, margin=margin, graph=True)
torch.cuda.synchronize()
N = 200
t0 = time.perf_counter()
for _ in range(N):
    st.run(d, focals, margin=margin, graph=True)
t1 = time.perf_counter()
g = st.last_graphs[-1]
cur = torch.cuda.current_stream().cuda_stream
for _ in range(N):
    st.ctx.lib.pano_graph_launch_sync(st.ctx.h, g, _lib._P(cur))
t2 = time.perf_counter()
print(f"run() {(t1 - t0) / N * 1e6:.1f} us; launch+wait {(t2 - t1) / N * 1e6:.1f} us")
pr = cProfile.Profile()
pr.enable()
for _ in range(N):
    st.run(d, focals, margin=margin, graph=True)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
