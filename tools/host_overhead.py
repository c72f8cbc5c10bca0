#!/usr/bin/env python3
"""Host-side cost of one graph-replayed stitch: total run() wall time vs the library call that
launches the graph and waits, and the Python around it (parrington, SIFT)."""
import os
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
lib, c = st.ctx.lib, st.ctx.h
g = st.last_graphs[-1]
cur = torch.cuda.current_stream().cuda_stream
N = 50
t0 = time.perf_counter()
for _ in range(N):
    st.run(d, focals, margin=margin, graph=True)
t1 = time.perf_counter()
for _ in range(N):
    lib.pano_graph_launch_sync(c, g, _lib._P(cur))
t2 = time.perf_counter()
for _ in range(N):
    lib.pano_graph_launch(c, g)
t3 = time.perf_counter()
torch.cuda.synchronize()
t4 = time.perf_counter()
print(f"run(): {(t1 - t0) / N * 1e6:.1f} us/stitch; launch+wait only: {(t2 - t1) / N * 1e6:.1f} us; "
      f"launch only (async, {N} queued): {(t3 - t2) / N * 1e6:.1f} us CPU per launch, "
      f"drain {(t4 - t3) * 1e3:.1f} ms; back-to-back GPU time {(t4 - t2) / N * 1e6:.1f} us/graph")
# wake-up: the same launch, then a busy poll of the stream instead of the blocking sync
s = torch.cuda.current_stream()
t5 = time.perf_counter()
for _ in range(N):
    lib.pano_graph_launch(c, g)
    while not s.query():
        pass
t6 = time.perf_counter()
# the host work of run() alone: its Python around a replay, with the GPU already done
st.run(d, focals, margin=margin, graph=True)
torch.cuda.synchronize()
launch_sync = lib.pano_graph_launch_sync
lib.pano_graph_launch_sync = lambda *a: 0            # no GPU work: pure host path
t7 = time.perf_counter()
for _ in range(N):
    st.run(d, focals, margin=margin, graph=True)
t8 = time.perf_counter()
lib.pano_graph_launch_sync = launch_sync
print(f"launch + spin on hipStreamQuery: {(t6 - t5) / N * 1e6:.1f} us/stitch; "
      f"run()'s host path alone: {(t8 - t7) / N * 1e6:.1f} us")
