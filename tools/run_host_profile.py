#!/usr/bin/env python3
"""Diagnostic: cProfile of run()'s host path with the graph launch stubbed (parrington)."""
import sys, time, cProfile, pstats, io
sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch, numpy as np
from vfx_image_stitching_amd import data
from vfx_image_stitching_amd.pipeline import Stitcher
_, frames, focals, margin = data.load_set("parrington")
st = Stitcher("sift"); dev = st.upload(frames)
for _ in range(3): st.run(dev, focals, margin=margin, graph=True)
torch.cuda.synchronize()
lib = st.ctx.lib
real = lib.pano_graph_launch_sync
lib.pano_graph_launch_sync = lambda *a: 0
t0 = time.perf_counter()
for _ in range(2000): st.run(dev, focals, margin=margin, graph=True)
print("host path", (time.perf_counter() - t0) / 2000 * 1e6, "us")
pr = cProfile.Profile(); pr.enable()
for _ in range(2000): st.run(dev, focals, margin=margin, graph=True)
pr.disable()
s = io.StringIO(); pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18); print(s.getvalue()[:3500])
