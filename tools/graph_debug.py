#!/usr/bin/env python3
"""Diagnose hipGraph replay: after each run(graph=True), compare every Stitcher buffer with
the eager run's values.  Usage: python tools/graph_debug.py [sift|harris] [set]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vfx_image_stitching_amd import data                      # noqa: E402
from vfx_image_stitching_amd.pipeline import Stitcher        # noqa: E402

method = sys.argv[1] if len(sys.argv) > 1 else "harris"
setname = sys.argv[2] if len(sys.argv) > 2 else "grail"
names, frames, focals, margin = data.load_set(setname)
st = Stitcher(method)
dev = st.upload(frames)
st.run(dev, focals, margin=margin)
torch.cuda.synchronize()
snap = {k: v.clone() for k, v in st._buf.items()}
print("buffers:", {k: tuple(v.shape) for k, v in snap.items()}, flush=True)
for it in range(5):
    res = st.run(dev, focals, margin=margin, graph=True)
    torch.cuda.synchronize()
    diffs = []
    for k, v in st._buf.items():
        if k not in snap:
            diffs.append(f"{k}:new")
            continue
        a, b = v.cpu().numpy(), snap[k].cpu().numpy()
        if a.shape != b.shape or not np.array_equal(a.view(np.uint8), b.view(np.uint8)):
            nd = int((a.view(np.uint8) != b.view(np.uint8)).sum()) if a.shape == b.shape else -1
            diffs.append(f"{k}:{nd}B")
    cnt = st._buf["counts"].cpu().numpy().tolist()
    print(f"iter {it}: graphs={len(st._graphs)} diffs={diffs or 'none'} counts={cnt[:6]}",
          flush=True)
