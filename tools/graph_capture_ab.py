#!/usr/bin/env python3
"""Diagnostic: graph-replayed parrington stitch time for the first capture and for
re-captures after release_graphs(), with the blur tail forked to its side stream and with
PANO_TAIL_MAIN=1 (one chain)."""
import os
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402

from vfx_image_stitching_amd import data  # noqa: E402
from vfx_image_stitching_amd.pipeline import Stitcher  # noqa: E402

_, frames, focals, margin = data.load_set("parrington")
for mode, fresh in (("0", "0"), ("0", "1"), ("1", "0"), ("0", "1")):
    os.environ["PANO_TAIL_MAIN"] = mode
    os.environ["PANO_FRESH_SIDE"] = fresh
    st = Stitcher("sift")
    dev = st.upload(frames)
    out = []
    for cap in range(4):
        if cap:
            st.release_graphs()
        for _ in range(3):
            st.run(dev, focals, margin=margin, graph=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            st.run(dev, focals, margin=margin, graph=True)
        out.append(round((time.perf_counter() - t0) / 20 * 1e3, 3))
    st.release_graphs()
    print(f"PANO_TAIL_MAIN={mode} PANO_FRESH_SIDE={fresh}: first capture then 3 re-captures: {out} ms",
          flush=True)
