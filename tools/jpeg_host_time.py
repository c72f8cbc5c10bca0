#!/usr/bin/env python3
"""Host-side cost of the file-to-file leg (bench.py jpeg_inclusive) at parrington: the
pano_jpeg_decode call alone (header parse, table build, pinned staging, enqueue), the decode's
GPU time, the encode call (GPU work + D2H of the file bytes), and the whole leg.

    python tools/jpeg_host_time.py [reps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from vfx_image_stitching_amd import data, jpeg  # noqa: E402
from vfx_image_stitching_amd.pipeline import Stitcher  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
names, bufs = data.load_set_jpegs("parrington")
_, frames, focals, margin = data.load_set("parrington")
st = Stitcher("sift")
dev = st.upload(frames)
for _ in range(3):
    jpeg.decode_batch(bufs, out=dev, status=True)
    r = st.run(dev, focals, margin=margin, graph=True)
    jpeg.encode(r.panorama)
torch.cuda.synchronize()
tick = time.perf_counter
acc = {k: 0.0 for k in ("decode_call", "decode_gpu", "run", "encode", "leg")}
for _ in range(reps):
    t0 = tick()
    jpeg.decode_batch(bufs, out=dev, status=True)
    t1 = tick()
    torch.cuda.synchronize()
    t2 = tick()
    r = st.run(dev, focals, margin=margin, graph=True)
    t3 = tick()
    jpeg.encode(r.panorama)
    t4 = tick()
    acc["decode_call"] += t1 - t0
    acc["decode_gpu"] += t2 - t1
    acc["run"] += t3 - t2
    acc["encode"] += t4 - t3
    acc["leg"] += t4 - t0
print({k: round(v / reps * 1e3, 4) for k, v in acc.items()}, "ms")
g0 = st.ctx.generation()
torch.cuda.synchronize()
t0 = tick()
for _ in range(reps):
    st.run(dev, focals, margin=margin, graph=True)
t1 = tick()
print("run alone", round((t1 - t0) / reps * 1e3, 4), "ms; generation", g0, st.ctx.generation())
# decode then run with the GPU idle for the same host time (is it the decode or the pause?)
t_dec = acc["decode_call"] / reps
acc2 = 0.0
for _ in range(reps):
    torch.cuda.synchronize()
    t2 = tick()
    while tick() - t2 < t_dec:
        pass
    torch.cuda.synchronize()
    t2 = tick()
    st.run(dev, focals, margin=margin, graph=True)
    acc2 += tick() - t2
print("run after an idle pause", round(acc2 / reps * 1e3, 4), "ms")
acc3 = 0.0
for _ in range(reps):
    jpeg.decode_batch(bufs, out=dev, status=True)
    torch.cuda.synchronize()
    t2 = tick()
    st.run(dev, focals, margin=margin, graph=True)
    acc3 += tick() - t2
print("run right after a decode", round(acc3 / reps * 1e3, 4), "ms; generation", st.ctx.generation())
