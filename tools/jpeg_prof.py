#!/usr/bin/env python3
"""JPEG decode timing: N decodes of a set's 18 files (GPU), host-side call time vs the
synchronised time; run under rocprofv3 --kernel-trace --stats for the per-kernel split.
  python3 tools/jpeg_prof.py [N] [set]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from vfx_image_stitching_amd import data, jpeg  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 20
name = sys.argv[2] if len(sys.argv) > 2 else "parrington"
_, bufs = data.load_set_jpegs(name)
out, st = jpeg.decode_batch(bufs, status=True)
torch.cuda.synchronize()
t_call = 0.0
t0 = time.perf_counter()
for _ in range(N):
    a = time.perf_counter()
    jpeg.decode_batch(bufs, out=out, status=True)
    t_call += time.perf_counter() - a
torch.cuda.synchronize()
el = (time.perf_counter() - t0) / N
st_ = jpeg.last_stats(len(bufs))
print("sync stats (nsub, fix candidates, serial):", st_[:, :3].sum(0).tolist(), "max serial/frame", int(st_[:, 2].max()))
print(f"{name}: {len(bufs)} files, {sum(map(len, bufs))} bytes: {el * 1e3:.3f} ms per batch decode "
      f"(host call {t_call / N * 1e3:.3f} ms); status {st.cpu().tolist()}")
