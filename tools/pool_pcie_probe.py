#!/usr/bin/env python3
"""Where the host-to-host StitchPool form loses its overlap (round 6): ms per parrington stitch
of StitchPool.run_sequence with device items, host items (upload only), device items with
to_host (download only), and both; K stitches each, 4 contexts.

    python tools/pool_pcie_probe.py [K]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vfx_image_stitching_amd import data  # noqa: E402
from vfx_image_stitching_amd.pipeline import StitchPool  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 60
names, frames, focals, margin = data.load_set("parrington")
pool = StitchPool("sift", contexts=int(os.environ.get("CTX", "4")))
dev = pool.upload(frames)
host = torch.from_numpy(np.ascontiguousarray(frames)).pin_memory()


def run(items, to_host):
    for _ in pool.run_sequence(items[:4 * len(pool.members) + 2], margin=margin, to_host=to_host):
        pass
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in pool.run_sequence(items, margin=margin, to_host=to_host):
        pass
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / len(items) * 1e3


for name, src, th in (("device", dev, False), ("upload", host, False), ("download", dev, True),
                      ("both", host, True), ("device again", dev, False)):
    print(f"{name:14s} {run([(src, focals)] * K, th):.4f} ms per stitch", flush=True)

# host-bound or device-bound?  Time the host spends blocked in event waits (event.synchronize
# and the graph-launch-and-wait call) against the wall time, for the device and host forms
_blocked = [0.0]
_sync = torch.cuda.Event.synchronize


def _timed_sync(self):
    t = time.perf_counter()
    _sync(self)
    _blocked[0] += time.perf_counter() - t


torch.cuda.Event.synchronize = _timed_sync
for name, src, th in (("device", dev, False), ("both", host, True)):
    items = [(src, focals)] * K
    for _ in pool.run_sequence(items[:4 * len(pool.members) + 2], margin=margin, to_host=th):
        pass
    torch.cuda.synchronize()
    _blocked[0] = 0.0
    t0 = time.perf_counter()
    for _ in pool.run_sequence(items, margin=margin, to_host=th):
        pass
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / K * 1e3
    print(f"{name:14s} {ms:.4f} ms per stitch, host blocked in event waits {_blocked[0] / K * 1e3:.4f} ms per stitch",
          flush=True)
