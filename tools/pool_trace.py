#!/usr/bin/env python3
"""StitchPool run for a kernel trace, and its analysis: the union-busy fraction of the GPU
over the steady-state window and how much of it two stitches overlap.
    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/pool_trace.py
    python3 tools/pool_trace.py --analyze DIR/run_kernel_trace.csv"""
import csv
import sys

if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(sys.argv[2])))
    marks = [s for s, _, n in rows if "gray_frames" in n]
    # steady state: from the 10th to the 10th-last stitch start
    t0, t1 = marks[10], marks[-10]
    iv = [(max(s, t0), min(e, t1)) for s, e, _ in rows if e > t0 and s < t1]
    ev = sorted([(s, 1) for s, e in iv if e > s] + [(e, -1) for s, e in iv if e > s])
    depth, last, busy, two = 0, t0, 0, 0
    for t, d in ev:
        if depth > 0:
            busy += t - last
        if depth > 1:
            two += t - last
        depth += d
        last = t
    span = t1 - t0
    n = len(marks) - 20
    print(f"{n} stitches in {span / 1e3:.1f} us ({span / 1e3 / n:.1f} us each): GPU busy {busy / span:.1%}, "
          f">= 2 kernels at once {two / span:.1%}")
    sys.exit(0)

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402

from vfx_image_stitching_amd import data  # noqa: E402
from vfx_image_stitching_amd.pipeline import StitchPool  # noqa: E402

_, frames, focals, margin = data.load_set("parrington")
pool = StitchPool("sift", contexts=int(sys.argv[1]) if len(sys.argv) > 1 else 2)
dev = pool.upload(frames)
for _ in pool.run_sequence([(dev, focals)] * 60, margin=margin):
    pass
torch.cuda.synchronize()
