#!/usr/bin/env python3
"""Per kernel class HBM bytes per step from FETCH_SIZE / WRITE_SIZE passes (see pmc_traffic.sh).
The first stitch of the run is a warm-up (allocations) and is skipped."""
import collections
import csv
import glob
import json
import os
import re
import sys

# device kernel name -> libpano profiler class (_lib.KERNELS)
CLASSES = [
    (r"^(gray_frames|blur_fast|blur_level|blur_tail|blur_chain|blur_pair)", "blur_level"),
    (r"^(extrema_scan|extrema_stream|localize)", "extrema_localize"),
    (r"^orientation", "orientation"),
    (r"^(rank_keys|bucket_|emit_keypoints)", "sort_dedup"),
    (r"^(descriptor|desc_order)", "descriptor"),
    (r"^(pack_rows|row_norms|row_consts)", "row_norms"),
    (r"^(dist_bf16|dist_mfma|dist_u8|dist_i8)", "dist_mfma"),
    (r"^reduce_parts", "reduce_parts"),
    (r"^(pair_shifts|pair_compact|pair_votes|pair_select)", "pair_shifts"),
    (r"^(composite|plan_device)", "composite_step"),
    (r"^(bbox_|gray_bbox)", "gray_bbox"),
    # timing-class names of _lib.KERNELS: the inverse-map pair (cyl_columns, cyl_inverse)
    # fills the slots the scatter pair (cyl_scatter, cyl_gather) named first
    (r"^(cyl_scatter|cyl_columns|cyl_tile)", "cyl_scatter"),
    (r"^(cyl_gather|cyl_inverse)", "cyl_gather"),
    (r"^jpeg_", "jpeg_decode"),
]


def cls(name):
    k = name.replace("(anonymous namespace)::", "").split("(")[0]
    k = k[5:] if k.startswith("void ") else k
    for pat, c in CLASSES:
        if re.match(pat, k):
            return c
    return None


root, runs = sys.argv[1], int(sys.argv[2])
work = sys.argv[3] if len(sys.argv) > 3 else "parrington"
out = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, tools/pmc_traffic.sh, {work} SIFT step",
       "correction": "bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (profiles/r01_fetch_calibration.txt)",
       "classes": {}}
acc = collections.defaultdict(lambda: collections.defaultdict(float))
launches = collections.defaultdict(int)
steps = None
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    rows = []
    for f in glob.glob(os.path.join(root, c, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    # a stitch starts with its projection launch; the first stitch (allocations, captures) is
    # skipped and the rest are averaged.  Round 5's table divided three stitches by two: the
    # one-launch projection (cyl_tile) was missing from the class patterns, so nothing was
    # skipped and every class read 1.5x its true bytes per step.
    starts = [i for i, r in enumerate(rows) if cls(r["Kernel_Name"]) == "cyl_scatter"]
    if len(starts) != runs:
        sys.exit(f"{c}: {len(starts)} stitches found in the trace, {runs} expected")
    steps = runs - 1
    for r in rows[starts[1]:]:
        k = cls(r["Kernel_Name"])
        if k is None:
            continue
        acc[k][c] += float(r["Counter_Value"]) * 1024
        if c == "FETCH_SIZE":
            launches[k] += 1
out["steps"] = steps
for k, v in acc.items():
    out["classes"][k] = {"hbm_bytes_per_step": round((2 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) / steps),
                         "read_bytes_per_step": round(2 * v["FETCH_SIZE"] / steps),
                         "write_bytes_per_step": round(v["WRITE_SIZE"] / steps),
                         "launches_per_step": launches[k] / steps}
print(json.dumps(out, indent=1, sort_keys=True))
