#!/usr/bin/env python3
"""Per-launch HBM bytes of the pyramid (S1-S4) and extrema (S5/S6) launches of one stitch, from
the FETCH_SIZE / WRITE_SIZE passes of tools/pmc_traffic.sh, each launch named by the planes it
reads and writes (attribute the blur's traffic to named buffers).

    python3 tools/pmc_per_launch.py gpurun_out/pmct N parrington|synthetic

Columns: measured read / write MB per launch (averaged over the stitches after the first,
bytes = 2 * FETCH_SIZE + WRITE_SIZE, profiles/r01_fetch_calibration.txt), the launch's design
bytes (the planes it must touch: its input level read once, the levels it writes written once),
and the launch's share of SURVEY 8(d)'s algorithmic S1-S4 figure (3 P + 32 sum(Po) per frame:
gray in, three kept Gaussian levels and five DoG planes per octave out, no inter-level reads).
"""
import csv
import glob
import math
import os
import re
import sys

MB = 1e6


def rows_of(root, counter):
    rows = []
    for f in glob.glob(os.path.join(root, counter, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def short(name):
    k = name.replace("(anonymous namespace)::", "")
    k = k[5:] if k.startswith("void ") else k
    return k.split("(")[0]


def octaves(h, w):
    """sift_impl.py:59-63 and :96 -- octave shapes of the x2 base."""
    n = int(round(math.log(min(2 * h, 2 * w)) / math.log(2) - 1))
    shp = [(2 * h, 2 * w)]
    for _ in range(1, n):
        hh, ww = shp[-1]
        shp.append((int(hh / 2), int(ww / 2)))
    return shp


def main():
    root, runs, work = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    n, (h, w) = {"parrington": (18, (512, 384)), "synthetic": (19, (1080, 1920))}[work]
    shp = octaves(h, w)
    P = h * w
    fetch, write = rows_of(root, "FETCH_SIZE"), rows_of(root, "WRITE_SIZE")
    wmap = {r["Dispatch_Id"]: float(r["Counter_Value"]) * 1024 for r in write}
    starts = [i for i, r in enumerate(fetch) if short(r["Kernel_Name"]).startswith("cyl_")]
    assert len(starts) == runs, (len(starts), runs)
    steps = [fetch[starts[i]:(starts[i + 1] if i + 1 < len(starts) else len(fetch))] for i in range(1, runs)]
    # launches of interest, in order, per step
    want = re.compile(r"^(gray_frames|blur_|extrema_|localize)")
    per = []
    for st in steps:
        per.append([(short(r["Kernel_Name"]), 2 * float(r["Counter_Value"]) * 1024, wmap[r["Dispatch_Id"]])
                    for r in st if want.match(short(r["Kernel_Name"]))])
    L = len(per[0])
    assert all(len(p) == L for p in per), [len(p) for p in per]
    avg = [(per[0][i][0], sum(p[i][1] for p in per) / len(per), sum(p[i][2] for p in per) / len(per))
           for i in range(L)]
    alg_total = n * (3 * P + 32 * sum(a * b for a, b in shp))
    # name the blur launches by the launch sequence (sift_pyramid.hip pano_sift_pyramid)
    o, lvl = 0, 0
    lines = []
    tot = {"r": 0.0, "w": 0.0, "dr": 0.0, "dw": 0.0}
    o_tail = next((k for k in range(1, len(shp)) if shp[k][0] <= 64 and shp[k][1] <= 64), len(shp))
    for k, rb, wb in avg:
        Po = None
        if k == "gray_frames":
            what, dr, dw = "BGR frames -> gray u8", 3 * P * n, P * n
            alg = 3 * P * n
        elif k.startswith("blur_fast<0"):
            Po = shp[0][0] * shp[0][1]
            what, dr, dw = "o0 base: gray -> G0", P * n, 4 * Po * n
            alg = 0
            o, lvl = 0, 0
        elif k.startswith("blur_fast<2"):
            o, lvl = o + 1, 1
            Po = shp[o][0] * shp[o][1]
            what = f"o{o} L1: G{o - 1}[3] (every 2nd row) -> G1 + DoG0"
            dr, dw = 8 * Po * n, 8 * Po * n
            alg = 4 * Po * n * 2          # SURVEY: G1 + DoG0 written
        elif k.startswith("blur_fast<1"):
            lvl += 1
            Po = shp[o][0] * shp[o][1]
            if lvl == 5:
                what, dr, dw = f"o{o} L5: G4 -> DoG4", 4 * Po * n, 4 * Po * n
                alg = 4 * Po * n
            else:
                what, dr, dw = f"o{o} L{lvl}: G{lvl - 1} -> G{lvl} + DoG{lvl - 1}", 4 * Po * n, 8 * Po * n
                alg = (8 if lvl <= 3 else 4) * Po * n     # SURVEY keeps G1..G3
        elif k.startswith("blur_tail"):
            sp = sum(a * b for a, b in shp[o_tail:])
            pv = shp[o_tail - 1][0] * shp[o_tail - 1][1]
            what = f"tail o{o_tail}..o{len(shp) - 1}: one workgroup per frame, all levels"
            dr, dw = 2 * pv * n, 36 * sp * n
            alg = 32 * sp * n
        elif k.startswith("extrema_stream") or k.startswith("extrema_scan"):
            what, dr, dw, alg = "S5 scan of DoG planes (5 per octave)", None, None, None
        elif k.startswith("localize"):
            what, dr, dw, alg = "S6 localize (3x3x3 cubes of candidates)", None, None, None
        else:
            what, dr, dw, alg = "", None, None, None
        if dr is not None:
            tot["r"] += rb
            tot["w"] += wb
            tot["dr"] += dr
            tot["dw"] += dw
        ratio = (rb + wb) / (dr + dw) if dr else float("nan")
        lines.append(f"{k[:34]:34s} {what[:52]:52s} {rb / MB:9.2f} {wb / MB:9.2f} "
                     + (f"{dr / MB:9.2f} {dw / MB:9.2f} {ratio:6.2f} {alg / MB:9.2f}" if dr is not None
                        else f"{'':9s} {'':9s} {'':6s} {'':9s}"))
    print(f"# {work}: {n} frames of {h}x{w}, octaves {shp}; {len(per)} stitches averaged "
          f"(the first of {runs} skipped)")
    print("# MB = 1e6 bytes per launch; read = 2 * FETCH_SIZE, write = WRITE_SIZE "
          "(profiles/r01_fetch_calibration.txt)")
    print(f"{'kernel':34s} {'planes':52s} {'read':>9s} {'write':>9s} {'d_read':>9s} {'d_write':>9s} "
          f"{'meas/d':>6s} {'SURVEY':>9s}")
    for ln in lines:
        print(ln)
    print(f"# S1-S4 launches: measured {tot['r'] / MB:.1f} MB read + {tot['w'] / MB:.1f} MB written = "
          f"{(tot['r'] + tot['w']) / MB:.1f} MB per stitch; design (each launch's planes once) "
          f"{tot['dr'] / MB:.1f} + {tot['dw'] / MB:.1f} = {(tot['dr'] + tot['dw']) / MB:.1f} MB; "
          f"SURVEY 8(d) algorithmic {alg_total / MB:.1f} MB")
    print(f"# measured / design = {(tot['r'] + tot['w']) / (tot['dr'] + tot['dw']):.3f}; "
          f"measured / SURVEY = {(tot['r'] + tot['w']) / alg_total:.3f}")


if __name__ == "__main__":
    main()
