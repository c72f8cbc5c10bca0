#!/usr/bin/env python3
"""Sweep OpenCV float32 GaussianBlur arithmetic variants against the PUBLISHED SIFT panoramas.

The author's ``Result/sift_{grail,prtn}_result.jpg`` (tests/golden/published/) were made by
the reference with real OpenCV.  For each blur variant of oracle/cv2_compat.py (taps x row
pass x column pass, see oracle/cv_blur.c) this runs the oracle's whole SIFT stitch of
parrington and grail (features per frame on a process pool, then match, RANSAC, drift,
blend, crop) and compares the q95 re-encoded panorama with the published JPEG:
shape, zero-offset PSNR and identical-byte fraction when the shapes agree, band-aligned
PSNR otherwise.  Test/diagnostic tooling: it imports the oracle, never the product.

    python tools/blur_variants.py [--variants legacy:f64:f64,bitexact:fma:symfma ...] [--jobs 8]
Writes one JSON line per (variant, set) to stdout and, with --out, to a file.
"""
from __future__ import annotations

import argparse
import itertools
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PUB = {"grail": "sift_grail_result.jpg", "parrington": "sift_prtn_result.jpg"}


def _features(args):
    spec, setname, i = args
    from oracle import cv2_compat, sift, stitch
    from vfx_image_stitching_amd import data
    cv2_compat.set_blur_variant(spec)
    names, frames, focals, margin = data.load_set(setname)
    cyl = stitch.cylindrical(frames[i], focals[i])
    k, d = sift.detect_and_describe(cyl)
    return spec, setname, i, k, d


def all_variants():
    return [f"{t}:{r}:{c}" for t, r, c in itertools.product(
        ("legacy", "bitexact"), ("f64", "fma", "mul"), ("f64", "symfma", "symmul", "fma"))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="all")
    ap.add_argument("--sets", default="grail,parrington")
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    variants = all_variants() if a.variants == "all" else a.variants.split(",")
    sets = a.sets.split(",")
    from oracle import stitch
    from vfx_image_stitching_amd import data, quality
    meta = {s: data.load_set(s) for s in sets}
    work = [(v, s, i) for v in variants for s in sets for i in range(len(meta[s][1]))]
    feats = {}
    t0 = time.time()
    with mp.get_context("spawn").Pool(a.jobs) as pool:
        for spec, s, i, k, d in pool.imap_unordered(_features, work):
            feats[(spec, s, i)] = (k, d)
    sys.stderr.write(f"features: {len(work)} frames in {time.time() - t0:.0f}s\n")
    out = open(a.out, "a") if a.out else None
    for v in variants:
        for s in sets:
            names, frames, focals, margin = meta[s]
            fs = [feats[(v, s, i)] for i in range(len(frames))]
            pano, shifts, pairs, _ = stitch.stitch(list(frames), list(focals), "sift", margin,
                                                   features=fs)
            with open(os.path.join(ROOT, "tests", "golden", "published", PUB[s]), "rb") as f:
                pub = quality.decode_jpeg(f.read())
            rep = quality.compare_published(pano, pub)
            rep.update({"variant": v, "set": s,
                        "shifts": [[round(float(x), 4), round(float(y), 4)] for x, y in shifts],
                        "n_kp": [int(len(k)) for k, _ in fs]})
            line = json.dumps(rep)
            print(line, flush=True)
            if out:
                out.write(line + "\n")
    if out:
        out.close()


if __name__ == "__main__":
    main()
