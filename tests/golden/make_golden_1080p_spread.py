#!/usr/bin/env python3
"""Golden fixture for BASELINE config 5 beyond its first pairs: four more pairs spread over the
144-frame synthetic 1080p sequence, from the ORACLE (as make_golden_1080p.py, whose docstring
says why not from the reference itself: ~25 min per 1080p frame plus ~50 min per pair).

Pairs (35, 36), (71, 72), (107, 108), (142, 143) of ``data.synthetic_sequence(n_frames=144,
h=1080, w=1920)``: each frame generated on its own (start = i, count = 2).

Written to tests/golden/synthetic_1080p_spread.npz / .json, kept small (the tree travels with
every GPU run):
  * per frame: the keypoint count, the cylindrical digest, the SHA-256 of each exact keypoint
    field over the whole table (x, y, response as float32, octave as int32: the fields the
    first-pairs test compares with equality), and every 4th row of size and angle (compared
    within the first-pairs test's bars);
  * per pair: the oracle's NN match count under desc_thresh, the ransac move and the winning
    pair (image_stitching_sift.py:63-111 semantics).

Usage:  python tests/golden/make_golden_1080p_spread.py        (~10 min, 8 GB peak)
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from make_golden_1080p import digest, nn_chunked  # noqa: E402
from oracle import sift as osift  # noqa: E402
from oracle import stitch as ostitch  # noqa: E402
from vfx_image_stitching_amd import data  # noqa: E402

PAIRS = (35, 71, 107, 142)
SUB = 4
EXACT = (("x", np.float32), ("y", np.float32), ("response", np.float32), ("octave", np.int32))


def main():
    out, meta = {}, {"pairs_at": list(PAIRS), "shape": [1080, 1920], "sub": SUB, "per_frame": {}, "pairs": []}
    for p in PAIRS:
        frames, focals, _ = data.synthetic_sequence(n_frames=144, h=1080, w=1920, start=p, count=2)
        feats = []
        for k in range(2):
            i = p + k
            t = time.time()
            cyl = ostitch.cylindrical(frames[k], focals[k])
            kps, desc = osift.detect_and_describe(cyl)
            du8 = desc.astype(np.uint8)
            assert np.array_equal(du8.astype(np.float32), desc)
            pf = {"count": int(len(du8)), "cyl_digest": digest(cyl)}
            for name, dt in EXACT:
                pf[f"{name}_digest"] = digest(np.asarray(kps[name]).astype(dt))
            meta["per_frame"][str(i)] = pf
            out[f"f{i}_size_sub"] = np.asarray(kps["size"], np.float64)[::SUB]
            out[f"f{i}_angle_sub"] = np.asarray(kps["angle"], np.float64)[::SUB]
            feats.append((kps, desc))
            print(f"frame {i}: {len(du8)} keypoints, {time.time() - t:.1f} s", flush=True)
        (kA, dA), (kB, dB) = feats
        j, dist = nn_chunked(dA, dB)
        matches = [((float(kA["x"][a]), float(kA["y"][a])), (float(kB["x"][j[a]]), float(kB["y"][j[a]])))
                   for a in range(len(dA)) if dist[a] < 25000]
        move, pair = ostitch.ransac(matches, 3)
        meta["pairs"].append({"pair": [p, p + 1], "n_matches": len(matches), "move": list(move),
                              "best_pair": [list(pair[0]), list(pair[1])]})
        print(f"pair {p}: {len(matches)} matches, move {move}", flush=True)
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "synthetic_1080p_spread.npz"), **out)
    with open(os.path.join(REPO, "tests", "golden", "synthetic_1080p_spread.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
