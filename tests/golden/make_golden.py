#!/usr/bin/env python3
"""Generate golden fixtures by running the REFERENCE's own Python in this container.

The reference (/root/reference, read-only) imports ``cv2``, which is absent; this script
injects ``oracle.cv2_compat`` as ``sys.modules['cv2']`` and then imports and runs the
reference modules verbatim.  The only other patches are the ones SURVEY.md section 8c lists:

* ``os.path.basename -> ntpath.basename`` (pano.txt stores Windows paths; quirk 1),
* ``builtins.input`` (the drivers prompt for folder, pano.txt and crop margin),
* JPEG output is captured in memory (``CV2_COMPAT_NO_DISK``) because the reference
  folder is read-only.

Recorders wrap the reference's per-pair functions so that every intermediate the build is
judged on (cylindrical frames, per-frame features, matches, per-pair shifts, per-step
mosaics, the cropped panorama) is captured.  The reference source never leaves this
container: only data (inputs, outputs, digests) is written under tests/golden/.

Usage::

    python tests/golden/make_golden.py pack            # input frames -> data/*.npz
    python tests/golden/make_golden.py harris parrington|grail|out
    python tests/golden/make_golden.py sift_pair       # config 2: prtn00 + prtn01
    python tests/golden/make_golden.py sift parrington|grail   # 10-15 min each
    python tests/golden/make_golden.py probes          # numpy-semantics vectors
"""
from __future__ import annotations

import builtins
import hashlib
import io
import json
import ntpath
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference"
GOLD = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)

from oracle import cv2_compat  # noqa: E402

SETS = {"parrington": 15, "grail": 17, "out": 30}   # README.md:51-54 crop margins


def digest(a) -> str:
    a = np.ascontiguousarray(a)
    h = hashlib.sha256()
    h.update(f"{a.dtype.str}{a.shape}".encode())
    h.update(a.tobytes())
    return h.hexdigest()


def import_reference():
    os.environ["CV2_COMPAT_NO_DISK"] = "1"
    sys.modules["cv2"] = cv2_compat
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import importlib
    mods = {}
    for name in ("sift_impl", "image_stitching_sift", "image_stitching_harris"):
        mods[name] = importlib.import_module(name)
    return mods


def kp_table(kps):
    """KeyPoints -> structured float32/int arrays (exact f32 storage)."""
    return {
        "x": np.array([k.pt[0] for k in kps], np.float32),
        "y": np.array([k.pt[1] for k in kps], np.float32),
        "size": np.array([k.size for k in kps], np.float32),
        "angle": np.array([k.angle for k in kps], np.float32),
        "response": np.array([k.response for k in kps], np.float32),
        "octave": np.array([k.octave for k in kps], np.int64),
    }


# ------------------------------------------------------------------------------ pack
def cmd_pack():
    """Pack each input set's JPEG bytes + pano.txt focal list into data/<set>.npz.

    The GPU box has no /root/reference, so inputs travel as data.  The JPEG bytes are
    stored verbatim (decoded with PIL at run time: identical pixels to cv2.imread per
    SURVEY.md 8c) together with the parsed pano.txt order and focal lengths.
    """
    mods = import_reference()
    ref_read = mods["image_stitching_sift"].read_pano_data
    os.makedirs(os.path.join(REPO, "data"), exist_ok=True)
    for s in SETS:
        paths, focals = ref_read(os.path.join(REF, s, "pano.txt"))
        names = [ntpath.basename(p) for p in paths]
        blobs = {}
        for n in names:
            with open(os.path.join(REF, s, n), "rb") as f:
                blobs[n] = np.frombuffer(f.read(), np.uint8)
        np.savez(os.path.join(REPO, "data", f"{s}_frames.npz"),
                 order=np.array(names), focals=np.array(focals, np.float64),
                 margin=np.int64(SETS[s]), **{f"jpg_{n}": b for n, b in blobs.items()})
        print(s, len(names), "frames packed")


# ------------------------------------------------------------------------------ drivers
class Recorder:
    def __init__(self):
        self.shift_calls = []
        self.feature_calls = {}
        self.blend_steps = []


def run_driver(kind: str, s: str, mods, rec: Recorder):
    mod = mods["image_stitching_sift" if kind == "sift" else "image_stitching_harris"]
    answers = iter([os.path.join(REF, s), "", str(SETS[s])])
    builtins_input = builtins.input
    basename = os.path.basename
    builtins.input = lambda prompt="": next(answers)
    os.path.basename = ntpath.basename
    cyl_frames = []
    orig_cyl = mod.cylindrical_projection
    orig_blend = mod.blend_two_images
    shift_name = "compute_shift_sift" if kind == "sift" else "compute_shift_harris"
    orig_shift = getattr(mod, shift_name)

    def cyl(img, f):
        out = orig_cyl(img, f)
        cyl_frames.append((digest(img), float(f), digest(out)))
        return out

    def shift(a, b, *args, **kw):
        t0 = time.time()
        res = orig_shift(a, b, *args, **kw)
        rec.shift_calls.append({"a": digest(a), "b": digest(b), "move": [float(v) for v in res[0]],
                                "pair": None if res[1] is None else [[float(v) for v in p] for p in res[1]],
                                "sec": time.time() - t0})
        print(f"  pair {len(rec.shift_calls)}: {res[0]}  {time.time() - t0:.1f}s", flush=True)
        return res

    def blend(shift_vec, ref_match, a, b):
        out = orig_blend(shift_vec, ref_match, a, b)
        rec.blend_steps.append({"shift": [float(v) for v in shift_vec],
                                "pair": [[float(v) for v in p] for p in ref_match],
                                "shape": list(out.shape), "digest": digest(out)})
        return out

    mod.cylindrical_projection = cyl
    mod.blend_two_images = blend
    setattr(mod, shift_name, shift)
    try:
        cv2_compat._WRITES.clear()
        t0 = time.time()
        mod.run_panorama()
        wall = time.time() - t0
    finally:
        builtins.input = builtins_input
        os.path.basename = basename
        mod.cylindrical_projection = orig_cyl
        mod.blend_two_images = orig_blend
        setattr(mod, shift_name, orig_shift)
    (path, pano), = cv2_compat._WRITES.items()
    return pano, cyl_frames, wall


def published_digest(path):
    img = cv2_compat.imread(path)
    return digest(img), list(img.shape)


def cmd_harris(s):
    mods = import_reference()
    rec = Recorder()
    harris = mods["image_stitching_harris"]
    orig_feat = harris.compute_keypoints_and_descriptors_harris

    def feat(img, max_points=200):
        kps, descs = orig_feat(img, max_points=max_points)
        key = digest(img)
        if key not in rec.feature_calls:
            rec.feature_calls[key] = (np.array(kps, np.int64).reshape(-1, 2), descs.copy())
        return kps, descs

    harris.compute_keypoints_and_descriptors_harris = feat
    try:
        pano, cyl, wall = run_driver("harris", s, mods, rec)
    finally:
        harris.compute_keypoints_and_descriptors_harris = orig_feat
    rt = cv2_compat.jpeg_q95_roundtrip(pano)
    out = {"set": s, "wall_s": wall, "margin": SETS[s], "cyl": cyl,
           "shifts": rec.shift_calls, "steps": rec.blend_steps,
           "pano_shape": list(pano.shape), "pano_digest": digest(pano),
           "pano_q95_digest": digest(rt)}
    pub = {"parrington": "Result/harris_prtn_result.jpg", "grail": "Result/harris_grail_result.jpg"}
    if s in pub:
        d, shp = published_digest(os.path.join(REF, pub[s]))
        out["published_result"] = {"file": pub[s], "digest": d, "shape": shp,
                                   "identical_after_q95": d == out["pano_q95_digest"]}
        step_dir = os.path.join(REF, f"pano_step_{s}")
        steps_pub = []
        for i in range(1, 18):
            d, shp = published_digest(os.path.join(step_dir, f"pano{i}.jpg"))
            steps_pub.append({"file": f"pano_step_{s}/pano{i}.jpg", "digest": d, "shape": shp})
        out["published_steps"] = steps_pub
    # per-frame Harris features, in cylindrical-frame order
    feats = {}
    order = [c[2] for c in cyl]
    for i, key in enumerate(order):
        if key in rec.feature_calls:
            kps, descs = rec.feature_calls[key]
            feats[f"kps_{i}"] = kps
            feats[f"desc_{i}"] = descs
    np.savez_compressed(os.path.join(GOLD, f"harris_{s}_features.npz"), **feats)
    with open(os.path.join(GOLD, f"harris_{s}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("set", "wall_s", "pano_shape")}),
          out.get("published_result"))


def cmd_sift_pair():
    """Config 2: cyl(prtn00, f=704.968) + cyl(prtn01, f=706.469) -> one compute_shift_sift."""
    mods = import_reference()
    sift = mods["sift_impl"]
    st = mods["image_stitching_sift"]
    paths, focals = st.read_pano_data(os.path.join(REF, "parrington", "pano.txt"))
    names = [ntpath.basename(p) for p in paths]
    fmap = dict(zip(names, focals))
    frames = {}
    for n in ("prtn00.jpg", "prtn01.jpg", "prtn02.jpg"):
        img = cv2_compat.imread(os.path.join(REF, "parrington", n))
        frames[n] = st.cylindrical_projection(img, fmap[n])
    out = {}
    arrays = {}
    for n, cyl in frames.items():
        t0 = time.time()
        # stage-by-stage, exactly as compute_keypoints_and_descriptors chains them
        gray = cv2_compat.cvtColor(cyl, cv2_compat.COLOR_BGR2GRAY).astype("float32")
        base = sift.generate_base_image(gray, 1.6, 0.5)
        no = sift.compute_number_of_octaves(base.shape)
        ks = sift.generate_gaussian_kernels(1.6, 3)
        gimgs = sift.generate_gaussian_images(base, no, ks)
        dogs = sift.generate_DoG_images(gimgs)
        raw = sift.find_scale_space_extrema(gimgs, dogs, 3, 1.6, 5)
        raw_t = kp_table(raw)
        nodup = sift.remove_duplicate_keypoints(raw)
        conv = sift.convert_keypoints_to_input_image_size(nodup)
        desc = sift.generate_descriptors(conv, gimgs)
        sec = time.time() - t0
        # whole-function call must agree with the staged chain
        kps2, desc2 = sift.compute_keypoints_and_descriptors(cyl)
        assert np.array_equal(desc2, desc) and len(kps2) == len(conv)
        stem = n[:-4]
        for k, v in kp_table(conv).items():
            arrays[f"{stem}_kp_{k}"] = v
        for k, v in raw_t.items():
            arrays[f"{stem}_raw_{k}"] = v
        arrays[f"{stem}_desc"] = desc.astype(np.uint8)
        assert np.array_equal(desc.astype(np.uint8).astype(np.float32), desc)
        # pyramid probes: full octaves >= 2, a few rows of octaves 0-1
        for o, octv in enumerate(gimgs):
            for l, g in enumerate(octv):
                arrays[f"{stem}_g{o}_{l}_digest"] = np.frombuffer(digest(g).encode(), np.uint8)
                if o >= 3:
                    arrays[f"{stem}_g{o}_{l}"] = g
                else:
                    arrays[f"{stem}_g{o}_{l}_rows"] = g[::97]
        out[stem] = {"n_raw": len(raw), "n_kp": len(conv), "sec": sec,
                     "n_octaves": int(no), "sigmas": [float(v) for v in ks],
                     "cyl_digest": digest(cyl), "desc_digest": digest(desc)}
        print(stem, out[stem], flush=True)
    # config 2 pair, through the reference's own compute_shift_sift
    for a, b in (("prtn00", "prtn01"), ("prtn01", "prtn02")):
        t0 = time.time()
        move, pair = st.compute_shift_sift(frames[a + ".jpg"], frames[b + ".jpg"], ransac_thr=3,
                                           desc_thresh=25000)
        # matches as compute_shift_sift builds them (:63-79), for the match-kernel tests
        kA, dA = sift.compute_keypoints_and_descriptors(frames[a + ".jpg"])
        kB, dB = sift.compute_keypoints_and_descriptors(frames[b + ".jpg"])
        idx = []
        dist = []
        for i in range(len(dA)):
            d = dA[i] - dB
            dd = np.einsum("ij,ij->i", d.astype(np.float64), d.astype(np.float64))
            j = int(np.argmin(dd))
            idx.append(j)
            dist.append(dd[j])
        arrays[f"match_{a}_{b}_idx"] = np.array(idx, np.int64)
        arrays[f"match_{a}_{b}_dist"] = np.array(dist, np.float64)
        out[f"shift_{a}_{b}"] = {"move": [float(v) for v in move],
                                 "pair": [[float(v) for v in p] for p in pair],
                                 "sec": time.time() - t0}
        print(a, b, out[f"shift_{a}_{b}"], flush=True)
    np.savez_compressed(os.path.join(GOLD, "sift_pair.npz"), **arrays)
    with open(os.path.join(GOLD, "sift_pair.json"), "w") as f:
        json.dump(out, f, indent=1)


def cmd_sift(s):
    mods = import_reference()
    rec = Recorder()
    st = mods["image_stitching_sift"]
    orig_feat = st.compute_keypoints_and_descriptors

    def feat(img, *a, **kw):
        t0 = time.time()
        kps, descs = orig_feat(img, *a, **kw)
        key = digest(img)
        if key not in rec.feature_calls:
            t = kp_table(kps)
            rec.feature_calls[key] = {"n": len(kps), "kp_digest": digest(np.stack(
                [t["x"], t["y"], t["size"], t["angle"], t["response"]])),
                "oct_digest": digest(t["octave"]), "desc_digest": digest(descs),
                "sec": time.time() - t0, "table": t, "desc": descs.astype(np.uint8)}
        return kps, descs

    st.compute_keypoints_and_descriptors = feat
    try:
        pano, cyl, wall = run_driver("sift", s, mods, rec)
    finally:
        st.compute_keypoints_and_descriptors = orig_feat
    order = [c[2] for c in cyl]
    frames = []
    arrays = {}
    for i, key in enumerate(order):
        fc = rec.feature_calls.get(key)
        if fc is None:
            frames.append(None)
            continue
        frames.append({k: v for k, v in fc.items() if k not in ("table", "desc")})
        for k, v in fc["table"].items():
            arrays[f"f{i}_{k}"] = v
        arrays[f"f{i}_desc"] = fc["desc"]
    out = {"set": s, "wall_s": wall, "margin": SETS[s], "cyl": cyl, "frames": frames,
           "shifts": [{k: v for k, v in c.items()} for c in rec.shift_calls],
           "steps": rec.blend_steps, "pano_shape": list(pano.shape),
           "pano_digest": digest(pano)}
    np.savez_compressed(os.path.join(GOLD, f"sift_{s}_features.npz"), **arrays)
    with open(os.path.join(GOLD, f"sift_{s}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("set", "wall_s", "pano_shape")}))


def cmd_cyl():
    """Cylindrical projection of every frame of every set through the reference C1."""
    mods = import_reference()
    st = mods["image_stitching_sift"]
    out = {}
    for s in SETS:
        paths, focals = st.read_pano_data(os.path.join(REF, s, "pano.txt"))
        rows = []
        for p, f in zip(paths, focals):
            n = ntpath.basename(p)
            img = cv2_compat.imread(os.path.join(REF, s, n))
            cyl = st.cylindrical_projection(img, f)
            rows.append({"name": n, "focal": f, "in": digest(img), "out": digest(cyl)})
        out[s] = rows
        print(s, len(rows), flush=True)
    with open(os.path.join(GOLD, "cylindrical.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    cmd = sys.argv[1]
    if cmd == "pack":
        cmd_pack()
    elif cmd == "harris":
        cmd_harris(sys.argv[2])
    elif cmd == "sift_pair":
        cmd_sift_pair()
    elif cmd == "sift":
        cmd_sift(sys.argv[2])
    elif cmd == "cyl":
        cmd_cyl()
    else:
        raise SystemExit(__doc__)
