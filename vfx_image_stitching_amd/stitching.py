"""Shared drop-in functions of image_stitching_sift.py / image_stitching_harris.py.

The two reference scripts carry AST-identical copies of the warp / blend / crop helpers
(SURVEY.md section 2); both shim modules re-export these.  Every image computation runs
in libpano; only pano.txt parsing, np.pad-style layout and scalar geometry stay on the host.
"""
from __future__ import annotations

import ctypes
import ntpath
import os

import numpy as np

from . import _lib
from ._lib import PanoError, context, ptr


def _torch():
    import torch
    return torch


def _dev(a: np.ndarray):
    t = _torch()
    return t.from_numpy(np.ascontiguousarray(a)).to(t.device("cuda", context().device))


def read_pano_data(pano_file_path):
    """image_stitching_sift.py:12-46: a .jpg/.png line, then a float-only line = focal."""
    images, focuses, pending = [], [], None
    with open(pano_file_path, "r", encoding="utf-8") as f:
        lines = f.read().splitlines()
    for line in lines:
        low = line.strip().lower()
        if ".jpg" in low or ".png" in low:
            pending = line.strip()
        elif " " not in low and low:
            try:
                val = float(low)
            except ValueError:
                continue
            if pending is not None:
                images.append(pending)
                focuses.append(val)
                pending = None
    return images, focuses


def ransac(matches, dist_sq_thresh=3):
    """Translation vote over all matches on the GPU (image_stitching_sift.py:86-111)."""
    if len(matches) == 0:
        return (0, 0), None
    moves = [(a[0] - b[0], a[1] - b[1]) for a, b in matches]
    mv = _dev(np.array(moves, np.float64))
    t = _torch()
    out = t.empty(2, dtype=t.int32, device=mv.device)
    ctx = context()
    ctx.check(ctx.lib.pano_ransac_translate(ctx.h, ptr(mv), len(moves), float(dist_sq_thresh),
                                            ptr(out)))
    best = int(out.cpu()[0])
    return moves[best], matches[best]


def cylindrical_projection(img_bgr, focal_len):
    img = np.ascontiguousarray(img_bgr, np.uint8)
    h, w = img.shape[:2]
    src = _dev(img.reshape(1, h, w, 3))
    t = _torch()
    dst = t.empty_like(src)
    f = np.array([float(focal_len)], np.float64)
    ctx = context()
    ctx.check(ctx.lib.pano_cylindrical(ctx.h, ptr(src), ptr(dst), 1, h, w, _lib.f64p(f), None))
    return dst[0].cpu().numpy()


def pad_image(img_bgr, move_x, move_y):
    """Zero padding (image_stitching_sift.py:139-153): data layout only."""
    mx = int(round(move_x))
    my = int(round(move_y))
    py = (my, 0) if my >= 0 else (0, -my)
    px = (mx, 0) if mx >= 0 else (0, -mx)
    return np.pad(img_bgr, (py, px, (0, 0)), "constant")


def blend_two_images(shift_vec, ref_match, imgA, imgB):
    """image_stitching_sift.py:156-202 on the GPU (column flags, alpha ramp, truncation)."""
    A = np.ascontiguousarray(imgA, np.uint8)
    B = np.ascontiguousarray(imgB, np.uint8)
    dx, dy = shift_vec
    ref = np.array([ref_match[0][0], ref_match[0][1], ref_match[1][0], ref_match[1][1]],
                   np.float64)
    geom = np.zeros(8, np.int32)
    ov = ctypes.c_double()
    lib = _lib.load()
    rc = lib.pano_blend_geometry(float(dx), float(dy), _lib.f64p(ref), A.shape[0], A.shape[1],
                                 B.shape[0], B.shape[1], _lib.i32p(geom), ctypes.byref(ov))
    if rc:
        raise PanoError(rc, "pano_blend_geometry")
    if geom[6]:
        A, B = B, A
    HH, WW = int(geom[4]), int(geom[5])
    dA, dB = _dev(A), _dev(B)
    t = _torch()
    out = t.empty((HH, WW, 3), dtype=t.uint8, device=dA.device)
    ctx = context()
    ctx.check(ctx.lib.pano_blend_two(ctx.h, ptr(dA), A.shape[0], A.shape[1], ptr(dB), B.shape[0],
                                     B.shape[1], _lib.i32p(geom), ov.value, ptr(out)))
    return out.cpu().numpy()


def rectangle_crop(img, black_threshold, extra_margin):
    """image_stitching_sift.py:208-247 with the bbox reduction on the GPU."""
    h = img.shape[0]
    d = _dev(np.ascontiguousarray(img, np.uint8))
    t = _torch()
    bb = t.empty(4, dtype=t.int32, device=d.device)
    ctx = context()
    ctx.check(ctx.lib.pano_gray_bbox(ctx.h, ptr(d), img.shape[0], img.shape[1],
                                     int(black_threshold), ptr(bb)))
    y0, y1, x0, x1 = (int(v) for v in bb.cpu().numpy())
    if y1 < 0:
        return img
    y0 = max(0, y0 + extra_margin)
    y1 = min(h - 1, y1 - extra_margin)
    if y0 > y1 or x0 > x1:
        return img
    return img[y0:y1 + 1, x0:x1 + 1]


def resolve_paths(folder_path, img_paths):
    """run_panorama :280-281 with ntpath.basename (pano.txt holds Windows paths, quirk 1)."""
    out = []
    for p in img_paths:
        out.append(p if os.path.exists(p) else os.path.join(folder_path, ntpath.basename(p)))
    return out


def imread_bgr(path):
    from PIL import Image
    if not os.path.exists(path):
        return None
    with Image.open(path) as im:
        return np.ascontiguousarray(np.asarray(im.convert("RGB"))[..., ::-1])


def imwrite_jpeg(path, img_bgr, quality=95):
    from PIL import Image
    Image.fromarray(np.ascontiguousarray(img_bgr[..., ::-1])).save(path, quality=quality)


def _read_frames(paths, decode, st):
    """The cv2.imread loop (run_panorama :280-287): "gpu" decodes the set's JPEG files in one
    pano_jpeg_decode batch straight into device memory; "host" is PIL; "auto" takes the GPU
    when every file is a baseline JPEG of one size (the reference's sets are) and PIL
    otherwise (progressive files, other formats, mixed sizes)."""
    from . import jpeg
    if any(not os.path.exists(p) for p in paths):
        raise FileNotFoundError("a frame listed in pano.txt is missing")
    if decode != "host":
        bufs = [open(p, "rb").read() for p in paths]
        try:
            shapes = {jpeg.info(b)[:2] for b in bufs}
        except Exception:
            if decode == "gpu":
                raise
            shapes = None
        if shapes is not None and len(shapes) == 1:
            return jpeg.decode_batch(bufs, device=st.device.index)
        if decode == "gpu":
            raise ValueError("GPU decode needs JPEG frames of one size")
    return st.upload([imread_bgr(p) for p in paths])


def run_panorama(folder_path=".", pano_file=None, margin=15, method="sift", out_name=None,
                 write=True, decode="auto", encode="gpu"):
    """Non-interactive run_panorama: the three input() prompts become arguments.  The frames
    are read with the GPU JPEG decoder (decode, see _read_frames) and the panorama is written
    with the GPU JPEG encoder at cv2.imwrite's default quality 95 (encode="gpu"; "host" = PIL;
    both give the same bytes)."""
    import time
    from . import jpeg
    from .pipeline import Stitcher
    if not (folder_path.endswith("/") or folder_path.endswith("\\")):
        folder_path += "/"
    pano_file = pano_file or folder_path + "pano.txt"
    img_paths, focals = read_pano_data(pano_file)
    if not img_paths:
        raise ValueError("no valid entries in pano.txt")
    t0 = time.time()
    st = Stitcher(method)
    frames_dev = _read_frames(resolve_paths(folder_path, img_paths), decode, st)
    res = st.run(frames_dev, np.array(focals, np.float64), margin=margin)
    pano = res.panorama.cpu().numpy()
    if write:
        name = out_name or ("panoroma_sift.jpg" if method == "sift" else "panoroma_harris.jpg")
        if encode == "gpu":
            jpeg.imwrite(os.path.join(folder_path, name), res.panorama)
        else:
            imwrite_jpeg(os.path.join(folder_path, name), pano)
    res.timings["wall_with_io"] = time.time() - t0
    return pano, res
