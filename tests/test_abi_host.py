"""C-ABI surface and host-side logic (CPU-only; no kernel launches)."""
from __future__ import annotations

import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT
from oracle import cv2_compat, sift, stitch


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "pano.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(pano_[a-z_0-9]+)\s*\(", src, re.M)))


def test_library_exports_every_header_symbol():
    from vfx_image_stitching_amd import _lib
    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 24
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # and the Python binding declares exactly the header's functions
    assert sorted(_lib.SIGNATURES) == syms


def test_library_is_gfx950(tmp_path):
    # llvm-objdump --offloading extracts the bundles next to its input: run it on a copy
    import shutil
    lib = tmp_path / "libpano.so"
    shutil.copy(os.path.join(ROOT, "vfx_image_stitching_amd", "libpano.so"), lib)
    out = os.popen(f"/opt/rocm/lib/llvm/bin/llvm-objdump --offloading {lib} 2>&1").read()
    if "gfx950" not in out:
        # older objdump: grep the embedded bundle name
        data = open(os.path.join(ROOT, "vfx_image_stitching_amd", "libpano.so"), "rb").read()
        assert b"gfx950" in data


def test_sift_plan_matches_oracle():
    from vfx_image_stitching_amd import _lib
    lib = _lib.load()
    for (h, w) in [(512, 384), (571, 428), (1080, 1920), (17, 23)]:
        p = _lib.default_sift_params()
        no, nl = ctypes.c_int32(), ctypes.c_int32()
        sb = ctypes.c_double()
        sl = (ctypes.c_double * 8)()
        assert lib.pano_sift_plan(ctypes.byref(p), h, w, ctypes.byref(no), ctypes.byref(nl),
                                  ctypes.byref(sb), sl) == 0
        assert no.value == sift.n_octaves((2 * h, 2 * w))
        assert nl.value == 6
        assert list(sl)[:6] == list(sift.level_sigmas(1.6, 3))
        assert sb.value == float(np.sqrt(max(1.6 ** 2 - 1.0, 0.01)))


@pytest.mark.parametrize("sigma", [1.2489995996796799, 1.2262734984654078, 1.5450077936447955,
                                   1.9465878414647133, 2.4525469969308156, 3.090015587289591, 0.7])
def test_gaussian_taps_match_cv2_restatement(sigma):
    from vfx_image_stitching_amd import _lib
    lib = _lib.load()
    out = (ctypes.c_double * 64)()
    n = ctypes.c_int32()
    assert lib.pano_sift_taps(sigma, out, ctypes.byref(n)) == 0
    # OpenCV 4.x getGaussianKernel(CV_32F): the bit-exact kernel cast to f32 (the published
    # SIFT panoramas pin this form)
    k = cv2_compat.getGaussianKernelBitExact(cv2_compat.gaussian_ksize(sigma), sigma).astype(np.float32)
    assert n.value == len(k)
    np.testing.assert_array_equal(np.array(out[:n.value]), k.astype(np.float64))


def test_blend_geometry_matches_reference_arithmetic():
    from vfx_image_stitching_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(3)
    for _ in range(200):
        hA, wA, hB, wB = rng.integers(5, 60, 4)
        dx = float(rng.uniform(-40, 40))
        dy = float(rng.uniform(-5, 5))
        ref = np.array(rng.uniform(0, 50, 4), np.float64)
        geom = np.zeros(8, np.int32)
        ov = ctypes.c_double()
        assert lib.pano_blend_geometry(dx, dy, _lib.f64p(ref), int(hA), int(wA), int(hB), int(wB),
                                       _lib.i32p(geom), ctypes.byref(ov)) == 0
        sw, _, dyy, padA, padB, overlap = stitch.blend_geometry(
            (dx, dy), ((ref[0], ref[1]), (ref[2], ref[3])), int(wA), int(hA), int(wB), int(hB))
        A = np.ones((int(hA), int(wA), 3), np.uint8)
        B = np.ones((int(hB), int(wB), 3), np.uint8)
        if sw:
            A, B = B, A
        sa = stitch.pad_image(A, -padA, -dyy)
        sb = stitch.pad_image(B, padB, dyy)
        assert bool(geom[6]) == sw
        assert ov.value == overlap
        assert (geom[4], geom[5]) == (max(sa.shape[0], sb.shape[0]), max(sa.shape[1], sb.shape[1]))
        # placements: where the (all-ones) image lands inside its padded canvas
        ya, xa = np.argwhere(sa[..., 0])[0]
        yb, xb = np.argwhere(sb[..., 0])[0]
        assert (geom[0], geom[1], geom[2], geom[3]) == (ya, xa, yb, xb)


def test_plan_composite_reproduces_reference_mosaic_shape(gold_json):
    """pano_plan_composite replays the 17 blend geometries of the SIFT parrington run."""
    from vfx_image_stitching_amd import _lib
    from vfx_image_stitching_amd.pipeline import drift_correct
    lib = _lib.load()
    gold = gold_json("sift_parrington.json")
    shifts = [tuple(s["move"]) for s in gold["shifts"]]
    pairs = [s["pair"] for s in gold["shifts"]]
    corr = drift_correct(shifts)
    assert [list(c) for c in corr] == [s["shift"] for s in gold["steps"]]
    sh = np.ascontiguousarray(np.array(corr, np.float64))
    pr = np.ascontiguousarray(np.array([[a[0], a[1], b[0], b[1]] for a, b in pairs], np.float64))
    n = len(shifts) + 1
    steps = (_lib.Step * (n - 1))()
    first = np.zeros(2, np.int32)
    hw = np.zeros(2, np.int32)
    assert lib.pano_plan_composite(_lib.f64p(sh), _lib.f64p(pr), n, 512, 384, steps,
                                   _lib.i32p(first), _lib.i32p(hw)) == 0
    for i, st in enumerate(steps):
        assert [st.canvas_h, st.canvas_w, 3] == gold["steps"][i]["shape"]
    assert list(hw) == gold["steps"][-1]["shape"][:2]
    assert all(st.frame_is_a == 1 for st in steps)        # every parrington dx < 0


def test_read_pano_data_quirks(tmp_path):
    from vfx_image_stitching_amd.stitching import read_pano_data, resolve_paths
    p = tmp_path / "pano.txt"
    p.write_text("C:\\x\\a.jpg\n1 2\n\n512.5\nC:\\x\\b.JPG\n3 4 5\nC:\\x\\c.png\n700\n")
    imgs, foc = read_pano_data(str(p))
    # b.JPG has no focal line before the next image: dropped (quirk 2 of SURVEY)
    assert imgs == ["C:\\x\\a.jpg", "C:\\x\\c.png"] and foc == [512.5, 700.0]
    assert resolve_paths(str(tmp_path) + "/", imgs)[0].endswith("/a.jpg")
    assert stitch.read_pano_data(str(p)) == (imgs, foc)


def test_drift_correction():
    from vfx_image_stitching_amd.pipeline import drift_correct
    s = [(-10.0, 1.0), (-11.0, 2.0), (-9.0, 3.0)]
    assert drift_correct(s) == stitch.drift_correct(s) == [(-10.0, -1.0), (-11.0, 0.0), (-9.0, 1.0)]


def test_synthetic_generator_ground_truth():
    from vfx_image_stitching_amd import data
    frames, focals, jit = data.synthetic_sequence(n_frames=4, h=96, w=160, step=100, focal=150.0)
    assert frames.shape == (4, 96, 160, 3) and frames.dtype == np.uint8
    c0 = stitch.cylindrical(frames[0], focals[0])
    c1 = stitch.cylindrical(frames[1], focals[1])
    # frame 1's content = frame 0's shifted right by `step` (up to jitter rows)
    a = c0[20:70, 10:40].astype(int)
    dj = jit[1] - jit[0]
    b = c1[20 - dj:70 - dj, 110:140].astype(int)
    assert np.mean(np.abs(a - b)) < 3.0
