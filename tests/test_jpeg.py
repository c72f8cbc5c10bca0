"""JPEG decode: the reference's cv2.imread (image_stitching_sift.py:282)
on the GPU, bit-identical to libjpeg-turbo's default decode.

The oracle here is PIL (libjpeg-turbo, the decoder cv2.imread also runs; SURVEY.md 8(c)
measured PIL pixel-identical to cv2.imread on the reference's frames): every test compares
bytes.  CPU tests run the decoder's own per-thread functions through tools/jpeg_sim.cpp (the
kernels' logic replayed on the host) and check the header parser / C-ABI; ``-m gpu`` tests run
``pano_jpeg_decode`` itself.
"""
from __future__ import annotations

import io
import json
import os
import subprocess

import numpy as np
import pytest
from PIL import Image

from conftest import ROOT

SETS = ("parrington", "grail", "out")


def _set_jpegs(name):
    z = np.load(os.path.join(ROOT, "data", f"{name}_frames.npz"), allow_pickle=False)
    return [z[f"jpg_{n}"].tobytes() for n in (str(s) for s in z["order"])]


def _pil_bgr(buf: bytes) -> np.ndarray:
    with Image.open(io.BytesIO(buf)) as im:
        return np.ascontiguousarray(np.asarray(im.convert("RGB"))[..., ::-1])


def _encode(arr: np.ndarray, **kw) -> bytes:
    b = io.BytesIO()
    Image.fromarray(arr).save(b, "JPEG", **kw)
    return b.getvalue()


def _texture(h, w, seed, gray=False):
    """Smooth colour texture + noise: exercises long AC runs and flat regions alike."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    base = 128 + 60 * np.sin(xx / (7 + seed)) * np.cos(yy / 11.0)
    chans = [base + 40 * np.sin((xx + 13 * c) / (5.0 + c)) for c in range(3)]
    a = np.stack(chans, -1) + rng.normal(0, 12, (h, w, 3))
    a = np.clip(a, 0, 255).astype(np.uint8)
    return a[..., 0] if gray else a


# (h, w, gray, encoder kwargs): sizes off the MCU grid, every supported sampling, quality
# extremes, optimised (non-standard) Huffman tables
VARIANTS = [
    (512, 384, False, dict(quality=95)),
    (37, 53, False, dict(quality=75)),
    (61, 130, False, dict(quality=90, subsampling=0)),      # 4:4:4
    (45, 70, False, dict(quality=85, subsampling=1)),       # 4:2:2
    (99, 77, False, dict(quality=10)),
    (64, 96, False, dict(quality=100)),
    (83, 59, False, dict(quality=80, optimize=True)),
    (50, 71, True, dict(quality=90)),                       # grayscale
    (16, 16, False, dict(quality=50)),
]


def _variant_jpeg(i):
    h, w, gray, kw = VARIANTS[i]
    return _encode(_texture(h, w, i, gray), **kw)


# ------------------------------------------------------------------------------------- CPU
@pytest.fixture(scope="module")
def jpeg_sim(tmp_path_factory):
    """Build tools/jpeg_sim.cpp (host replay of the kernels' per-thread functions)."""
    out = tmp_path_factory.mktemp("jsim") / "jpeg_sim"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", "-o", str(out),
                    os.path.join(ROOT, "tools", "jpeg_sim.cpp"),
                    os.path.join(ROOT, "vfx_image_stitching_amd", "csrc", "jpeg_host.cpp")],
                   check=True, capture_output=True)
    return str(out)


def _sim(sim, buf, tmp_path, env=None):
    src, dst = tmp_path / "in.jpg", tmp_path / "out.bgr"
    src.write_bytes(buf)
    r = subprocess.run([sim, str(src), str(dst)], capture_output=True, text=True,
                       env=dict(os.environ, **(env or {})))
    st = json.loads(r.stdout)
    if st["status"]:
        return st, None
    return st, np.fromfile(dst, np.uint8).reshape(st["h"], st["w"], 3)


@pytest.mark.parametrize("name", SETS)
def test_sim_decode_equals_pil_on_reference_frames(jpeg_sim, tmp_path, name):
    fixes = 0
    for buf in _set_jpegs(name):
        st, out = _sim(jpeg_sim, buf, tmp_path)
        assert st["status"] == 0, st
        assert np.array_equal(out, _pil_bgr(buf))
        assert st["blocks"] >= st["total_blocks"]
        fixes += st["fixes"]
    # the start search resolves almost every subsequence from its candidates
    assert fixes <= 0.002 * 40000


@pytest.mark.parametrize("i", range(len(VARIANTS)))
def test_sim_decode_equals_pil_on_variants(jpeg_sim, tmp_path, i):
    buf = _variant_jpeg(i)
    st, out = _sim(jpeg_sim, buf, tmp_path)
    assert st["status"] == 0, st
    assert np.array_equal(out, _pil_bgr(buf))


def _with_trailer(buf: bytes) -> bytes:
    """A phone-style file: a second complete JPEG (an MPF secondary image / thumbnail) and a
    few junk bytes appended after EOI.  libjpeg stops at the first EOI and ignores the rest."""
    return buf + _encode(_texture(24, 40, 5), quality=60) + b"\x00\xffjunk"


def test_sim_decode_ignores_data_after_eoi(jpeg_sim, tmp_path):
    for buf in (_set_jpegs("parrington")[0], _variant_jpeg(2)):
        st, out = _sim(jpeg_sim, _with_trailer(buf), tmp_path)
        assert st["status"] == 0, st
        assert np.array_equal(out, _pil_bgr(buf))


def test_sim_without_warmup_still_exact(jpeg_sim, tmp_path):
    """No warm-up window (every warm candidate a guess at its subsequence's first bit): the
    fix candidates and the resolve fallback decode the subsequences from their true starts,
    and the result is still exact."""
    buf = _set_jpegs("parrington")[0]
    st, out = _sim(jpeg_sim, buf, tmp_path, env={"JPEG_SIM_W": "0"})
    assert st["fix_slots"] + st["fixes"] >= st["nsub"] // 2 and st["fixes"] > 0
    assert np.array_equal(out, _pil_bgr(buf))


def test_jpeg_info_and_refusals():
    from vfx_image_stitching_amd import jpeg
    from vfx_image_stitching_amd._lib import PANO_E_ARG, PANO_E_UNSUPPORTED, PanoError
    for name in SETS:
        for buf in _set_jpegs(name):
            h, w, c = jpeg.info(buf)
            with Image.open(io.BytesIO(buf)) as im:
                assert (w, h) == im.size and c == 3
    a = _texture(40, 40, 0)
    with pytest.raises(PanoError) as e:
        jpeg.info(_encode(a, progressive=True))
    assert e.value.code == PANO_E_UNSUPPORTED
    with pytest.raises(PanoError) as e:
        jpeg.info(_encode(a, restart_marker_blocks=2))
    assert e.value.code == PANO_E_UNSUPPORTED
    with pytest.raises(PanoError) as e:
        jpeg.info(b"\x89PNG\r\n\x1a\n" + bytes(64))
    assert e.value.code == PANO_E_ARG
    with pytest.raises(PanoError):
        jpeg.info(_encode(a)[:40])


# ------------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name", SETS)
def test_gpu_decode_equals_pil_on_reference_frames(gpu, name):
    from vfx_image_stitching_amd import data, jpeg
    bufs = _set_jpegs(name)
    out, st = jpeg.decode_batch(bufs, status=True)
    assert st.cpu().numpy().tolist() == [0] * len(bufs)
    _, frames, _, _ = data.load_set(name)          # PIL decode, pano.txt order
    assert np.array_equal(out.cpu().numpy(), frames)


@pytest.mark.gpu
def test_gpu_decode_equals_pil_on_variants(gpu):
    from vfx_image_stitching_amd import jpeg
    for i in range(len(VARIANTS)):
        buf = _variant_jpeg(i)
        out = jpeg.decode_batch([buf, buf])        # a batch of two: per-frame state
        ref = _pil_bgr(buf)
        got = out.cpu().numpy()
        assert np.array_equal(got[0], ref), (i, VARIANTS[i])
        assert np.array_equal(got[1], ref), (i, VARIANTS[i])


@pytest.mark.gpu
def test_gpu_decode_mixed_tables_in_one_batch(gpu):
    """Frames of one size with different quality, tables and sampling in one launch."""
    from vfx_image_stitching_amd import jpeg
    a = _texture(120, 160, 3)
    bufs = [_encode(a, quality=q, **kw) for q, kw in
            ((95, {}), (40, {}), (90, dict(subsampling=0)), (80, dict(subsampling=1)),
             (70, dict(optimize=True)))]
    got = jpeg.decode_batch(bufs).cpu().numpy()
    for g, b in zip(got, bufs):
        assert np.array_equal(g, _pil_bgr(b))


@pytest.mark.gpu
def test_gpu_decode_truncated_and_corrupt_streams(gpu):
    """A truncated scan reports PANO_E_ARG for that frame only; random corruption of the
    entropy bytes completes (bounded walks, bounds-checked writes) without touching the
    neighbouring frames."""
    from vfx_image_stitching_amd import jpeg
    from vfx_image_stitching_amd._lib import PANO_E_ARG
    good = _set_jpegs("parrington")[:3]
    trunc = good[1][: len(good[1]) // 2] + b"\xff\xd9"
    out, st = jpeg.decode_batch([good[0], trunc, good[2]], status=True)
    s = st.cpu().numpy()
    assert s[0] == 0 and s[2] == 0 and s[1] == PANO_E_ARG
    o = out.cpu().numpy()
    assert np.array_equal(o[0], _pil_bgr(good[0])) and np.array_equal(o[2], _pil_bgr(good[2]))
    rng = np.random.default_rng(7)
    bad = bytearray(good[1])
    for p in rng.integers(1000, len(bad) - 10, 40):
        bad[p] = int(rng.integers(0, 255))   # never 0xFF: no new markers
    out, st = jpeg.decode_batch([good[0], bytes(bad), good[2]], status=True)
    o = out.cpu().numpy()
    assert np.array_equal(o[0], _pil_bgr(good[0])) and np.array_equal(o[2], _pil_bgr(good[2]))


@pytest.mark.gpu
def test_gpu_decode_ignores_data_after_eoi(gpu):
    from vfx_image_stitching_amd import jpeg
    bufs = _set_jpegs("parrington")[:2]
    out, st = jpeg.decode_batch([_with_trailer(bufs[0]), bufs[1]], status=True)
    assert st.cpu().numpy().tolist() == [0, 0]
    o = out.cpu().numpy()
    assert np.array_equal(o[0], _pil_bgr(bufs[0])) and np.array_equal(o[1], _pil_bgr(bufs[1]))


@pytest.mark.gpu
def test_gpu_decode_refuses_mixed_sizes(gpu):
    from vfx_image_stitching_amd import jpeg
    from vfx_image_stitching_amd._lib import PanoError
    with pytest.raises(PanoError):
        jpeg.decode_batch([_encode(_texture(32, 32, 0)), _encode(_texture(32, 48, 0))])


# --------------------------------------------------------------------------------- encoder
# cv2.imwrite(path, panorama) (image_stitching_sift.py:386): libjpeg-turbo's default encoder at
# OpenCV's default quality 95; PIL's save(quality=q) runs the same encoder, byte for byte.
ENC_CASES = [(37, 53, 95), (64, 64, 95), (16, 16, 75), (100, 33, 50), (1, 1, 95), (2, 3, 95),
             (482, 700, 95), (17, 15, 10), (31, 47, 100)]


def _enc_image(h, w, seed):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    a = 128 + 60 * np.sin(xx / 7.0)[..., None] * np.cos(yy / 5.0)[..., None] + rng.normal(0, 20, (h, w, 3))
    return np.clip(a, 0, 255).astype(np.uint8)          # BGR


def _pil_encode_bgr(bgr, quality):
    return _encode(np.ascontiguousarray(bgr[..., ::-1]), quality=quality)


@pytest.fixture(scope="module")
def jpeg_enc_sim(tmp_path_factory):
    out = tmp_path_factory.mktemp("jesim") / "jpeg_enc_sim"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", "-o", str(out),
                    os.path.join(ROOT, "tools", "jpeg_enc_sim.cpp"),
                    os.path.join(ROOT, "vfx_image_stitching_amd", "csrc", "jpeg_host.cpp")],
                   check=True, capture_output=True)
    return str(out)


@pytest.mark.parametrize("case", range(len(ENC_CASES)))
def test_sim_encode_equals_pil_bytes(jpeg_enc_sim, tmp_path, case):
    h, w, q = ENC_CASES[case]
    img = _enc_image(h, w, case)
    (tmp_path / "in.bgr").write_bytes(img.tobytes())
    subprocess.run([jpeg_enc_sim, str(tmp_path / "in.bgr"), str(h), str(w), str(q), str(tmp_path / "o.jpg")],
                   check=True, capture_output=True)
    assert (tmp_path / "o.jpg").read_bytes() == _pil_encode_bgr(img, q)


@pytest.mark.gpu
def test_gpu_encode_equals_pil_bytes(gpu):
    import torch
    from vfx_image_stitching_amd import jpeg
    for case, (h, w, q) in enumerate(ENC_CASES):
        img = _enc_image(h, w, case)
        got = jpeg.encode(torch.from_numpy(img).cuda(), quality=q)
        assert got == _pil_encode_bgr(img, q), (h, w, q)


@pytest.mark.gpu
def test_gpu_encode_strided_view_and_roundtrip(gpu):
    """A crop view of a larger canvas (row pitch > 3 w) encodes like the contiguous crop, and
    the GPU decoder reads the file back exactly as PIL does."""
    import torch
    from vfx_image_stitching_amd import jpeg
    canvas = torch.from_numpy(_enc_image(300, 500, 9)).cuda()
    view = canvas[13:13 + 211, 41:41 + 377]
    got = jpeg.encode(view)
    ref = _pil_encode_bgr(view.cpu().numpy(), 95)
    assert got == ref
    back = jpeg.decode_batch([got]).cpu().numpy()[0]
    assert np.array_equal(back, _pil_bgr(got))


@pytest.mark.gpu
def test_gpu_encode_large_canvas(gpu):
    """A config-5-sized panorama (1080 x 24000, ~26 Mpx: ~400 k blocks, ~3 k length chunks and
    tens of thousands of stuffing chunks) encodes to PIL's q95 bytes; the chunk offsets come
    from one exclusive scan per pass (jpeg_enc_exscan), not per-workgroup prefix sums.  The
    encode time is printed for the record (JPEG encode)."""
    import time

    import torch
    from vfx_image_stitching_amd import jpeg
    img = torch.from_numpy(_enc_image(1080, 24000, 11)).cuda()
    got = jpeg.encode(img)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        got = jpeg.encode(img)
    ms = (time.perf_counter() - t0) / 3 * 1e3
    print(f"encode 1080x24000: {ms:.2f} ms, {len(got)} bytes")
    assert got == _pil_encode_bgr(img.cpu().numpy(), 95)
