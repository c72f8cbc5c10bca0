"""PSNR of a stitched panorama against a published reference panorama (BASELINE metric).

The metric's third part is "PSNR vs CPU ref" (BASELINE.json).  Two references exist:

* the reference's Python run in the build container on the restated OpenCV blur
  (tests/golden/*.json digests): the GPU panorama is bit-exact against it (PSNR = inf);
* the author's published panoramas (reference ``Result/sift_{grail,prtn}_result.jpg``,
  written by ``cv2.imwrite`` at its default quality 95, image_stitching_sift.py:385-386),
  made with real OpenCV, whose f32 GaussianBlur rounds differently.

For the second, the panorama goes through the same JPEG q95 encode the reference applies
(PIL's baseline encoder matches cv2.imwrite's for these files: the Harris path reproduces
the published Harris JPEGs pixel for pixel) and is compared on the decoded uint8 arrays.
When the shapes differ (parrington: one pair's sub-pixel shift rounds the other way, so the
canvas is one row / column larger), the comparison is band-aligned: each 256-column band of
the published image is matched at its best integer offset within +-3 px, and the PSNR of
all bands at those offsets is reported with the offsets.
"""
from __future__ import annotations

import io

import numpy as np


def jpeg_roundtrip(bgr: np.ndarray, quality: int = 95) -> np.ndarray:
    """uint8 BGR -> JPEG (PIL, baseline, 4:2:0 like cv2.imwrite) -> uint8 BGR."""
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(np.ascontiguousarray(bgr[..., ::-1])).save(buf, format="JPEG", quality=quality)
    return decode_jpeg(buf.getvalue())


def decode_jpeg(data: bytes) -> np.ndarray:
    """JPEG bytes -> uint8 BGR (cv2.imread semantics)."""
    from PIL import Image
    return np.ascontiguousarray(np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))[..., ::-1])


def mse(a: np.ndarray, b: np.ndarray) -> float:
    d = a.astype(np.float64) - b.astype(np.float64)
    return float(np.mean(d * d))


def psnr_from_mse(m: float) -> float:
    return float("inf") if m == 0 else float(10.0 * np.log10(255.0 ** 2 / m))


def psnr(a: np.ndarray, b: np.ndarray) -> float:
    return psnr_from_mse(mse(a, b))


def _window(a, b, dy, dx, c0, c1):
    """Published columns [c0, c1) of b against a shifted by (dy, dx); the overlap only."""
    ys_a, ys_b = max(0, dy), max(0, -dy)
    h = min(a.shape[0] - ys_a, b.shape[0] - ys_b)
    ca0, ca1 = c0 + dx, c1 + dx
    if ca0 < 0 or ca1 > a.shape[1] or h <= 0:
        return None
    return a[ys_a:ys_a + h, ca0:ca1], b[ys_b:ys_b + h, c0:c1]


def band_aligned(ours: np.ndarray, published: np.ndarray, band: int = 256, search: int = 3):
    """Per published column band: the (dy, dx) in [-search, search]^2 minimising the MSE.
    Returns (psnr over all bands at their offsets, [(c0, dy, dx, band psnr)])."""
    se, cnt, bands = 0.0, 0, []
    for c0 in range(0, published.shape[1], band):
        c1 = min(c0 + band, published.shape[1])
        best = None
        for dy in range(-search, search + 1):
            for dx in range(-search, search + 1):
                w = _window(ours, published, dy, dx, c0, c1)
                if w is None:
                    continue
                m = mse(*w)
                if best is None or m < best[0]:
                    best = (m, dy, dx, w[0].size)
        if best is None:
            continue
        se += best[0] * best[3]
        cnt += best[3]
        bands.append((c0, best[1], best[2], round(psnr_from_mse(best[0]), 2)))
    return psnr_from_mse(se / cnt if cnt else 0.0), bands


def compare_published(pano: np.ndarray, published: np.ndarray) -> dict:
    """The PSNR report of a (cropped, pre-JPEG) panorama against a published JPEG's pixels."""
    ours = jpeg_roundtrip(pano)
    rep = {"shape": list(pano.shape), "published_shape": list(published.shape)}
    if ours.shape == published.shape:
        rep["psnr_db"] = round(psnr(ours, published), 3)
        rep["identical_fraction"] = round(float(np.mean(ours == published)), 5)
        rep["alignment"] = "same shape, zero offset"
    else:
        p, bands = band_aligned(ours, published)
        rep["psnr_db"] = round(p, 3)
        offs = {}
        for _, dy, dx, _ in bands:
            offs[f"{dy},{dx}"] = offs.get(f"{dy},{dx}", 0) + 1
        rep["alignment"] = "256-column bands at their best offset within +-3 px"
        rep["band_offsets"] = offs
        rep["worst_band_psnr_db"] = min(b[3] for b in bands)
    return rep
