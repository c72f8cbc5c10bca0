"""Input sequences: the reference's image sets (packed under data/) and a synthetic generator.

``load_set('parrington')`` returns the frames in pano.txt order with their focal lengths,
exactly what run_panorama feeds its loop (image_stitching_sift.py:270-296).  The JPEG bytes
are stored verbatim in data/<set>_frames.npz (tests/golden/make_golden.py pack) and decoded
with PIL, which is pixel-identical to cv2.imread for these files.

``synthetic_sequence`` implements SURVEY.md section 8(d) config 5 (band-limited noise strip,
inverse-cylinder warped frames with a known step and vertical jitter).
"""
from __future__ import annotations

import io
import os

import numpy as np

DATA_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data")


def decode_jpeg(buf: bytes) -> np.ndarray:
    from PIL import Image
    with Image.open(io.BytesIO(buf)) as im:
        rgb = np.asarray(im.convert("RGB"))
    return np.ascontiguousarray(rgb[..., ::-1])


def load_set(name: str, data_dir: str = DATA_DIR):
    """-> (names, frames uint8 [n, h, w, 3] BGR, focals float64 [n], crop margin)."""
    z = np.load(os.path.join(data_dir, f"{name}_frames.npz"), allow_pickle=False)
    names = [str(s) for s in z["order"]]
    frames = np.stack([decode_jpeg(z[f"jpg_{n}"].tobytes()) for n in names])
    return names, frames, z["focals"].astype(np.float64), int(z["margin"])


def pair_frame(name: str, a: str, b: str, data_dir: str = DATA_DIR):
    """Two named frames of a set with their focals (config 2: prtn00 + prtn01)."""
    names, frames, focals, _ = load_set(name, data_dir)
    ia, ib = names.index(a), names.index(b)
    return frames[[ia, ib]], focals[[ia, ib]]


def cyclic_sequence(frames: np.ndarray, focals: np.ndarray, start: int, count: int):
    """Frames start, start+1, ... (mod n) of a 360-degree set (parrington is a full loop)."""
    n = len(frames)
    idx = [(start + k) % n for k in range(count)]
    return frames[idx], focals[idx]


def _blur_noise(rng, h, w, sigma):
    from scipy.ndimage import gaussian_filter
    return gaussian_filter(rng.standard_normal((h, w)), sigma, mode="wrap")


def synthetic_strip(height=1080, period=144 * 1229, seed=0):
    """Periodic texture strip: sum_s s * G_s(N(0,1)), scaled to 128 +- 45 z, 3 channels."""
    rng = np.random.default_rng(seed)
    acc = np.zeros((height, period))
    for s in (1.5, 4.0, 12.0, 32.0):
        acc += s * _blur_noise(rng, height, period, s)
    z = (acc - acc.mean()) / acc.std()
    base = 128 + 45 * z
    tint = np.array([0.95, 1.0, 1.05])
    return np.clip(base[..., None] * tint, 0, 255).astype(np.uint8)


def synthetic_sequence(n_frames=144, h=1080, w=1920, step=1229, focal=1600.0, seed=0,
                       jitter_seed=1, strip=None):
    """Frames whose cylindrical projections are shifted copies of one strip.

    Frame i samples the strip at columns starting at -i*step (mod period) through the
    inverse cylindrical map, so cylindrical_projection(frame_i) ~ strip window; ground
    truth dx = -step, dy = jitter[i+1] - jitter[i].
    """
    period = n_frames * step
    if strip is None:
        strip = synthetic_strip(h + 16, period, seed)
    jit = np.random.default_rng(jitter_seed).integers(-3, 4, n_frames)
    cx, cy = w // 2, h // 2
    xs = np.arange(w) - cx
    ys = np.arange(h) - cy
    # inverse cylinder: source pixel (x, y) of the planar frame sees cylinder column
    # f*atan(x/f) and height f*y/sqrt(x^2+f^2)
    xc = focal * np.arctan(xs / focal)
    yc = focal * ys[:, None] / np.sqrt(xs[None, :] ** 2 + focal ** 2)
    frames = np.empty((n_frames, h, w, 3), np.uint8)
    for i in range(n_frames):
        col = (np.rint(xc + cx).astype(np.int64) - i * step) % period
        row = np.clip(np.rint(yc + cy + 8 + jit[i]).astype(np.int64), 0, strip.shape[0] - 1)
        frames[i] = strip[row, col[None, :]]
    return frames, np.full(n_frames, focal), jit
