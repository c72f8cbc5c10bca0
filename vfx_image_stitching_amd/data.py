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


def load_set_jpegs(name: str, data_dir: str = DATA_DIR):
    """-> (names, JPEG file bytes) in pano.txt order: what cv2.imread reads
    (image_stitching_sift.py:282), for the GPU decode (vfx_image_stitching_amd.jpeg)."""
    z = np.load(os.path.join(data_dir, f"{name}_frames.npz"), allow_pickle=False)
    names = [str(s) for s in z["order"]]
    return names, [z[f"jpg_{n}"].tobytes() for n in names]


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


# Synthetic texture.  Band-limited value noise: four lattices
# (spacing 3, 8, 18, 48 px) of hashed uniform values, smoothstep-interpolated and summed.
# Every pixel is a pure function of its strip position (no global filter, no global
# normalisation), so any window of the strip -- one rank's frames, one frame -- is generated
# independently and bit-identically: rank r builds only the frames it owns.
_LATTICES = ((3, 1.0), (8, 1.6), (18, 2.4), (48, 3.0))   # (spacing px, amplitude)
_NOISE_STD = 1.84                                         # std of the lattice sum (measured)
_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def _hash01(seed: int, sid: int, ix: np.ndarray, iy: np.ndarray) -> np.ndarray:
    """splitmix64 of (seed, lattice id, ix, iy) -> float32 in [-1, 1)."""
    with np.errstate(over="ignore"):
        h = (ix.astype(np.uint64)[None, :] * np.uint64(0x9E3779B97F4A7C15)) ^ \
            (iy.astype(np.uint64)[:, None] * np.uint64(0xC2B2AE3D27D4EB4F)) ^ \
            np.uint64(((seed * 64 + sid) * 0x165667B19E3779F9) & 0xFFFFFFFFFFFFFFFF)
        h ^= h >> np.uint64(30)
        h *= np.uint64(0xBF58476D1CE4E5B9)
        h ^= h >> np.uint64(27)
        h *= np.uint64(0x94D049BB133111EB)
        h ^= h >> np.uint64(31)
    return (h >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -23) - np.float32(1.0)


def _smooth(t: np.ndarray) -> np.ndarray:
    return (t * t * (np.float32(3.0) - np.float32(2.0) * t)).astype(np.float32)


def synthetic_strip_window(u0: int, u1: int, height: int, period: int, seed: int = 0) -> np.ndarray:
    """Columns u0..u1 (unwrapped; the strip repeats every `period`) -> uint8 [height, u1-u0, 3]."""
    u = np.arange(u0, u1, dtype=np.int64) % period
    y = np.arange(height, dtype=np.int64)
    acc = np.zeros((height, u1 - u0), np.float32)
    for sid, (sp, amp) in enumerate(_LATTICES):
        L = max(1, period // sp)                       # lattice cells around the loop
        ix = u // sp
        tx = _smooth(((u - ix * sp).astype(np.float32) + np.float32(0.5)) / np.float32(sp))
        ix0, ix1 = ix % L, (ix + 1) % L
        iy = y // sp
        ty = _smooth(((y - iy * sp).astype(np.float32) + np.float32(0.5)) / np.float32(sp))
        lo, hi = int(iy.min()), int(iy.max()) + 1
        ly = np.arange(lo, hi + 1)
        cols = np.unique(np.concatenate([ix0, ix1]))
        lat = _hash01(seed, sid, cols, ly)             # [rows of lattice, used lattice cols]
        c0 = np.searchsorted(cols, ix0)
        c1 = np.searchsorted(cols, ix1)
        rows = lat[:, c0] + (lat[:, c1] - lat[:, c0]) * tx[None, :]          # x interpolation
        r0 = rows[iy - lo]
        r1 = rows[iy + 1 - lo]
        acc += np.float32(amp) * (r0 + (r1 - r0) * ty[:, None])             # y interpolation
    base = np.float32(128.0) + np.float32(45.0 / _NOISE_STD) * acc
    tint = np.array([0.95, 1.0, 1.05], np.float32)
    return np.clip(base[..., None] * tint, 0, 255).astype(np.uint8)


def synthetic_sequence(n_frames=144, h=1080, w=1920, step=1229, focal=1600.0, seed=0,
                       jitter_seed=1, start=0, count=None):
    """Frames start..start+count of a sequence whose cylindrical projections are shifted
    copies of one periodic strip (period n_frames * step).

    Frame i samples the strip at columns starting at -i*step through the inverse cylindrical
    map, so cylindrical_projection(frame_i) ~ strip window; ground truth dx = -step,
    dy = jitter[i+1] - jitter[i].  Frames do not depend on (start, count): any shard of the
    sequence is generated on its own.  Returns (frames, focals, jitter of those frames).
    """
    count = n_frames - start if count is None else count
    period = n_frames * step
    jit = np.random.default_rng(jitter_seed).integers(-3, 4, n_frames)
    cx, cy = w // 2, h // 2
    xs = np.arange(w) - cx
    ys = np.arange(h) - cy
    # inverse cylinder: source pixel (x, y) of the planar frame sees cylinder column
    # f*atan(x/f) and height f*y/sqrt(x^2+f^2)
    xc = focal * np.arctan(xs / focal)
    yc = focal * ys[:, None] / np.sqrt(xs[None, :] ** 2 + focal ** 2)
    colbase = np.rint(xc + cx).astype(np.int64)
    last = start + count - 1
    u0 = int(colbase.min()) - last * step
    u1 = int(colbase.max()) - start * step + 1
    strip = synthetic_strip_window(u0, u1, h + 16, period, seed)
    frames = np.empty((count, h, w, 3), np.uint8)
    for k in range(count):
        i = start + k
        col = colbase - i * step - u0
        row = np.clip(np.rint(yc + cy + 8 + jit[i]).astype(np.int64), 0, strip.shape[0] - 1)
        frames[k] = strip[row, col[None, :]]
    return frames, np.full(count, focal), jit[start:start + count]
