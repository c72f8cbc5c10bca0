"""Corrupt-JPEG corpus for the host sanitizer run (tools/host_sanitize.sh; SURVEY.md section 5,
"Race detection / sanitizers").

Seeds: the first packed reference frame of parrington, grail and out (data/*_frames.npz: the
reference's own files) and small PIL encodes of every sampling / table variant the decoder
accepts.  Mutations, each written as its own file:

* truncation at every header offset (step 3) and at random scan offsets;
* 1-3 random bit flips inside the header segments (DQT / DHT / SOF / SOS bytes);
* segment length fields replaced by 0, 1, 2, 0xFFFF and random values;
* random bytes (including 0xFF, i.e. new markers) written into the entropy-coded segment;
* a second JPEG and junk appended after EOI; a missing EOI; a doubled SOI.

    python tools/make_fuzz_corpus.py OUT_DIR [--small]
"""
from __future__ import annotations

import io
import os
import sys

import numpy as np
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _encode(arr, **kw):
    b = io.BytesIO()
    Image.fromarray(arr).save(b, "JPEG", **kw)
    return b.getvalue()


def _seeds(small: bool):
    rng = np.random.default_rng(0)
    out = []
    if not small:
        for name in ("parrington", "grail", "out"):
            z = np.load(os.path.join(ROOT, "data", f"{name}_frames.npz"), allow_pickle=False)
            out.append((f"{name}0", z[f"jpg_{z['order'][0]}"].tobytes()))
    tex = np.clip(128 + 50 * rng.standard_normal((48, 72, 3)), 0, 255).astype(np.uint8)
    for i, kw in enumerate((dict(quality=95), dict(quality=90, subsampling=0), dict(quality=85, subsampling=1),
                            dict(quality=80, optimize=True), dict(quality=30))):
        out.append((f"v{i}", _encode(tex, **kw)))
    out.append(("gray", _encode(tex[..., 0], quality=90)))
    return out


def _segments(buf: bytes):
    """(marker, offset of its length field, length) of every header segment up to SOS."""
    segs, i = [], 2
    while i + 4 <= len(buf) and buf[i] == 0xFF:
        m = buf[i + 1]
        ln = buf[i + 2] << 8 | buf[i + 3]
        segs.append((m, i + 2, ln))
        if m == 0xDA:
            break
        i += 2 + ln
    return segs


def mutate(buf: bytes, rng, n_trunc: int):
    segs = _segments(buf)
    sos = segs[-1]
    hdr_end = sos[1] + sos[2]
    yield "orig", buf
    for k, off in enumerate(range(2, hdr_end + 4, 3)):
        yield f"trunc_h{k}", buf[:off]
    for k, off in enumerate(rng.integers(hdr_end, len(buf), n_trunc)):
        yield f"trunc_s{k}", buf[:off]
    for k in range(60):
        b = bytearray(buf)
        for _ in range(int(rng.integers(1, 4))):
            p = int(rng.integers(2, hdr_end))
            b[p] ^= 1 << int(rng.integers(0, 8))
        yield f"flip{k}", bytes(b)
    for k, (m, lo, ln) in enumerate(segs):
        for v in (0, 1, 2, 0xFFFF, int(rng.integers(3, 400))):
            b = bytearray(buf)
            b[lo], b[lo + 1] = v >> 8, v & 255
            yield f"len{k}_{v}", bytes(b)
    for k in range(20):
        b = bytearray(buf)
        for p in rng.integers(hdr_end, len(buf) - 2, int(rng.integers(1, 30))):
            b[int(p)] = int(rng.integers(0, 256))
        yield f"scan{k}", bytes(b)
    yield "trailer", buf + buf[: len(buf) // 3] + b"\xff\x00junk\xff"
    yield "no_eoi", buf[:-2]
    yield "soi2", buf[:2] + buf


def main():
    out_dir = sys.argv[1]
    small = "--small" in sys.argv
    os.makedirs(out_dir, exist_ok=True)
    rng = np.random.default_rng(1)
    n = 0
    for name, buf in _seeds(small):
        for tag, b in mutate(buf, rng, 4 if name[0] != "v" else 10):
            with open(os.path.join(out_dir, f"{name}_{tag}.jpg"), "wb") as f:
                f.write(b)
            n += 1
    print(n)


if __name__ == "__main__":
    main()
