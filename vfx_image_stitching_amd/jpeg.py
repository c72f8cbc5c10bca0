"""JPEG decode on the GPU: the reference's ``cv2.imread``.

The reference reads every frame with ``cv2.imread(full_p)`` (image_stitching_sift.py:282,
image_stitching_harris.py:394), i.e. libjpeg-turbo's default decode to BGR uint8.
``pano_jpeg_decode`` runs that decode on the GPU for a batch of same-sized baseline files,
bit-identical to libjpeg-turbo (and to PIL, which the harness uses on the host):

    frames = decode_batch([open(p, 'rb').read() for p in paths])   # torch u8 [n, h, w, 3] BGR

Only headers are parsed on the host; the entropy-coded bytes go to the GPU in one copy and
the Huffman decode (self-synchronising, no restart markers needed), the islow IDCT, the fancy
chroma upsampling and the colour conversion run there.  Progressive / arithmetic-coded files
and chroma layouts other than 4:4:4 / 4:2:2 / 4:2:0 raise ``PanoError(PANO_E_UNSUPPORTED)``.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import PanoError, context, ptr


def info(buf: bytes) -> tuple[int, int, int]:
    """(h, w, components) of a JPEG held in memory (host only; raises on unsupported files)."""
    lib = _lib.load()
    h, w, c = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
    b = np.frombuffer(buf, np.uint8)
    rc = lib.pano_jpeg_info(b.ctypes.data_as(ctypes.c_void_p), b.size, ctypes.byref(h), ctypes.byref(w),
                            ctypes.byref(c))
    if rc != _lib.PANO_OK:
        raise PanoError(rc, "pano_jpeg_info: not a supported baseline JPEG")
    return h.value, w.value, c.value


def decode_batch(bufs, out=None, status: bool = False, device: int | None = None):
    """Decode same-sized JPEG files (bytes) into a device tensor u8 [n, h, w, 3] (BGR).

    ``out``: an existing contiguous device tensor of that shape to decode into.
    ``status``: also return the per-frame status tensor (int32 [n], 0 = ok); without it a
    frame whose scan is corrupt or truncated raises after the decode completes.
    """
    import torch
    bufs = [bytes(b) for b in bufs]
    if not bufs:
        raise PanoError(_lib.PANO_E_ARG, "decode_batch: no files")
    h, w, _ = info(bufs[0])
    ctx = context(device)
    dev = torch.device("cuda", ctx.device)
    if out is None:
        out = torch.empty((len(bufs), h, w, 3), dtype=torch.uint8, device=dev)
    elif tuple(out.shape) != (len(bufs), h, w, 3) or out.dtype != torch.uint8:
        raise PanoError(_lib.PANO_E_ARG, f"decode_batch: out must be uint8 {(len(bufs), h, w, 3)}")
    st = torch.empty(len(bufs), dtype=torch.int32, device=dev)
    arrs = [np.frombuffer(b, np.uint8) for b in bufs]
    ptrs = (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    lens = (ctypes.c_size_t * len(arrs))(*[a.size for a in arrs])
    ctx.check(ctx.lib.pano_jpeg_decode(ctx.h, len(arrs), ptrs, lens, ptr(out), h, w, ptr(st)))
    if status:
        return out, st
    s = st.cpu().numpy()
    bad = np.nonzero(s)[0]
    if bad.size:
        raise PanoError(int(s[bad[0]]), f"JPEG frame {int(bad[0])}: corrupt, truncated or unsupported scan")
    return out


def imread(path: str, device: int | None = None):
    """cv2.imread(path) for a baseline JPEG, decoded on the GPU: a torch u8 [h, w, 3] BGR
    device tensor (the reference's array, resident where the stitch needs it)."""
    with open(path, "rb") as f:
        return decode_batch([f.read()], device=device)[0]
