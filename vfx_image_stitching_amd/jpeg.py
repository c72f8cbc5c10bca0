"""JPEG decode and encode on the GPU: the reference's ``cv2.imread``
and ``cv2.imwrite``.

The reference reads every frame with ``cv2.imread(full_p)`` (image_stitching_sift.py:282,
image_stitching_harris.py:394), i.e. libjpeg-turbo's default decode to BGR uint8.
``pano_jpeg_decode`` runs that decode on the GPU for a batch of same-sized baseline files,
bit-identical to libjpeg-turbo (and to PIL, which the harness uses on the host):

    frames = decode_batch([open(p, 'rb').read() for p in paths])   # torch u8 [n, h, w, 3] BGR

``encode(img)`` is the reference's ``cv2.imwrite(path, panorama)`` (image_stitching_sift.py:386,
OpenCV's default quality 95): the file bytes, byte-identical to libjpeg-turbo's encoder (PIL's
``save(quality=q)``), computed on the GPU from the device image (a crop view is fine).

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


def last_stats(n: int, device: int | None = None) -> np.ndarray:
    """Per-frame synchronisation statistics of the last decode on this device: int32 [n, 4] =
    (subsequences, extra candidates, serial decodes, 0) -- pano_jpeg_stats."""
    ctx = context(device)
    out = np.zeros((n, 4), np.int32)
    ctx.check(ctx.lib.pano_jpeg_stats(ctx.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), n))
    return out


def imread(path: str, device: int | None = None):
    """cv2.imread(path) for a baseline JPEG, decoded on the GPU: a torch u8 [h, w, 3] BGR
    device tensor (the reference's array, resident where the stitch needs it)."""
    with open(path, "rb") as f:
        return decode_batch([f.read()], device=device)[0]


def encode(img, quality: int = 95) -> bytes:
    """JPEG file bytes of a u8 [h, w, 3] BGR device tensor (row-contiguous pixels; any row
    stride, e.g. the panorama view of the canvas), encoded on the GPU."""
    import torch
    if not img.is_cuda or img.dtype != torch.uint8 or img.dim() != 3 or img.shape[2] != 3:
        raise PanoError(_lib.PANO_E_ARG, "encode: expected a uint8 [h, w, 3] device tensor")
    if img.stride(2) != 1 or img.stride(1) != 3:
        raise PanoError(_lib.PANO_E_ARG, "encode: pixels of a row must be contiguous")
    h, w = int(img.shape[0]), int(img.shape[1])
    ctx = context(img.device.index)
    cap = ctypes.c_size_t(0)
    size = 1024 + h * w * 4
    # the file bytes come back through a pinned buffer kept per device (a pageable destination
    # makes the device -> host copy a staged one)
    out = _ENC_PIN.get(ctx.device)
    if out is None or out.numel() < size:
        out = _ENC_PIN[ctx.device] = torch.empty(max(size, 1 << 20), dtype=torch.uint8, pin_memory=True)
    rc = ctx.lib.pano_jpeg_encode(ctx.h, ctypes.c_void_p(img.data_ptr()), h, w, img.stride(0), int(quality),
                                  ctypes.c_void_p(out.data_ptr()), size, ctypes.byref(cap))
    ctx.check(rc)
    return out.numpy()[:cap.value].tobytes()


_ENC_PIN = {}                 # device -> pinned u8 buffer of pano_jpeg_encode's output


def imwrite(path: str, img, quality: int = 95) -> bool:
    """cv2.imwrite(path, img) for a device image, encoded on the GPU."""
    with open(path, "wb") as f:
        f.write(encode(img, quality))
    return True
