"""Restatement of the OpenCV (cv2) surface used by the reference -- TEST INFRASTRUCTURE.

The reference imports ``cv2`` at module top (sift_impl.py:5, image_stitching_sift.py:2,
image_stitching_harris.py:2).  OpenCV is not installed in this image, so this module
restates exactly the calls the reference makes:

==========================  ===========================================================
cv2 call                    reference call sites
==========================  ===========================================================
cvtColor(BGR2GRAY) uint8    sift_impl.py:28, image_stitching_harris.py:146, :394
resize(fx=fy=2, LINEAR)     sift_impl.py:53
resize(dsize, NEAREST)      sift_impl.py:96
GaussianBlur f32 (0,0),s    sift_impl.py:56,91
GaussianBlur f64 (21,21),2  image_stitching_harris.py:161-163
GaussianBlur f64 (9,9),4.5  image_stitching_harris.py:91
KeyPoint                    sift_impl.py:206,290
imread / imwrite            image_stitching_sift.py:282,386
==========================  ===========================================================

Numeric definitions (these ARE the oracle's definitions):

* BGR2GRAY on uint8 is OpenCV's fixed point ``(1868 B + 9617 G + 4899 R + 8192) >> 14``.
* GaussianBlur on float32 images (the SIFT path) is OpenCV 4.x's arithmetic, pinned by the
  author's published SIFT panoramas (grail pixel-identical): taps from
  getGaussianKernelBitExact cast to f32; ``ksize = rint(8 s + 1) | 1``; a row pass
  ``s = x0*k0; s = fma(x_i, k_i, s)`` in f32 over the taps in order, into an f32 buffer;
  a column pass in the symmetric form ``s = S0*kc; s = fma(S_+i + S_-i, k_i, s)`` in f32,
  i = 1..r outward from the centre (oracle/cv_blur.c).  BORDER_REFLECT_101 with periodic
  repetition for images narrower than the kernel.  Other arithmetic variants stay
  selectable for the sweep (``BLUR_VARIANT``).
* GaussianBlur on float64 images (the Harris path): taps ``t_i = exp(-x_i^2 / (2 s^2))``
  normalised by their double sum, separable, each output accumulated in double in tap
  order (pinned pixel-identically by the published Harris panoramas).
* INTER_LINEAR (x2): ``sx = (dx + 0.5) * inv - 0.5``, clamped at both edges, f32 weights;
  exact for integer-valued inputs.
* INTER_NEAREST: ``sx = min(floor(dx * (1 / (dst_w / src_w))), src_w - 1)``.
* KeyPoint: float32 storage of pt/size/angle/response, angle default -1, class_id -1.
* imread: PIL decode -> BGR uint8 (pixel-identical to cv2.imread for these JPEGs, SURVEY
  section 8c); imwrite: PIL JPEG quality 95.
"""
from __future__ import annotations

import math
import os

import numpy as np

COLOR_BGR2GRAY = 6
COLOR_RGB2GRAY = 7
COLOR_BGR2RGB = 4
COLOR_RGB2BGR = 4
COLOR_GRAY2BGR = 8
COLOR_GRAY2RGB = 8
INTER_NEAREST = 0
INTER_LINEAR = 1
IMREAD_COLOR = 1
IMREAD_GRAYSCALE = 0
BORDER_REFLECT_101 = 4
BORDER_DEFAULT = 4

__version__ = "oracle-restatement"


# --------------------------------------------------------------------------- color
def bgr_to_gray_u8(img: np.ndarray) -> np.ndarray:
    """OpenCV fixed-point BGR->GRAY for uint8 (coefficients 1868/9617/4899, shift 14)."""
    b = img[..., 0].astype(np.int32)
    g = img[..., 1].astype(np.int32)
    r = img[..., 2].astype(np.int32)
    return ((b * 1868 + g * 9617 + r * 4899 + 8192) >> 14).astype(np.uint8)


def cvtColor(img, code):
    img = np.asarray(img)
    if code == COLOR_BGR2GRAY:
        if img.dtype != np.uint8:
            raise NotImplementedError("BGR2GRAY is restated for uint8 only (all reference call sites)")
        return bgr_to_gray_u8(img)
    if code == COLOR_RGB2GRAY:
        return bgr_to_gray_u8(img[..., ::-1])
    if code == COLOR_BGR2RGB:
        return np.ascontiguousarray(img[..., ::-1])
    if code == COLOR_GRAY2BGR:
        return np.ascontiguousarray(np.repeat(img[..., None], 3, axis=2))
    raise NotImplementedError(f"cvtColor code {code}")


# --------------------------------------------------------------------------- resize
def _linear_map(dst_n: int, src_n: int, inv_scale: float):
    """OpenCV INTER_LINEAR source index + f32 weight per destination index."""
    scale = 1.0 / inv_scale
    idx0 = np.empty(dst_n, np.int64)
    idx1 = np.empty(dst_n, np.int64)
    w1 = np.empty(dst_n, np.float32)
    for d in range(dst_n):
        fx = (d + 0.5) * scale - 0.5
        sx = math.floor(fx)
        fx -= sx
        if sx < 0:
            fx, sx = 0.0, 0
        if sx >= src_n - 1:
            fx, sx = 0.0, src_n - 1
        idx0[d] = sx
        idx1[d] = min(sx + 1, src_n - 1)
        w1[d] = np.float32(fx)
    return idx0, idx1, w1


def resize(img, dsize, fx=0.0, fy=0.0, interpolation=INTER_LINEAR):
    img = np.asarray(img)
    h, w = img.shape[:2]
    if dsize is None or tuple(dsize) == (0, 0):
        dw, dh = int(round(w * fx)), int(round(h * fy))
        inv_x, inv_y = float(fx), float(fy)
    else:
        dw, dh = int(dsize[0]), int(dsize[1])
        inv_x, inv_y = dw / w, dh / h
    if interpolation == INTER_NEAREST:
        ifx, ify = 1.0 / inv_x, 1.0 / inv_y
        xs = np.minimum(np.floor(np.arange(dw) * ifx).astype(np.int64), w - 1)
        ys = np.minimum(np.floor(np.arange(dh) * ify).astype(np.int64), h - 1)
        return np.ascontiguousarray(img[ys][:, xs])
    if interpolation == INTER_LINEAR:
        if img.dtype != np.float32:
            raise NotImplementedError("INTER_LINEAR restated for float32 (sift_impl.py:53)")
        x0, x1, wx = _linear_map(dw, w, inv_x)
        y0, y1, wy = _linear_map(dh, h, inv_y)
        wx0 = np.float32(1) - wx
        wy0 = np.float32(1) - wy
        hor = img[:, x0] * wx0 + img[:, x1] * wx          # f32, exact for integer input
        out = hor[y0] * wy0[:, None] + hor[y1] * wy[:, None]
        return out.astype(np.float32)
    raise NotImplementedError(f"interpolation {interpolation}")


# --------------------------------------------------------------------------- gaussian
def gaussian_ksize(sigma: float, depth_is_u8: bool = False) -> int:
    """OpenCV: ksize = cvRound(sigma * (depth==CV_8U ? 3 : 4) * 2 + 1) | 1."""
    v = sigma * (3 if depth_is_u8 else 4) * 2 + 1
    return int(np.rint(v)) | 1


def getGaussianKernel(ksize: int, sigma: float, ktype=np.float64) -> np.ndarray:
    """getGaussianKernel for sigma > 0 (every reference call passes sigma > 0)."""
    if sigma <= 0:
        sigma = ((ksize - 1) * 0.5 - 1) * 0.3 + 0.8
    scale2x = -0.5 / (sigma * sigma)
    dt = np.dtype(ktype)
    taps = np.empty(ksize, dt)
    s = 0.0
    for i in range(ksize):
        x = i - (ksize - 1) * 0.5
        t = math.exp(scale2x * x * x)
        taps[i] = t
        s += float(taps[i])
    s = 1.0 / s
    for i in range(ksize):
        taps[i] = float(taps[i]) * s
    return taps


def getGaussianKernelBitExact(ksize: int, sigma: float) -> np.ndarray:
    """OpenCV 4.x getGaussianKernel (via getGaussianKernelBitExact, imgproc/src/smooth.dispatch.cpp).

    softdouble arithmetic is IEEE double without contraction, which Python floats are; the
    one difference is OpenCV's own softdouble ``exp`` against libm's (both within an ulp of
    double, far below the f32 rounding of the taps).  Per tap: ``exp(x*x * (-0.125 / s^2))``
    with the integer ``x = 1 - n, 3 - n, ...`` (twice the offset), the sum as
    ``2 * sum(side taps) + 1``, and every tap multiplied by ``1 / sum``; the centre tap is
    ``1 / sum`` itself.  Returned as float64 (the caller casts to the kernel dtype).
    """
    if sigma <= 0:
        sigma = ((ksize - 1) * 0.5 - 1) * 0.3 + 0.8
    scale2x = -0.125 / (sigma * sigma)
    n2 = (ksize - 1) // 2
    vals = []
    s = 0.0
    x = 1 - ksize
    for _ in range(n2):
        t = math.exp(float(x * x) * scale2x)
        vals.append(t)
        s += t
        x += 2
    s *= 2.0
    s += 1.0
    if ksize % 2 == 0:
        s += 1.0
    mul1 = 1.0 / s
    out = np.empty(ksize, np.float64)
    if ksize % 2 == 1:
        out[n2] = mul1
    for i in range(n2):
        t = vals[i] * mul1
        out[i] = t
        out[ksize - 1 - i] = t
    return out


# f32 GaussianBlur arithmetic variants (oracle/cv_blur.c).  "taps:row:col" with
#   taps  legacy   -- getGaussianKernel above (f32 taps summed in double; OpenCV 3.x)
#         bitexact -- getGaussianKernelBitExact (OpenCV 4.x)
#   row   f64 | fma | mul   (f64 accumulate; f32 sequential fused; f32 sequential unfused)
#   col   f64 | symfma | symmul | fma   (f32 symmetric pair form fused / unfused; f32 sequential)
# The default, bitexact:fma:symfma (OpenCV 4.x taps; RowVec_32f and SymmColumnVec_32f under
# FMA3), reproduces the author's published SIFT grail panorama pixel for pixel and the
# parrington one at its published shape (tools/blur_variants.py); legacy:f64:f64
# is the round-1/2 definition.
_ROW_MODES = {"f64": 0, "fma": 1, "mul": 2}
_COL_MODES = {"f64": 0, "symfma": 1, "symmul": 2, "fma": 3}
DEFAULT_BLUR = "bitexact:fma:symfma"
BLUR_VARIANT = os.environ.get("CV2_COMPAT_BLUR", DEFAULT_BLUR)
_CVB = None


def set_blur_variant(spec: str) -> None:
    global BLUR_VARIANT
    taps, row, col = spec.split(":")
    if taps not in ("legacy", "bitexact") or row not in _ROW_MODES or col not in _COL_MODES:
        raise ValueError(f"blur variant {spec!r}")
    BLUR_VARIANT = spec


def _cv_blur_lib():
    global _CVB
    if _CVB is None:
        import ctypes
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libcv_blur.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle`")
        lib = ctypes.CDLL(path)
        fp = ctypes.POINTER(ctypes.c_float)
        lib.cvb_gaussian_f32.argtypes = [fp, fp, fp, ctypes.c_int, ctypes.c_int, fp, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int]
        lib.cvb_gaussian_f32.restype = ctypes.c_int
        _CVB = lib
    return _CVB


def gaussian_f32_variant(img: np.ndarray, ksize: int, sigma: float, spec: str) -> np.ndarray:
    """Square-kernel f32 GaussianBlur under an arithmetic variant (see BLUR_VARIANT)."""
    import ctypes
    taps, row, col = spec.split(":")
    if taps == "legacy":
        k = getGaussianKernel(ksize, sigma, np.float32)
    else:
        k = getGaussianKernelBitExact(ksize, sigma).astype(np.float32)
    k = np.ascontiguousarray(k, np.float32)
    src = np.ascontiguousarray(img, np.float32)
    h, w = src.shape
    dst = np.empty_like(src)
    tmp = np.empty_like(src)
    fp = ctypes.POINTER(ctypes.c_float)
    rc = _cv_blur_lib().cvb_gaussian_f32(src.ctypes.data_as(fp), dst.ctypes.data_as(fp),
                                         tmp.ctypes.data_as(fp), h, w, k.ctypes.data_as(fp),
                                         ksize, _ROW_MODES[row], _COL_MODES[col])
    if rc != 0:
        raise ValueError("cvb_gaussian_f32 refused its arguments")
    return dst


def reflect101(idx: np.ndarray, n: int) -> np.ndarray:
    """BORDER_REFLECT_101 index map, periodic for offsets beyond one reflection."""
    if n == 1:
        return np.zeros_like(idx)
    period = 2 * n - 2
    i = np.mod(idx, period)
    return np.where(i >= n, period - i, i)


def sep_filter_pass(img: np.ndarray, taps: np.ndarray, axis: int, out_dtype) -> np.ndarray:
    """One separable pass: sum_i taps[i] * img[refl(x + i - r)] in double, tap order."""
    n = img.shape[axis]
    r = (len(taps) - 1) // 2
    base = np.arange(n)
    src = img.astype(np.float64)
    acc = np.zeros(src.shape, np.float64)
    for i in range(len(taps)):
        idx = reflect101(base + i - r, n)
        acc += float(taps[i]) * np.take(src, idx, axis=axis)
    return acc.astype(out_dtype)


def GaussianBlur(img, ksize, sigmaX, dst=None, sigmaY=0, borderType=BORDER_REFLECT_101):
    img = np.asarray(img)
    if img.dtype not in (np.float32, np.float64):
        raise NotImplementedError("GaussianBlur restated for float32/float64 images only")
    if sigmaY is None or sigmaY <= 0:
        sigmaY = sigmaX
    kw, kh = (int(ksize[0]), int(ksize[1])) if ksize is not None else (0, 0)
    if kw <= 0:
        kw = gaussian_ksize(sigmaX)
    if kh <= 0:
        kh = gaussian_ksize(sigmaY)
    kt = img.dtype.type
    if kt is np.float32 and BLUR_VARIANT != "legacy:f64:f64":
        if kw != kh or sigmaX != sigmaY or img.ndim != 2:
            raise NotImplementedError("f32 GaussianBlur restated for square kernels (all call sites)")
        return gaussian_f32_variant(img, kw, sigmaX, BLUR_VARIANT)
    kx = getGaussianKernel(kw, sigmaX, kt)
    ky = getGaussianKernel(kh, sigmaY, kt)
    if img.ndim != 2:
        raise NotImplementedError("GaussianBlur restated for single-channel images")
    rows = sep_filter_pass(img, kx, axis=1, out_dtype=kt)
    return sep_filter_pass(rows, ky, axis=0, out_dtype=kt)


# --------------------------------------------------------------------------- KeyPoint
class KeyPoint:
    """cv2.KeyPoint restatement: float32 storage, Python-float read-back."""

    __slots__ = ("_x", "_y", "_size", "_angle", "_response", "octave", "class_id")

    def __init__(self, x=0.0, y=0.0, size=0.0, angle=-1.0, response=0.0, octave=0, class_id=-1):
        self._x = np.float32(x)
        self._y = np.float32(y)
        self._size = np.float32(size)
        self._angle = np.float32(angle)
        self._response = np.float32(response)
        self.octave = int(octave)
        self.class_id = int(class_id)

    @property
    def pt(self):
        return (float(self._x), float(self._y))

    @pt.setter
    def pt(self, v):
        self._x = np.float32(v[0])
        self._y = np.float32(v[1])

    size = property(lambda s: float(s._size), lambda s, v: setattr(s, "_size", np.float32(v)))
    angle = property(lambda s: float(s._angle), lambda s, v: setattr(s, "_angle", np.float32(v)))
    response = property(lambda s: float(s._response),
                        lambda s, v: setattr(s, "_response", np.float32(v)))

    def __repr__(self):
        return (f"KeyPoint(pt={self.pt}, size={self.size}, angle={self.angle}, "
                f"response={self.response}, octave={self.octave})")


# --------------------------------------------------------------------------- I/O
def imread(path, flags=IMREAD_COLOR):
    from PIL import Image
    if not os.path.exists(path):
        return None
    with Image.open(path) as im:
        rgb = np.asarray(im.convert("RGB"))
    bgr = np.ascontiguousarray(rgb[..., ::-1])
    if flags == IMREAD_GRAYSCALE:
        return bgr_to_gray_u8(bgr)
    return bgr


_WRITES: dict = {}


def imwrite(path, img, params=None):
    """JPEG q95 via PIL.  The array is also kept in ``_WRITES`` for the golden generator."""
    from PIL import Image
    img = np.asarray(img)
    _WRITES[path] = img.copy()
    if os.environ.get("CV2_COMPAT_NO_DISK"):
        return True
    rgb = img[..., ::-1] if img.ndim == 3 else img
    Image.fromarray(np.ascontiguousarray(rgb)).save(path, quality=95)
    return True


def jpeg_q95_roundtrip(img_bgr: np.ndarray) -> np.ndarray:
    """Encode with PIL q95 and decode again (how the published JPEGs were produced)."""
    import io
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(np.ascontiguousarray(img_bgr[..., ::-1])).save(buf, format="JPEG", quality=95)
    buf.seek(0)
    with Image.open(buf) as im:
        return np.ascontiguousarray(np.asarray(im.convert("RGB"))[..., ::-1])
