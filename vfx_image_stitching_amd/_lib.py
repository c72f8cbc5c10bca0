"""ctypes binding of libpano.so (include/pano.h).

This is the ONLY way the package reaches the GPU: every compute entry point of the
reference-compatible API below goes through these symbols.  There is deliberately no CPU
fallback; if the shared library is missing or no HIP device is present, calls raise.
torch is used only to own device buffers and to provide the current HIP stream.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PANO_CTX_TAIL_MAIN = 1        # pano_ctx_set_flags: the blur tail on the context's own stream
PANO_CTX_MATCH_WHOLE = 2      # pano_ctx_set_flags: no candidate splits in the distance GEMM
# PANO_LIB: an alternative build of the same ABI (A/B timing of two revisions, tools/ab_build.sh)
LIB_PATH = os.environ.get("PANO_LIB") or os.path.join(_HERE, "libpano.so")

PANO_OK = 0
PANO_E_ARG = -1
PANO_E_HIP = -2
PANO_E_OVERFLOW = -3
PANO_E_NOMATCH = -4
PANO_E_UNSUPPORTED = -5
DESC_DIM = 128
ORI_MAX_PEAKS = 18          # PANO_ORI_MAX_PEAKS


class PanoError(RuntimeError):
    """Raised when a libpano call returns a non-zero status."""

    def __init__(self, code, msg):
        super().__init__(f"libpano error {code}: {msg}")
        self.code = code


class KP(ctypes.Structure):
    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("size", ctypes.c_float),
                ("angle", ctypes.c_float), ("response", ctypes.c_float),
                ("octave", ctypes.c_int32)]


KP_NP = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                  ("response", "<f4"), ("octave", "<i4")])


class SiftParams(ctypes.Structure):
    _fields_ = [("sigma", ctypes.c_double), ("num_intervals", ctypes.c_int32),
                ("assumed_blur", ctypes.c_double), ("border", ctypes.c_int32),
                ("contrast_threshold", ctypes.c_double), ("eigen_ratio", ctypes.c_double),
                ("max_iter", ctypes.c_int32), ("radius_factor", ctypes.c_double),
                ("peak_ratio", ctypes.c_double), ("scale_factor", ctypes.c_double),
                ("scale_multiplier", ctypes.c_double), ("descriptor_max", ctypes.c_double)]


class PairRec(ctypes.Structure):
    _fields_ = [("dx", ctypes.c_double), ("dy", ctypes.c_double), ("xA", ctypes.c_double),
                ("yA", ctypes.c_double), ("xB", ctypes.c_double), ("yB", ctypes.c_double),
                ("n_matches", ctypes.c_int32), ("votes", ctypes.c_int32),
                ("best", ctypes.c_int32), ("status", ctypes.c_int32)]


PAIR_NP = np.dtype([("dx", "<f8"), ("dy", "<f8"), ("xA", "<f8"), ("yA", "<f8"),
                    ("xB", "<f8"), ("yB", "<f8"), ("n_matches", "<i4"), ("votes", "<i4"),
                    ("best", "<i4"), ("status", "<i4")])


class HomographyRec(ctypes.Structure):
    _fields_ = [("H", ctypes.c_double * 9), ("n_matches", ctypes.c_int32),
                ("inliers", ctypes.c_int32), ("hyp_inliers", ctypes.c_int32),
                ("status", ctypes.c_int32)]


HOMOGRAPHY_NP = np.dtype([("H", "<f8", (9,)), ("n_matches", "<i4"), ("inliers", "<i4"),
                          ("hyp_inliers", "<i4"), ("status", "<i4")])


class Step(ctypes.Structure):
    _fields_ = [("frame_x", ctypes.c_int32), ("frame_y", ctypes.c_int32),
                ("canvas_x", ctypes.c_int32), ("canvas_y", ctypes.c_int32),
                ("canvas_h", ctypes.c_int32), ("canvas_w", ctypes.c_int32),
                ("frame_is_a", ctypes.c_int32), ("pad", ctypes.c_int32),
                ("overlap_range", ctypes.c_double)]


_P = ctypes.c_void_p
_I = ctypes.c_int
_D = ctypes.c_double
_PI32 = ctypes.POINTER(ctypes.c_int32)
_PD = ctypes.POINTER(ctypes.c_double)

# symbol -> (restype, argtypes); mirrors include/pano.h one to one
SIGNATURES = {
    "pano_ctx_create": (_I, [_I, _P, ctypes.POINTER(_P)]),
    "pano_ctx_destroy": (_I, [_P]),
    "pano_ctx_set_stream": (_I, [_P, _P]),
    "pano_ctx_set_flags": (_I, [_P, _I]),
    "pano_ctx_reserve": (_I, [_P, _I, _I, _I, _I]),
    "pano_sync": (_I, [_P]),
    "pano_ctx_release_scratch": (_I, [_P]),
    "pano_last_error": (ctypes.c_char_p, [_P]),
    "pano_ctx_generation": (ctypes.c_uint64, [_P]),
    "pano_version": (ctypes.c_char_p, []),
    "pano_sift_default_params": (None, [ctypes.POINTER(SiftParams)]),
    "pano_sift_plan": (_I, [ctypes.POINTER(SiftParams), _I, _I, _PI32, _PI32, _PD, _PD]),
    "pano_sift_taps": (_I, [_D, _PD, _PI32]),
    "pano_cylindrical": (_I, [_P, _P, _P, _I, _I, _I, _PD, _P]),
    "pano_sift": (_I, [_P, _P, _I, _I, _I, ctypes.POINTER(SiftParams), _P, _P, _I, _P]),
    "pano_sift_u8": (_I, [_P, _P, _I, _I, _I, ctypes.POINTER(SiftParams), _P, _P, _P, _I, _P]),
    "pano_sift_pyramid": (_I, [_P, _P, _I, _I, _I, ctypes.POINTER(SiftParams)]),
    "pano_sift_base": (_I, [_P, _P, _I, _I, _I, ctypes.POINTER(SiftParams), _P]),
    "pano_sift_pyramid_base": (_I, [_P, _P, _I, _I, _I, _I, ctypes.POINTER(SiftParams)]),
    "pano_sift_pyramid_kernels": (_I, [_P, _P, _I, _I, _I, _I, ctypes.POINTER(ctypes.c_double), _I]),
    "pano_sift_reserve_levels": (_I, [_P, _I, _I, _I, _I, _I]),
    "pano_sift_set_level": (_I, [_P, _I, _I, _I, _I, _P]),
    "pano_sift_dog": (_I, [_P]),
    "pano_sift_extrema": (_I, [_P, ctypes.POINTER(SiftParams), _P, _I, _P]),
    "pano_sift_describe": (_I, [_P, ctypes.POINTER(SiftParams), _P, _P, _I, _P]),
    "pano_sift_localize": (_I, [_P, ctypes.POINTER(SiftParams), ctypes.POINTER(_P), _I, _I, _I, _I, _P, _I,
                                _P, _P]),
    "pano_sift_orient": (_I, [_P, ctypes.POINTER(SiftParams), _P, _I, _I, _I, _P, _I, _P, _P]),
    "pano_sift_level_shape": (_I, [_P, _I, _PI32, _PI32, _PI32]),
    "pano_sift_copy_level": (_I, [_P, _I, _I, _I, _I, _P]),
    "pano_harris": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P]),
    "pano_match": (_I, [_P, _P, _P, _I, _PI32, _I, _I, _P, _P, _P]),
    "pano_match_u8": (_I, [_P, _P, _P, _P, _I, _PI32, _I, _P, _P, _P]),
    "pano_pair_shifts": (_I, [_P, _P, _P, _P, _I, _PI32, _I, _P, _P, _P, _D, _D, _D, _P]),
    "pano_ransac_translate": (_I, [_P, _P, _I, _D, _P]),
    "pano_pair_homography": (_I, [_P, _P, _P, _I, _PI32, _I, _P, _P, _P, _D, _D, _D, _I,
                                  ctypes.c_uint64, _I, _P, _P]),
    "pano_plan_composite": (_I, [_PD, _PD, _I, _I, _I, ctypes.POINTER(Step), _PI32, _PI32]),
    "pano_composite": (_I, [_P, _P, _P, _I, _I, _I, ctypes.POINTER(Step), _PI32, _P, _I, _I]),
    "pano_composite_bbox": (_I, [_P, _P, _P, _I, _I, _I, ctypes.POINTER(Step), _PI32, _P, _I, _I,
                                 _I, _P]),
    "pano_plan_device_bytes": (ctypes.c_size_t, []),
    "pano_plan_device": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "pano_band_plan": (_I, [_P, _P, _I, _I, _I, _I, _P, _P]),
    "pano_band_layout_row": (_I, [_P, _P, _P, _P, _P]),
    "pano_composite_planned": (_I, [_P, _P, _P, _I, _I, _I, _P, _P, _I, _I, _I, _P]),
    "pano_plan_composite_device": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _I, _I, _I, _P]),
    "pano_composite_sequential": (_I, [_P, _P, _P, _I, _I, _I, ctypes.POINTER(Step), _PI32, _P,
                                       _I, _I]),
    "pano_blend_geometry": (_I, [_D, _D, _PD, _I, _I, _I, _I, _PI32, _PD]),
    "pano_blend_two": (_I, [_P, _P, _I, _I, _P, _I, _I, _PI32, _D, _P]),
    "pano_gray_bbox": (_I, [_P, _P, _I, _I, _I, _P]),
    "pano_gray_bgr_f32": (_I, [_P, _P, _I, _I, _I, _P]),
    "pano_desc_norms_u8": (_I, [_P, _P, _I, _P]),
    "pano_jpeg_info": (_I, [_P, ctypes.c_size_t, _PI32, _PI32, _PI32]),
    "pano_jpeg_decode": (_I, [_P, _I, _P, _P, _P, _I, _I, _P]),
    "pano_jpeg_stats": (_I, [_P, _PI32, _I]),
    "pano_jpeg_encode": (_I, [_P, _P, _I, _I, ctypes.c_int64, _I, _P, ctypes.c_size_t,
                              ctypes.POINTER(ctypes.c_size_t)]),
    "pano_prof_enable": (_I, [_P, _I]),
    "pano_prof_read": (_I, [_P, _I, ctypes.POINTER(ctypes.c_int), _PD, _PD, _PD]),
    "pano_graph_begin": (_I, [_P]),
    "pano_graph_end": (_I, [_P, ctypes.POINTER(_P)]),
    "pano_graph_launch": (_I, [_P, _P]),
    "pano_graph_launch_sync": (_I, [_P, _P, _P]),
    "pano_graph_launch_stream": (_I, [_P, _P, _P]),
    "pano_copy_async": (_I, [_P, _P, _P, ctypes.c_size_t]),
    "pano_graph_prof": (_I, [_P, _I, ctypes.POINTER(ctypes.c_int), _PD]),
    "pano_graph_destroy": (_I, [_P]),
}

# kernel classes of pano_prof_enable (include/pano.h PANO_K_*)
KERNELS = ["cyl_scatter", "cyl_gather", "blur_level", "extrema_localize", "orientation",
           "sort_dedup", "descriptor", "row_norms", "dist_mfma", "dist_direct", "reduce_parts",
           "pair_shifts", "composite_step", "gray_bbox", "to_gray", "structure_blur", "response",
           "nms", "select_top", "harris_desc", "jpeg_decode"]
K_ALL = len(KERNELS)

_lib = None
_lock = threading.Lock()


def load(path: str = LIB_PATH):
    """Load libpano.so and declare every exported signature (no GPU needed)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise PanoError(PANO_E_ARG, f"{path} not built (run __graft_entry__.build())")
            lib = ctypes.CDLL(path)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def default_sift_params(**overrides) -> SiftParams:
    p = SiftParams()
    load().pano_sift_default_params(ctypes.byref(p))
    for k, v in overrides.items():
        setattr(p, k, v)
    return p


# ----------------------------------------------------------------------------- context
class Context:
    """One libpano context per (device, stream).  Owns the library's scratch memory."""

    def __init__(self, device: int = 0):
        import torch
        if not torch.cuda.is_available():
            raise PanoError(PANO_E_HIP, "no HIP device visible: the HIP path is the only path")
        self.h = None
        self.device = device
        self.lib = load()
        self._torch = torch
        h = _P()
        stream = torch.cuda.current_stream(device).cuda_stream
        rc = self.lib.pano_ctx_create(device, _P(stream), ctypes.byref(h))
        if rc != PANO_OK:
            raise PanoError(rc, "pano_ctx_create failed")
        self.h = h

    def check(self, rc):
        if rc != PANO_OK:
            raise PanoError(rc, (self.lib.pano_last_error(self.h) or b"").decode())

    def set_flags(self, flags: int):
        """pano_ctx_set_flags: scheduling options of this context (PANO_CTX_*)."""
        self.check(self.lib.pano_ctx_set_flags(self.h, int(flags)))

    def bind_stream(self):
        stream = self._torch.cuda.current_stream(self.device).cuda_stream
        self.check(self.lib.pano_ctx_set_stream(self.h, _P(stream)))

    def sync(self):
        self.check(self.lib.pano_sync(self.h))

    def release_scratch(self):
        """Free the scratch this context grew (pano_ctx_release_scratch); graphs captured
        before are stale afterwards (the generation changes)."""
        self.check(self.lib.pano_ctx_release_scratch(self.h))

    def generation(self) -> int:
        """Scratch generation (include/pano.h): changes when the context re-allocates scratch,
        which invalidates every hipGraph captured before."""
        return int(self.lib.pano_ctx_generation(self.h))

    def prof_enable(self, kernel):
        k = kernel if isinstance(kernel, int) else (K_ALL if kernel == "all" else KERNELS.index(kernel))
        self.check(self.lib.pano_prof_enable(self.h, k))

    # ---- hipGraph capture / replay of launch sequences (include/pano.h)
    def graph_begin(self):
        self.check(self.lib.pano_graph_begin(self.h))

    def graph_end(self):
        g = _P()
        self.check(self.lib.pano_graph_end(self.h, ctypes.byref(g)))
        return g

    def graph_launch(self, g):
        self.check(self.lib.pano_graph_launch(self.h, g))

    def graph_prof(self, g, kernel):
        k = kernel if isinstance(kernel, int) else (K_ALL if kernel == "all" else KERNELS.index(kernel))
        n, tot = ctypes.c_int(), ctypes.c_double()
        rc = self.lib.pano_graph_prof(g, k, ctypes.byref(n), ctypes.byref(tot))
        if rc:
            hip = (PANO_E_HIP - rc) // 100 if rc < PANO_E_HIP else None
            raise PanoError(rc, f"pano_graph_prof: hipEventElapsedTime failed (hipError {hip})")
        return {"launches": n.value, "total_ms": tot.value}

    def graph_destroy(self, g):
        self.lib.pano_graph_destroy(g)

    def prof_read(self, kernel):
        k = kernel if isinstance(kernel, int) else (K_ALL if kernel == "all" else KERNELS.index(kernel))
        n = ctypes.c_int()
        tot, mn, mx = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        self.check(self.lib.pano_prof_read(self.h, k, ctypes.byref(n), ctypes.byref(tot),
                                           ctypes.byref(mn), ctypes.byref(mx)))
        return {"launches": n.value, "total_ms": tot.value, "min_ms": mn.value, "max_ms": mx.value}

    def close(self):
        if getattr(self, "h", None):
            self.lib.pano_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_ctxs: dict = {}


def context(device: int | None = None) -> Context:
    import torch
    if device is None:
        device = torch.cuda.current_device()
    ctx = _ctxs.get(device)
    if ctx is None:
        ctx = Context(device)
        _ctxs[device] = ctx
    ctx.bind_stream()
    return ctx


def ptr(t) -> _P:
    """Device pointer of a torch tensor (must be contiguous and on a HIP device)."""
    if not t.is_cuda:
        raise PanoError(PANO_E_ARG, "expected a device tensor")
    if not t.is_contiguous():
        raise PanoError(PANO_E_ARG, "expected a contiguous tensor")
    return _P(t.data_ptr())


def f64p(a: np.ndarray):
    """Pointer into a caller-owned float64 C-contiguous array (no temporaries)."""
    if a.dtype != np.float64 or not a.flags.c_contiguous:
        raise PanoError(PANO_E_ARG, "expected a C-contiguous float64 array")
    return a.ctypes.data_as(_PD)


def i32p(a: np.ndarray):
    """Pointer into a caller-owned int32 C-contiguous array (no temporaries)."""
    if a.dtype != np.int32 or not a.flags.c_contiguous:
        raise PanoError(PANO_E_ARG, "expected a C-contiguous int32 array")
    return a.ctypes.data_as(_PI32)
