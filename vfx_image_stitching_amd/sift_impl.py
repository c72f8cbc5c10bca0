"""Drop-in replacement for /root/reference/sift_impl.py backed by libpano (gfx950).

``compute_keypoints_and_descriptors`` keeps the reference signature and return types
(list of KeyPoint, float32 [N, 128]) -- sift_impl.py:15-39 -- but runs the whole chain
(S1..S9 of SURVEY.md section 8a) as HIP kernels.  The scalar helpers are restated on the
host (they are shape/parameter arithmetic); the pyramid stage functions the GUI calls
(sift_visualizeUI.py:104-115) read the levels back from the device pyramid built for the
same image.
"""
from __future__ import annotations

from functools import cmp_to_key

import numpy as np

from . import _lib
from .keypoint import KeyPoint, from_records

float_tolerance = 1e-7

_stitchers: dict = {}
_last_pyramid: dict = {}


def _stitcher(sigma, num_intervals, assumed_blur, border):
    """One Stitcher per parameter set; its keypoint capacity grows on demand (features_fit)."""
    from .pipeline import Stitcher
    key = (sigma, num_intervals, assumed_blur, border)
    st = _stitchers.get(key)
    if st is None:
        st = Stitcher("sift", cap=4096, sift_params=dict(
            sigma=sigma, num_intervals=num_intervals, assumed_blur=assumed_blur, border=border))
        _stitchers[key] = st
    return st


def _as_bgr_u8(image) -> np.ndarray:
    img = np.asarray(image)
    if img.dtype != np.uint8:
        r = np.rint(img)
        if not (np.array_equal(r, img) and img.min() >= 0 and img.max() <= 255):
            raise NotImplementedError("libpano SIFT takes 8-bit images (the reference's inputs)")
        img = r.astype(np.uint8)
    if img.ndim == 2:
        # (1868 g + 9617 g + 4899 g + 8192) >> 14 == g: gray survives the BGR2GRAY step
        img = np.repeat(img[..., None], 3, axis=2)
    if img.ndim != 3 or img.shape[2] != 3:
        raise ValueError("expected an H x W x 3 BGR or H x W gray image")
    return np.ascontiguousarray(img)


def compute_keypoints_and_descriptors(image, sigma=1.6, num_intervals=3, assumed_blur=0.5,
                                      image_border_width=5):
    bgr = _as_bgr_u8(image)
    st = _stitcher(sigma, num_intervals, assumed_blur, image_border_width)
    kps, desc, counts = st.features_fit(st.upload(bgr[None]))
    n = int(counts.cpu()[0])
    st.ctx.sync()
    rec = kps[0, :n].cpu().numpy().view(_lib.KP_NP).reshape(-1)
    d = desc[0, :n].cpu().numpy().astype(np.float32)
    _last_pyramid["key"] = (bgr.shape, sigma, num_intervals, assumed_blur)
    _last_pyramid["stitcher"] = st
    return from_records(rec), d


# ------------------------------------------------------------------ scalar stage helpers
def compute_number_of_octaves(image_shape):
    return int(np.round(np.log(min(image_shape)) / np.log(2) - 1))


def generate_gaussian_kernels(sigma, num_intervals):
    n = num_intervals + 3
    k = 2 ** (1. / num_intervals)
    out = np.zeros(n)
    out[0] = sigma
    for i in range(1, n):
        prev = (k ** (i - 1)) * sigma
        out[i] = np.sqrt((k * prev) ** 2 - prev ** 2)
    return out


def compare_keypoints(kp1, kp2):
    """Sort order of sift_impl.py:299-311 (x, y ascending; size descending; ...)."""
    for a, b in ((kp1.pt[0], kp2.pt[0]), (kp1.pt[1], kp2.pt[1])):
        if a != b:
            return a - b
    if kp1.size != kp2.size:
        return kp2.size - kp1.size
    if kp1.angle != kp2.angle:
        return kp1.angle - kp2.angle
    if kp1.response != kp2.response:
        return kp2.response - kp1.response
    return kp2.class_id - kp1.class_id


def remove_duplicate_keypoints(keypoints):
    if len(keypoints) < 2:
        return keypoints
    keypoints.sort(key=cmp_to_key(compare_keypoints))
    out = [keypoints[0]]
    for kp in keypoints[1:]:
        last = out[-1]
        if last.pt != kp.pt or last.size != kp.size or last.angle != kp.angle:
            out.append(kp)
    return out


def convert_keypoints_to_input_image_size(keypoints):
    for kp in keypoints:
        kp.pt = (kp.pt[0] * 0.5, kp.pt[1] * 0.5)
        kp.size *= 0.5
        kp.octave = (kp.octave & ~255) | ((kp.octave - 1) & 255)
    return list(keypoints)


def unpack_octave(keypoint):
    octave = keypoint.octave & 255
    layer = (keypoint.octave >> 8) & 255
    if octave >= 128:
        octave |= -128
    scale = 1 / np.float32(1 << octave) if octave >= 0 else np.float32(1 << -octave)
    return octave, layer, scale


# ------------------------------------------------------------------ pyramid stages (GUI)
class _DevicePyramid:
    """Pyramid levels of one image built by libpano, read back on demand."""

    def __init__(self, image_u8, sigma, num_intervals, assumed_blur):
        import ctypes
        self.st = _stitcher(sigma, num_intervals, assumed_blur, 5)
        self.bgr = _as_bgr_u8(image_u8)
        dev = self.st.upload(self.bgr[None])
        ctx = self.st.ctx
        ctx.check(ctx.lib.pano_sift_pyramid(ctx.h, _lib.ptr(dev), 1, self.bgr.shape[0],
                                            self.bgr.shape[1], ctypes.byref(self.st.params)))
        self._dev = dev
        self.levels = num_intervals + 3

    def level(self, octave, level, dog=False):
        import ctypes
        ctx = self.st.ctx
        h, w, no = (ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32())
        ctx.check(ctx.lib.pano_sift_level_shape(ctx.h, octave, ctypes.byref(h), ctypes.byref(w),
                                                ctypes.byref(no)))
        out = self.st.torch.empty((h.value, w.value), dtype=self.st.torch.float32,
                                  device=self.st.device)
        ctx.check(ctx.lib.pano_sift_copy_level(ctx.h, 0, octave, level, int(dog), _lib.ptr(out)))
        return out.cpu().numpy()

    def n_octaves(self):
        import ctypes
        ctx = self.st.ctx
        h, w, no = (ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32())
        ctx.check(ctx.lib.pano_sift_level_shape(ctx.h, 0, ctypes.byref(h), ctypes.byref(w),
                                                ctypes.byref(no)))
        return no.value


class _BaseImage(np.ndarray):
    """ndarray carrying the device pyramid it was read from (for the next stage call)."""
    pyramid = None


def generate_base_image(image, sigma, assumed_blur):
    if sigma is None:
        sigma = 1.6
    pyr = _DevicePyramid(image, sigma, 3, assumed_blur)
    base = pyr.level(0, 0).view(_BaseImage)
    base.pyramid = pyr
    return base


def generate_gaussian_images(image, num_octaves, gaussian_kernels):
    pyr = getattr(image, "pyramid", None)
    if pyr is None:
        raise NotImplementedError("generate_gaussian_images needs the base from generate_base_image")
    no = min(num_octaves, pyr.n_octaves())
    out = np.empty((no, pyr.levels), dtype=object)
    for o in range(no):
        for l in range(pyr.levels):
            out[o, l] = pyr.level(o, l)
    _last_pyramid["gauss"] = (out, pyr)
    return out


def generate_DoG_images(gaussian_images):
    ent = _last_pyramid.get("gauss")
    if ent is None or ent[0] is not gaussian_images:
        return np.array([[b - a for a, b in zip(o, o[1:])] for o in gaussian_images], dtype=object)
    _, pyr = ent
    no = gaussian_images.shape[0]
    out = np.empty((no, pyr.levels - 1), dtype=object)
    for o in range(no):
        for l in range(pyr.levels - 1):
            out[o, l] = pyr.level(o, l, dog=True)
    return out


__all__ = ["KeyPoint", "compute_keypoints_and_descriptors", "compute_number_of_octaves",
           "generate_gaussian_kernels", "compare_keypoints", "remove_duplicate_keypoints",
           "convert_keypoints_to_input_image_size", "unpack_octave", "generate_base_image",
           "generate_gaussian_images", "generate_DoG_images"]
