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


def _as_bgr_u8(image):
    """The frame as u8 BGR for the batched chain, or None when the reference's arithmetic
    differs from that chain's: a float32 BGR image goes through cv2.cvtColor's float formula
    (not the u8 fixed-point one), a non-integer gray image through float levels.  BGR images
    of other depths are refused as cv2.cvtColor would treat them: float64 (and every other
    depth cv2 has no BGR2GRAY for) raises ValueError like cv2's "Unsupported depth" error;
    uint16, which cv2 converts with its 16-bit fixed-point path, raises NotImplementedError
    (no fixture pins that path)."""
    img = np.asarray(image)
    if img.ndim == 3 and img.shape[2] == 3:
        if img.dtype == np.uint8:
            return np.ascontiguousarray(img)
        if img.dtype == np.float32:
            return None
        if img.dtype == np.uint16:
            raise NotImplementedError("16-bit BGR input: cv2's 16-bit BGR2GRAY path is not restated")
        raise ValueError(f"cvtColor(BGR2GRAY): unsupported depth {img.dtype} (cv2 takes uint8, "
                         "uint16 and float32)")
    if img.ndim != 2:
        raise ValueError("expected an H x W x 3 BGR or H x W gray image")
    if img.dtype != np.uint8:
        r = np.rint(img)
        if not (np.array_equal(r, img) and img.min() >= 0 and img.max() <= 255):
            return None
        img = r.astype(np.uint8)
    # (1868 g + 9617 g + 4899 g + 8192) >> 14 == g: gray survives the BGR2GRAY step
    return np.ascontiguousarray(np.repeat(img[..., None], 3, axis=2))


def _frame_u8(image):
    """_as_bgr_u8 for the batched pair paths (compute_shift_sift, match_homography), whose
    reference inputs are cv2.imread frames: other images are refused."""
    bgr = _as_bgr_u8(image)
    if bgr is None:
        raise NotImplementedError("the pair paths take 8-bit frames (cv2.imread's); "
                                  "compute_keypoints_and_descriptors takes float images")
    return bgr


def _gray_f32(image):
    """sift_impl.py:27-29 for the images the batched chain does not take: cv2.cvtColor
    BGR2GRAY of a float32 BGR image (B * 0.114 + G * 0.587 + R * 0.299 in float32, OpenCV's
    scalar order; its SIMD body may fuse -- parity unpinned for float BGR input, no cv2 here),
    computed on the device by pano_gray_bgr_f32, then astype(float32)."""
    img = np.asarray(image)
    if img.ndim == 2:
        return np.ascontiguousarray(img, np.float32)
    ctx, torch, dev = _dev()
    h, w = img.shape[:2]
    t = torch.from_numpy(np.ascontiguousarray(img, np.float32)).to(dev)
    g = torch.empty((h, w), dtype=torch.float32, device=dev)
    ctx.check(ctx.lib.pano_gray_bgr_f32(ctx.h, _lib.ptr(t), 1, h, w, _lib.ptr(g)))
    ctx.sync()
    return g.cpu().numpy()


def compute_keypoints_and_descriptors(image, sigma=1.6, num_intervals=3, assumed_blur=0.5,
                                      image_border_width=5):
    bgr = _as_bgr_u8(image)
    if bgr is None:
        # the reference's own sequence (sift_impl.py:27-38) through the stage functions below,
        # every stage a libpano launch: float images whose gray is not an 8-bit one
        gray = _gray_f32(image)
        base = generate_base_image(gray, sigma, assumed_blur)
        gauss = generate_gaussian_images(base, compute_number_of_octaves(base.shape),
                                         generate_gaussian_kernels(sigma, num_intervals))
        dogs = generate_DoG_images(gauss)
        kps = find_scale_space_extrema(gauss, dogs, num_intervals, sigma, image_border_width)
        kps = convert_keypoints_to_input_image_size(remove_duplicate_keypoints(kps))
        return kps, generate_descriptors(kps, gauss)
    st = _stitcher(sigma, num_intervals, assumed_blur, image_border_width)
    kps, desc, counts = st.features_fit(st.upload(bgr[None]))
    n = int(counts.cpu()[0])
    st.ctx.sync()
    rec = kps[0, :n].cpu().numpy().view(_lib.KP_NP).reshape(-1)
    d = desc[0, :n].cpu().numpy().astype(np.float32)
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


# ------------------------------------------------------------------ stage functions (GUI)
# sift_visualizeUI.py:104-115 calls the stages one by one with numpy arrays in between.  Each
# stage here is a pure function of its arguments computed by libpano: its inputs go to the
# device, the stage's kernels run there (the same kernels as compute_keypoints_and_descriptors),
# and the outputs come back as the reference's types.  Pyramids are ``np.ndarray`` of dtype
# object, shape (octaves, levels), like the reference's np.array(pyramid, dtype=object).
def _dev():
    import torch
    ctx = _lib.context()
    return ctx, torch, torch.device("cuda", ctx.device)


def _f32_2d(a, what):
    a = np.asarray(a)
    if a.ndim != 2:
        raise ValueError(f"{what}: expected a single-channel 2-D image, got shape {a.shape}")
    return np.ascontiguousarray(a, np.float32)


def _params(sigma=1.6, num_intervals=3, assumed_blur=0.5, border=5, contrast_threshold=0.04):
    return _lib.default_sift_params(sigma=float(sigma), num_intervals=int(num_intervals),
                                    assumed_blur=float(assumed_blur), border=int(border),
                                    contrast_threshold=float(contrast_threshold))


def _pyramid_shapes(pyr, what):
    """(octaves, levels) and the octave-0 shape of an object pyramid; every octave must halve
    the previous one (floor), as generate_gaussian_images builds them."""
    pyr = np.asarray(pyr, dtype=object)
    if pyr.ndim != 2:
        raise ValueError(f"{what}: expected an (octaves, levels) object array")
    no, nl = pyr.shape
    h, w = np.asarray(pyr[0, 0]).shape
    for o in range(no):
        for l in range(nl):
            if np.asarray(pyr[o, l]).shape != (h, w):
                raise ValueError(f"{what}: level ({o}, {l}) has shape {np.asarray(pyr[o, l]).shape}, "
                                 f"expected {(h, w)}")
        h, w = h // 2, w // 2
    return pyr, no, nl


def _upload_pyramid(gauss, dogs=None):
    """Reserve a resident pyramid shaped like `gauss` and copy its levels (and `dogs`) in."""
    ctx, torch, dev = _dev()
    g, no, nl = _pyramid_shapes(gauss, "gaussian_images")
    H0, W0 = np.asarray(g[0, 0]).shape
    ctx.check(ctx.lib.pano_sift_reserve_levels(ctx.h, 1, H0, W0, no, nl))
    keep = []
    for o in range(no):
        for l in range(nl):
            t = torch.from_numpy(_f32_2d(g[o, l], "gaussian_images")).to(dev)
            keep.append(t)
            ctx.check(ctx.lib.pano_sift_set_level(ctx.h, 0, o, l, 0, _lib.ptr(t)))
    if dogs is not None:
        d = np.asarray(dogs, dtype=object)
        if d.ndim != 2 or d.shape != (no, nl - 1):
            raise ValueError(f"dog_images: expected shape {(no, nl - 1)}, got {d.shape}")
        for o in range(no):
            for l in range(nl - 1):
                a = _f32_2d(d[o, l], "dog_images")
                if a.shape != np.asarray(g[o, 0]).shape:
                    raise ValueError(f"dog_images: level ({o}, {l}) shape {a.shape}")
                t = torch.from_numpy(a).to(dev)
                keep.append(t)
                ctx.check(ctx.lib.pano_sift_set_level(ctx.h, 0, o, l, 1, _lib.ptr(t)))
    torch.cuda.current_stream(dev).synchronize()      # the host tensors may go now
    return ctx, no, nl


def _read_levels(ctx, no, nl, dog):
    import ctypes
    _, torch, dev = _dev()
    out = np.empty((no, nl), dtype=object)
    for o in range(no):
        h, w = ctypes.c_int32(), ctypes.c_int32()
        ctx.check(ctx.lib.pano_sift_level_shape(ctx.h, o, ctypes.byref(h), ctypes.byref(w), None))
        for l in range(nl):
            t = torch.empty((h.value, w.value), dtype=torch.float32, device=dev)
            ctx.check(ctx.lib.pano_sift_copy_level(ctx.h, 0, o, l, int(dog), _lib.ptr(t)))
            out[o, l] = t.cpu().numpy()
    return out


def generate_base_image(image, sigma, assumed_blur):
    """sift_impl.py:45-56: x2 INTER_LINEAR + GaussianBlur(sigma_diff) of a gray f32 image
    (pano_sift_base).  Exact for integer-valued gray levels (every reference caller's case)."""
    import ctypes
    if sigma is None:
        sigma = 1.6
    g = _f32_2d(image, "generate_base_image")
    ctx, torch, dev = _dev()
    src = torch.from_numpy(g).to(dev)
    h, w = g.shape
    out = torch.empty((2 * h, 2 * w), dtype=torch.float32, device=dev)
    p = _params(sigma=sigma, assumed_blur=assumed_blur)
    ctx.check(ctx.lib.pano_sift_base(ctx.h, _lib.ptr(src), 1, h, w, ctypes.byref(p), _lib.ptr(out)))
    return out.cpu().numpy()


def generate_gaussian_images(image, num_octaves, gaussian_kernels):
    """sift_impl.py:82-97 on any f32 base image and any kernel list (pano_sift_pyramid_kernels):
    per octave level l = GaussianBlur(level l - 1, gaussian_kernels[l]), next base =
    INTER_NEAREST 1/2 of level -3."""
    import ctypes
    k = np.ascontiguousarray(np.asarray(gaussian_kernels, np.float64).ravel())
    if len(k) < 3:
        # the reference indexes level -3 for the next octave's base
        raise IndexError("generate_gaussian_images needs at least 3 kernels")
    base = _f32_2d(image, "generate_gaussian_images")
    ctx, torch, dev = _dev()
    src = torch.from_numpy(base).to(dev)
    H0, W0 = base.shape
    rc = ctx.lib.pano_sift_pyramid_kernels(ctx.h, _lib.ptr(src), 1, H0, W0, int(num_octaves),
                                           k.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), len(k))
    try:
        ctx.check(rc)
    except _lib.PanoError as e:
        if e.code == _lib.PANO_E_UNSUPPORTED:     # a kernel wider than PANO_MAX_TAPS, > max levels
            raise NotImplementedError(str(e)) from e
        raise
    no = ctypes.c_int32()
    ctx.check(ctx.lib.pano_sift_level_shape(ctx.h, 0, None, None, ctypes.byref(no)))
    return _read_levels(ctx, no.value, len(k), dog=False)


def generate_DoG_images(gaussian_images):
    """sift_impl.py:100-111: G[l+1] - G[l] per octave (pano_sift_dog on the uploaded levels)."""
    ctx, no, nl = _upload_pyramid(gaussian_images)
    ctx.check(ctx.lib.pano_sift_dog(ctx.h))
    return _read_levels(ctx, no, nl - 1, dog=True)


def _raw_keypoints(ctx, p, cap=8192):
    import ctypes
    _, torch, dev = _dev()
    while True:
        raw = torch.empty((1, cap, 6), dtype=torch.int32, device=dev)
        counts = torch.zeros((1,), dtype=torch.int32, device=dev)
        ctx.check(ctx.lib.pano_sift_extrema(ctx.h, ctypes.byref(p), _lib.ptr(raw), cap, _lib.ptr(counts)))
        ctx.sync()
        n = int(counts.cpu()[0])
        if n < 0:
            raise _lib.PanoError(_lib.PANO_E_OVERFLOW, "pano_sift_extrema: scratch capacity exceeded")
        if n <= cap:
            return raw[0, :n].cpu().numpy().view(_lib.KP_NP).reshape(-1)
        cap = 1 << int(n - 1).bit_length()


def find_scale_space_extrema(gaussian_images, dog_images, num_intervals, sigma, border,
                             contrast_threshold=0.04):
    """sift_impl.py:117-140: extrema -> quadratic-fit localisation -> orientations, every
    candidate of every octave (pano_sift_extrema).  Returns the oriented keypoints before
    remove_duplicate_keypoints, in the reference's scan order, base-image coordinates."""
    ctx, no, nl = _upload_pyramid(gaussian_images, dog_images)
    if nl != int(num_intervals) + 3:
        raise ValueError(f"{nl} levels per octave do not fit num_intervals={num_intervals}")
    p = _params(sigma=sigma, num_intervals=num_intervals, border=border,
                contrast_threshold=contrast_threshold)
    return from_records(_raw_keypoints(ctx, p))


def generate_descriptors(keypoints, gaussian_images, window_width=4, num_bins=8, scale_multiplier=3,
                         descriptor_max_value=0.2):
    """sift_impl.py:361-526 for the given keypoints (input-image coordinates, converted octave
    field) on the given pyramid (pano_sift_describe).  float32 [N, 128]."""
    import ctypes
    if window_width != 4 or num_bins != 8:
        raise NotImplementedError("libpano's descriptor is the reference's 4 x 4 x 8 layout")
    kps = list(keypoints)
    if not kps:
        return np.array([], dtype="float32")
    g, no, nl = _pyramid_shapes(gaussian_images, "gaussian_images")
    rec = np.zeros(len(kps), _lib.KP_NP)
    for i, kp in enumerate(kps):
        octv, lyr, _ = unpack_octave(kp)
        if not (0 <= octv + 1 < no and 0 <= lyr < nl):
            raise IndexError(f"keypoint {i}: octave {octv}, layer {lyr} outside the pyramid "
                             f"({no} octaves, {nl} levels)")
        vals = (kp.pt[0], kp.pt[1], kp.size, kp.angle, kp.response)
        if not np.all(np.isfinite(vals)):
            raise ValueError(f"keypoint {i}: non-finite fields {vals}")
        rec[i] = (*vals, kp.octave)
    ctx, _, _ = _upload_pyramid(g)
    _, torch, dev = _dev()
    n = len(kps)
    k_dev = torch.from_numpy(rec.view(np.int32).reshape(1, n, 6).copy()).to(dev)
    counts = torch.tensor([n], dtype=torch.int32, device=dev)
    desc = torch.empty((1, n, 128), dtype=torch.float32, device=dev)
    p = _lib.default_sift_params(scale_multiplier=float(scale_multiplier),
                                 descriptor_max=float(descriptor_max_value))
    ctx.check(ctx.lib.pano_sift_describe(ctx.h, ctypes.byref(p), _lib.ptr(k_dev), _lib.ptr(counts), n,
                                         _lib.ptr(desc)))
    return desc[0].cpu().numpy()


# ------------------------------------------------------------------ per-candidate helpers
# find_scale_space_extrema's building blocks (sift_impl.py:143-293).  The two that do real work
# -- the quadratic-fit localisation and the orientation histogram -- run on the GPU through
# pano_sift_localize / pano_sift_orient, i.e. the batched kernels' own device code
# (localize_one, orient_one in sift_features.hip); they also take whole candidate lists
# (localize_extrema, orient_keypoints), which is how a caller should use them.  The 3 x 3 x 3
# predicates are written in the separable / stencil form the extrema kernel evaluates.
_AXES_XYS = (2, 1, 0)          # cube axes of the reference's derivative order (x, y, scale)


def _nb(cube, **shift):
    """The cube value at the centre (1, 1, 1) moved by shift {axis: +-1}."""
    at = [1, 1, 1]
    for ax, d in shift.items():
        at[int(ax[1:])] += d
    return cube[tuple(at)]


def is_pixel_an_extremum(prev_patch, curr_patch, next_patch, threshold):
    """sift_impl.py:143-163.  The centre belongs to its own 3 x 3 x 3 cube, so "v >= every one
    of the 26 neighbours" is v == max(cube) (and "<=" is v == min(cube)): the form
    extrema_stream / extrema_scan evaluate.  NaN anywhere fails both, as in the reference."""
    cube = np.stack((np.asarray(prev_patch), np.asarray(curr_patch), np.asarray(next_patch)))
    v = cube[1, 1, 1]
    if not abs(v) > threshold:
        return False
    return bool(v == (cube.max() if v > 0 else cube.min()))


def compute_gradient_at_center_pixel(cube):
    """sift_impl.py:217-224: half the difference of the centre's +1 / -1 neighbours along x, y
    and scale."""
    c = np.asarray(cube)
    return np.array([0.5 * (_nb(c, **{f"a{ax}": 1}) - _nb(c, **{f"a{ax}": -1})) for ax in _AXES_XYS])


def compute_hessian_at_center_pixel(cube):
    """sift_impl.py:227-240: the (x, y, scale) Hessian of the cube.  Diagonal: (v+ - 2v) + v-;
    mixed terms: ((v++ - v+-) - v-+) + v--, over (slower axis, faster axis), times 1/4."""
    c = np.asarray(cube)
    v = c[1, 1, 1]

    def d2(i, j):
        a, b = _AXES_XYS[i], _AXES_XYS[j]
        if a == b:
            return (_nb(c, **{f"a{a}": 1}) - 2 * v) + _nb(c, **{f"a{a}": -1})
        s, f = f"a{min(a, b)}", f"a{max(a, b)}"
        return 0.25 * (((_nb(c, **{s: 1, f: 1}) - _nb(c, **{s: 1, f: -1})) - _nb(c, **{s: -1, f: 1}))
                       + _nb(c, **{s: -1, f: -1}))

    return np.array([[d2(i, j) for j in range(3)] for i in range(3)])


def _dog_planes(dog_octave, num_intervals):
    """The octave's DoG levels as device tensors (ni + 2 planes of one shape)."""
    _, torch, dev = _dev()
    levels = [_f32_2d(d, "dog_octave") for d in dog_octave]
    if len(levels) != int(num_intervals) + 2:
        raise ValueError(f"dog_octave: {len(levels)} levels for num_intervals={num_intervals} "
                         f"(expected {int(num_intervals) + 2})")
    shape = levels[0].shape
    if any(l.shape != shape for l in levels):
        raise ValueError("dog_octave: levels of different shapes")
    return [torch.from_numpy(l).to(dev) for l in levels], shape


def localize_extrema(candidates, octave, num_intervals, dog_octave, sigma, contrast_threshold, border,
                     eigen_ratio=10, max_iter=5):
    """localize_extremum_via_quadratic_fit for every (x, y, layer) of ``candidates`` (one
    octave) in one launch (pano_sift_localize): a list with, per candidate, (KeyPoint, layer)
    or None."""
    import ctypes
    cand = np.ascontiguousarray(np.asarray(candidates, dtype=np.int64).reshape(-1, 3))
    n = len(cand)
    if n == 0:
        return []
    if cand.min() < -(1 << 31) or cand.max() >= (1 << 31):
        raise IndexError("candidate coordinates out of range")
    ctx, torch, dev = _dev()
    planes, (h, w) = _dog_planes(dog_octave, num_intervals)
    ptrs = (ctypes.c_void_p * len(planes))(*[t.data_ptr() for t in planes])
    c_dev = torch.from_numpy(cand.astype(np.int32)).to(dev)
    out = torch.empty((n, 6), dtype=torch.int32, device=dev)
    layer = torch.empty((n,), dtype=torch.int32, device=dev)
    p = _lib.default_sift_params(sigma=float(sigma), num_intervals=int(num_intervals), border=int(border),
                                 contrast_threshold=float(contrast_threshold),
                                 eigen_ratio=float(eigen_ratio), max_iter=int(max_iter))
    ctx.check(ctx.lib.pano_sift_localize(ctx.h, ctypes.byref(p), ptrs, len(planes), h, w, int(octave),
                                         _lib.ptr(c_dev), n, _lib.ptr(out), _lib.ptr(layer)))
    rec = out.cpu().numpy().view(_lib.KP_NP).reshape(-1)
    lay = layer.cpu().numpy()
    if (lay == -2).any():
        i = int(np.argmax(lay == -2))
        raise IndexError(f"candidate {i} {tuple(cand[i])}: its 3x3x3 cube leaves the DoG levels")
    return [None if l < 0 else (KeyPoint(float(r["x"]), float(r["y"]), float(r["size"]), -1.0,
                                         float(r["response"]), int(r["octave"])), int(l))
            for r, l in zip(rec, lay)]


def localize_extremum_via_quadratic_fit(x, y, layer, octave, num_intervals, dog_octave, sigma,
                                        contrast_threshold, border, eigen_ratio=10, max_iter=5):
    """sift_impl.py:169-211 for one extremum on the GPU (pano_sift_localize): at most max_iter
    Newton steps on the 3x3x3 cube / 255, the contrast and edge tests; (KeyPoint, layer) or
    None, the reference's max_iter quirk included."""
    return localize_extrema([(x, y, layer)], octave, num_intervals, dog_octave, sigma, contrast_threshold,
                            border, eigen_ratio, max_iter)[0]


def orient_keypoints(keypoints, octave, gauss_img, radius_factor=3, num_bins=36, peak_ratio=0.8,
                     scale_factor=1.5):
    """compute_keypoints_with_orientations for every keypoint of one octave in one launch
    (pano_sift_orient): a list of lists of oriented KeyPoints, peak order."""
    import ctypes
    if num_bins != 36:
        raise NotImplementedError("libpano's orientation histogram has the reference's 36 bins")
    kps = list(keypoints)
    if not kps:
        return []
    img = _f32_2d(gauss_img, "gauss_img")
    ctx, torch, dev = _dev()
    rec = np.zeros(len(kps), _lib.KP_NP)
    for i, kp in enumerate(kps):
        rec[i] = (kp.pt[0], kp.pt[1], kp.size, kp.angle, kp.response, kp.octave)
    n = len(kps)
    g = torch.from_numpy(img).to(dev)
    k_dev = torch.from_numpy(rec.view(np.int32).reshape(n, 6).copy()).to(dev)
    out = torch.empty((n, _lib.ORI_MAX_PEAKS, 6), dtype=torch.int32, device=dev)
    counts = torch.empty((n,), dtype=torch.int32, device=dev)
    p = _lib.default_sift_params(radius_factor=float(radius_factor), peak_ratio=float(peak_ratio),
                                 scale_factor=float(scale_factor))
    ctx.check(ctx.lib.pano_sift_orient(ctx.h, ctypes.byref(p), _lib.ptr(g), img.shape[0], img.shape[1],
                                       int(octave), _lib.ptr(k_dev), n, _lib.ptr(out), _lib.ptr(counts)))
    o = out.cpu().numpy().view(_lib.KP_NP).reshape(n, _lib.ORI_MAX_PEAKS)
    c = counts.cpu().numpy()
    if (c < 0).any():
        i = int(np.argmax(c < 0))
        raise ValueError(f"keypoint {i}: non-finite position or an orientation window above 1024 px")
    return [[KeyPoint(*kps[i].pt, kps[i].size, float(r["angle"]), kps[i].response, kps[i].octave)
             for r in o[i, :c[i]]] for i in range(n)]


def compute_keypoints_with_orientations(keypoint, octave, gauss_img, radius_factor=3, num_bins=36,
                                        peak_ratio=0.8, scale_factor=1.5):
    """sift_impl.py:246-293 for one keypoint on the GPU (pano_sift_orient): one KeyPoint per
    orientation-histogram peak >= peak_ratio * max, parabolically interpolated."""
    return orient_keypoints([keypoint], octave, gauss_img, radius_factor, num_bins, peak_ratio,
                            scale_factor)[0]


__all__ = ["KeyPoint", "compute_keypoints_and_descriptors", "compute_number_of_octaves",
           "generate_gaussian_kernels", "compare_keypoints", "remove_duplicate_keypoints",
           "convert_keypoints_to_input_image_size", "unpack_octave", "generate_base_image",
           "generate_gaussian_images", "generate_DoG_images", "find_scale_space_extrema",
           "is_pixel_an_extremum", "localize_extremum_via_quadratic_fit",
           "compute_gradient_at_center_pixel", "compute_hessian_at_center_pixel",
           "compute_keypoints_with_orientations", "generate_descriptors", "localize_extrema",
           "orient_keypoints"]
