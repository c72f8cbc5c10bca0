"""Batched MI355X stitching pipeline: the numeric body of run_panorama on the GPU.

Reference flow (image_stitching_sift.py:290-384, image_stitching_harris.py:460-542):
cylindrical projection of every frame -> per adjacent pair: features of both frames, NN
match, translation RANSAC -> vertical drift correction -> sequential pad + blend fold ->
rectangle crop.

Here every stage runs as libpano kernels over the whole frame batch, on one HIP stream:

    pano_cylindrical   all frames, one launch (cyl_tile)
    pano_sift_u8 / pano_harris   all frames once (the reference recomputes interior frames for
                       both of their pairs; features are a pure function of the frame)
    pano_match_u8      all pairs (exact i8 MFMA distance GEMM on the descriptor bytes for SIFT;
                       pano_match's bf16 / f32 MFMA forms for f32 descriptors)
    pano_pair_shifts   all pairs (match filter + exhaustive vote RANSAC)
    pano_plan_composite_device   drift correction + composite plan on the GPU, then the
                       planned composite into a capacity-sized canvas, crop box fused
      -- one pinned copy of the records, crop box and plan header (~1.3 KB): the one host
         read per stitch; the host-planned form (pano_plan_composite + pano_composite_bbox,
         two reads) runs when the device plan reports an overflow or a three-frame column --
"""
from __future__ import annotations

import ctypes
import os
import time
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import PanoError, context, ptr


BBOX_SLOTS = 64                         # include/pano.h PANO_BBOX_SLOTS
_BOX_SIGN = np.array([1, -1, 1, -1], np.int32)


class Features(tuple):
    """(keypoints, descriptors, counts) of a batch, plus the descriptors' squared norms when
    they are bytes (pano_sift_u8): what pano_match_u8 reads."""

    def __new__(cls, feats, norms):
        t = super().__new__(cls, feats)
        t.norms = norms
        return t


@dataclass
class StitchResult:
    panorama: "object"                 # torch uint8 [H', W', 3] on device (a view of canvas)
    canvas: "object"                   # full mosaic before the crop, torch uint8 on device
    shifts: list                       # raw per-pair (dx, dy), reference order
    pairs: list                        # per-pair best match ((xA, yA), (xB, yB)) or None
    records: np.ndarray                # PAIR_NP records
    bbox: tuple                        # (y0, y1, x0, x1) crop rows/cols, inclusive
    timings: dict = field(default_factory=dict)
    host: "object" = None              # StitchPool.run_sequence(to_host=True): the panorama in
                                       # pinned host memory (numpy view)


def drift_correct(shifts):
    """run_panorama :336-365 -- spread the accumulated dy evenly over the pairs."""
    total = 0
    for _, dy in shifts:
        total = total + dy
    n = len(shifts) + 1
    avg = total / (n - 1) if n > 1 else 0
    return [(dx, dy - avg) for dx, dy in shifts]


class Stitcher:
    """Reusable device state for stitching sequences of equally sized frames.

    Stitchers share the device's default libpano context (its scratch: pyramid, keypoints,
    descriptors, ...), and every call is ordered on the caller's current stream; two Stitchers
    whose work may overlap on the device (different streams) each need their own context:
    ``Stitcher(..., ctx=_lib.Context(device))``."""

    def __init__(self, method: str = "sift", device: int | None = None, cap: int = 4096,
                 max_points: int = 200, ransac_thr: float = 3.0, desc_thresh: float | None = None,
                 sift_params: dict | None = None, match: str | None = None, ratio: float = 0.0,
                 ctx=None):
        import os
        import torch
        self.torch = torch
        self.method = method
        self.ctx = ctx if ctx is not None else context(device)
        self.device = torch.device("cuda", self.ctx.device)
        self.cap = cap if method == "sift" else max_points
        self.max_points = max_points
        self.ransac_thr = float(ransac_thr)
        self.desc_thresh = float(desc_thresh if desc_thresh is not None
                                 else (25000 if method == "sift" else 1.0))
        self.params = _lib.default_sift_params(**(sift_params or {}))
        # Lowe ratio test (0 = off, as the reference's stitcher; the visualiser uses 0.7 with
        # FLANN, sift_visualizeUI.py:252-257)
        self.ratio = float(ratio)
        # SIFT descriptors + distance GEMM: "u8" (bytes from the descriptor kernel straight into
        # the LDS-staged bf16 GEMM, pano_sift_u8 + pano_match_u8), "bf16" (f32 descriptors
        # packed to bf16 rows) or "f32" (f32 MFMA); all exact for integer descriptors
        self.match = match or os.environ.get("PANO_MATCH", "u8")
        self._buf = {}
        self._graphs = {}                # key -> (pano_graph, outputs of the captured call)
        self._gstream = None             # private stream for capture / replay
        self.last_graphs = []            # graphs replayed by the last run(graph=True)
        self.canvas_cap = None           # (Hcap, Wcap) of the device-planned canvas; None: auto
        self._graph_mode = False
        self._fast = None                # (key, replay state) of run()'s graph fast path
        self._fast_key = None
        self._views = {}                 # key -> (canvas view, panorama view) of _crop_planned
        # output slots of the device-planned stitch (run_sequence keeps two stitches in flight):
        # slot s has its own result / canvas / pinned head buffers, hence its own graph and
        # fast-path state; run() uses slot 0
        self._slot = 0
        self._slot_state = {}            # slot -> (fast, fast_key, head_np) while not current
        self._stage = {}                 # slot -> staging frame buffer (run_sequence, distinct items)
        self._head_np = None

    # ------------------------------------------------------------------ buffers
    def _get(self, name, shape, dtype):
        t = self._buf.get(name)
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype:
            if t is not None and self._graphs:
                # captured graphs hold the old buffer's address: re-capture, never replay them
                self.release_graphs()
            t = self.torch.empty(shape, dtype=dtype, device=self.device)
            self._buf[name] = t
        return t

    def upload(self, frames) -> "object":
        """uint8 [n, h, w, 3] host array (or list of frames) -> device tensor."""
        if isinstance(frames, (list, tuple)):
            frames = np.stack(frames)
        frames = np.ascontiguousarray(frames, np.uint8)
        return self.torch.from_numpy(frames).to(self.device, non_blocking=False)

    # ------------------------------------------------------------------ stages
    def cylindrical(self, frames_dev, focals):
        n, h, w, _ = frames_dev.shape
        out = self._get("cyl", (n, h, w, 3), self.torch.uint8)
        colnz = self._get("colnz", (n, w), self.torch.uint8)
        f = np.ascontiguousarray(focals, np.float64)
        self.ctx.check(self.ctx.lib.pano_cylindrical(self.ctx.h, ptr(frames_dev), ptr(out), n, h, w,
                                                     _lib.f64p(f), ptr(colnz)))
        return out, colnz

    def features(self, frames_dev):
        n, h, w, _ = frames_dev.shape
        T = self.torch
        if self.method == "sift":
            kps = self._get("kps", (n, self.cap, 6), T.int32)
            counts = self._get("counts", (n,), T.int32)
            if self.match == "u8":
                desc = self._get("desc_u8", (n, self.cap, 128), T.uint8)
                norms = self._get("norms", (n, self.cap), T.int32)
                self.ctx.check(self.ctx.lib.pano_sift_u8(self.ctx.h, ptr(frames_dev), n, h, w,
                                                         ctypes.byref(self.params), ptr(kps), ptr(desc),
                                                         ptr(norms), self.cap, ptr(counts)))
                return Features((kps, desc, counts), norms)
            desc = self._get("desc", (n, self.cap, 128), T.float32)
            self.ctx.check(self.ctx.lib.pano_sift(self.ctx.h, ptr(frames_dev), n, h, w,
                                                  ctypes.byref(self.params), ptr(kps), ptr(desc),
                                                  self.cap, ptr(counts)))
            return kps, desc, counts
        xy = self._get("xy", (n, self.max_points, 2), T.int32)
        desc = self._get("desc", (n, self.max_points, 128), T.float32)
        counts = self._get("counts", (n,), T.int32)
        self.ctx.check(self.ctx.lib.pano_harris(self.ctx.h, ptr(frames_dev), n, h, w,
                                                self.max_points, ptr(xy), ptr(desc), ptr(counts)))
        return xy, desc, counts

    def features_fit(self, frames_dev):
        """features() with the SIFT keypoint capacity grown until every frame's keypoints
        fit (the reference has no limit; one host read of the counts per call)."""
        while True:
            feats = self.features(frames_dev)
            if self.method != "sift":
                return feats
            c = feats[2].cpu().numpy()
            if (c < 0).any():
                raise PanoError(_lib.PANO_E_OVERFLOW, "SIFT extrema exceeded the internal capacity")
            if c.max(initial=0) <= self.cap:
                return feats
            self.cap = 1 << int(np.ceil(np.log2(int(c.max()))))

    def features_of(self, images):
        """Features of host frames that may differ in shape (the reference computes each
        frame on its own: image_stitching_sift.py:59-60): equal shapes run as one batch,
        otherwise frame by frame, gathered into one [n][cap] feature set for pair_records."""
        T = self.torch
        imgs = [np.ascontiguousarray(i, np.uint8) for i in images]
        if len({i.shape for i in imgs}) == 1:
            return self.features_fit(self.upload(np.stack(imgs)))
        parts = []
        for img in imgs:
            pts, desc, counts = self.features_fit(self.upload(img[None]))
            parts.append((pts.clone(), desc.clone(), counts.clone()))
        cap = max(p[1].shape[1] for p in parts)
        n = len(parts)
        pts = T.zeros((n, cap) + tuple(parts[0][0].shape[2:]), dtype=parts[0][0].dtype, device=self.device)
        desc = T.zeros((n, cap, 128), dtype=parts[0][1].dtype, device=self.device)
        counts = T.cat([p[2] for p in parts])
        for i, (p, d, _) in enumerate(parts):
            pts[i, :p.shape[1]] = p[0]
            desc[i, :d.shape[1]] = d[0]
        if desc.dtype == T.uint8:
            return Features((pts, desc, counts), self.desc_norms(desc))
        return pts, desc, counts

    def desc_norms(self, desc):
        """Exact squared norms [frames][cap] i32 of byte descriptors [frames][cap][128]
        (pano_desc_norms_u8), for byte rows that did not come out of pano_sift_u8."""
        T = self.torch
        d = desc.contiguous()
        norms = T.empty(d.shape[:-1], dtype=T.int32, device=d.device)
        self.ctx.check(self.ctx.lib.pano_desc_norms_u8(self.ctx.h, ptr(d), d.numel() // 128, ptr(norms)))
        return norms

    def pair_records(self, feats, pairs, out=None):
        T = self.torch
        pts, desc, counts = feats
        P = len(pairs)
        cap = desc.shape[1]
        hp = np.ascontiguousarray(np.array(pairs, np.int32).reshape(-1))
        best = self._get("best", (P, cap), T.int32)
        d1 = self._get("d1", (P, cap), T.float32)
        # the second-best distance is only computed when the Lowe ratio test needs it (the
        # reference's stitcher has none: image_stitching_sift.py:63-79)
        exact = (1 if self.match == "f32" else 2) if self.method == "sift" else 0
        d2 = self._get("d2", (P, cap), T.float32) if (self.ratio > 0 or exact != 2) else None
        d2p = ptr(d2) if d2 is not None else None
        if desc.dtype == T.uint8:
            norms = getattr(feats, "norms", None)
            if norms is None:
                norms = self.desc_norms(desc)
            self.ctx.check(self.ctx.lib.pano_match_u8(self.ctx.h, ptr(desc), ptr(norms), ptr(counts), cap,
                                                      _lib.i32p(hp), P, ptr(best), ptr(d1), d2p))
        else:
            self.ctx.check(self.ctx.lib.pano_match(self.ctx.h, ptr(desc), ptr(counts), cap,
                                                   _lib.i32p(hp), P, exact, ptr(best), ptr(d1), d2p))
        recs = out if out is not None else self._get("recs", (P, 64), T.uint8)
        kps_p = ptr(pts) if self.method == "sift" else None
        xy_p = None if self.method == "sift" else ptr(pts)
        self.ctx.check(self.ctx.lib.pano_pair_shifts(self.ctx.h, kps_p, xy_p, ptr(counts), cap,
                                                     _lib.i32p(hp), P, ptr(best), ptr(d1), d2p,
                                                     self.desc_thresh, self.ratio, self.ransac_thr,
                                                     ptr(recs)))
        return recs, (best, d1, d2)

    def plan(self, n, h, w, shifts_corr, pairs_xy):
        sh = np.ascontiguousarray(np.array(shifts_corr, np.float64).reshape(-1, 2))
        pr = np.ascontiguousarray(np.array(pairs_xy, np.float64).reshape(-1, 4))
        steps = (_lib.Step * max(n - 1, 1))()
        first = np.zeros(2, np.int32)
        hw = np.zeros(2, np.int32)
        rc = self.ctx.lib.pano_plan_composite(_lib.f64p(sh), _lib.f64p(pr), n, h, w, steps,
                                              _lib.i32p(first), _lib.i32p(hw))
        if rc:
            raise PanoError(rc, "pano_plan_composite")
        return steps, first, (int(hw[0]), int(hw[1]))

    def composite(self, cyl, colnz, shifts_corr, pairs_xy, bbox=False, sequential=False,
                  graph=False):
        """The mosaic loop on a pre-sized canvas; optionally the crop bbox in the same pass."""
        n, h, w, _ = cyl.shape
        steps, first, (H, W) = self.plan(n, h, w, shifts_corr, pairs_xy)
        canvas = self._get("canvas", (H, W, 3), self.torch.uint8)
        lib, c = self.ctx.lib, self.ctx.h
        if sequential:
            self.ctx.check(lib.pano_composite_sequential(c, ptr(cyl), ptr(colnz), n, h, w, steps,
                                                         _lib.i32p(first), ptr(canvas), H, W))
            return canvas
        bb = self._get("bbox", (4,), self.torch.int32) if bbox else None

        def seg():
            self.ctx.check(lib.pano_composite_bbox(c, ptr(cyl), ptr(colnz), n, h, w, steps,
                                                   _lib.i32p(first), ptr(canvas), H, W, 0,
                                                   ptr(bb) if bbox else None))

        if graph:
            key = ("composite", cyl.data_ptr(), colnz.data_ptr(), tuple(cyl.shape), bytes(steps),
                   first.tobytes(), H, W, canvas.data_ptr(), bb.data_ptr() if bbox else 0)
            self._replay(key, seg)
        else:
            seg()
        return (canvas, bb) if bbox else canvas

    def bbox(self, img, thr=0):
        H, W, _ = img.shape
        bb = self._get("bbox", (4,), self.torch.int32)
        self.ctx.check(self.ctx.lib.pano_gray_bbox(self.ctx.h, ptr(img), H, W, thr, ptr(bb)))
        return bb

    def _raw_stream(self):
        """The caller's current HIP stream handle (torch's raw-stream accessor: the public
        ``current_stream(device)`` builds a Stream object, a few microseconds per call)."""
        get = getattr(self.torch._C, "_cuda_getCurrentRawStream", None)
        if get is not None:
            return get(self.device.index)
        return self.torch.cuda.current_stream(self.device).cuda_stream

    # ------------------------------------------------------------------ hipGraph replay
    def _replay(self, key, fn):
        """fn() through a cached hipGraph: one eager call sizes every scratch buffer, the
        second is captured; later calls with the same key replay it (same device pointers
        and kernel arguments -- the key must pin everything fn's launches depend on)."""
        T = self.torch
        # capture needs a non-default stream: graphs are captured and replayed on a private
        # stream ordered after the caller's stream on entry, and the caller's after it on exit
        if self._gstream is None:
            self._gstream = T.cuda.Stream(self.device)
        outer = T.cuda.current_stream(self.device)
        self._gstream.wait_stream(outer)
        try:
            with T.cuda.stream(self._gstream):
                self.ctx.bind_stream()
                dbg = os.environ.get("PANO_DEBUG_SYNC") == "1"
                ent = self._graph_entry(key)
                if ent is None:
                    fn()
                    if dbg:
                        T.cuda.synchronize()
                        print(f"[pano graph] eager ok {key[0]}", flush=True)
                    self.ctx.graph_begin()
                    try:
                        out = fn()
                    except BaseException:
                        try:
                            self.ctx.graph_destroy(self.ctx.graph_end())
                        except PanoError:
                            pass
                        raise
                    g = self.ctx.graph_end()
                    if len(self._graphs) >= 16:
                        self._drop_graph(next(iter(self._graphs)))
                    # the scratch generation the graph's pointers belong to (pano_ctx_generation)
                    ent = self._graphs[key] = (g, out, self.ctx.generation())
                self.ctx.graph_launch(ent[0])
                self.last_graphs.append(ent[0])
                if dbg:
                    T.cuda.synchronize()
                    print(f"[pano graph] replay ok {key[0]}", flush=True)
        finally:
            outer.wait_stream(self._gstream)
            self.ctx.bind_stream()
        return ent[1]

    def _graph_entry(self, key):
        """The cached graph of key if it is still valid: a graph captured before the context
        re-allocated its scratch (another call needed more, on this or another Stitcher of
        the same device) references freed memory and is dropped here, to be re-captured."""
        ent = self._graphs.get(key)
        if ent is not None and ent[2] != self.ctx.generation():
            self._drop_graph(key)
            ent = None
        return ent

    def _drop_graph(self, key):
        g = self._graphs.pop(key)[0]
        if self._fast is not None and self._fast[1][0] is g:
            self._fast = None
        for sl, st in list(self._slot_state.items()):
            if st[0] is not None and st[0][1][0] is g:
                self._slot_state[sl] = (None, None, st[2])
        self.ctx.graph_destroy(g)

    def release_graphs(self):
        self._fast = None
        self._slot_state = {sl: (None, None, st[2]) for sl, st in self._slot_state.items()}
        for ent in self._graphs.values():
            self.ctx.graph_destroy(ent[0])
        self._graphs.clear()

    def records(self, frames_dev, focals, graph: bool = False):
        """Cylindrical projection, features, matching and RANSAC of a frame sequence.

        Returns (cyl, colnz, recs_dev); with graph=True the launches replay a hipGraph."""
        n = frames_dev.shape[0]
        if n < 2:
            raise PanoError(_lib.PANO_E_ARG, "need at least two frames")

        def seg():
            cyl, colnz = self.cylindrical(frames_dev, focals)
            feats = self.features(cyl)
            recs_dev, _ = self.pair_records(feats, [(i, i + 1) for i in range(n - 1)])
            return cyl, colnz, recs_dev

        if not graph:
            return seg()
        key = ("records", frames_dev.data_ptr(), tuple(frames_dev.shape),
               tuple(float(f) for f in np.asarray(focals, np.float64)), self.method, self.match,
               bytes(self.params), self.cap, self.max_points, self.ransac_thr, self.desc_thresh, self.ratio)
        return self._replay(key, seg)

    # ------------------------------------------------------------------ device-planned run
    def _planned(self, frames_dev, focals):
        """The whole stitch as ONE launch chain (one hipGraph with graph=True): records, the
        device plan (drift correction + composite geometry, pano_plan_device) and the planned
        composite into a capacity-sized canvas.  Returns (cyl, colnz, head, canvas) where head
        is the single host read: the records, the crop box and the plan header."""
        T = self.torch
        n, h, w, _ = frames_dev.shape
        P = n - 1
        lib, c = self.ctx.lib, self.ctx.h
        off_bb = P * 64
        off_plan = (off_bb + 4 * BBOX_SLOTS * 4 + 255) // 256 * 256
        sfx = f"@{self._slot}" if self._slot else ""
        res = self._get("result" + sfx, (off_plan + int(lib.pano_plan_device_bytes()),), T.uint8)
        # canvas capacity: every step pads by at most one frame width (|dx| <= w for real
        # overlaps) and the drift-corrected rows stay within one frame height; a plan above
        # it reports PANO_E_OVERFLOW and run() composites with the host plan instead
        Hcap, Wcap = self.canvas_cap or (2 * h, (n + 2) * w)
        canvas = self._get("canvas_cap" + sfx, (Hcap * Wcap * 3,), T.uint8)

        nhead = off_plan + 32
        pin = self._buf.get("head_pin" + sfx)
        if pin is None or pin.numel() < nhead:
            if pin is not None and self._graphs:
                # graphs captured under an earlier key copy their head into the old block:
                # drop them (the key below also carries the pinned address)
                self.release_graphs()
            pin = T.empty(max(nhead, 4096), dtype=T.uint8, pin_memory=True)
            self._buf["head_pin" + sfx] = pin
        self._head_np = pin.numpy()

        def seg():
            cyl, colnz = self.cylindrical(frames_dev, focals)
            feats = self.features(cyl)
            recs_dev, _ = self.pair_records(feats, [(i, i + 1) for i in range(P)], out=res[:off_bb])
            # the plan (drift + geometry) and the composite tables in one launch, then the pixels
            self.ctx.check(lib.pano_plan_composite_device(c, ptr(recs_dev), ptr(cyl), ptr(colnz), n, h, w,
                                                          int(self.method != "sift"), ptr(res[off_plan:]),
                                                          ptr(canvas), Hcap, Wcap, 0,
                                                          ptr(res[off_bb:off_plan])))
            # the records, crop box and plan header to pinned host memory: the one host read
            self.ctx.check(lib.pano_copy_async(c, _lib._P(pin.data_ptr()), ptr(res), nhead))
            return cyl, colnz

        self._key_planned = key = (
            "planned", frames_dev.data_ptr(), tuple(frames_dev.shape),
            tuple(float(f) for f in np.asarray(focals, np.float64)), self.method, self.match,
            bytes(self.params), self.cap, self.max_points, self.ransac_thr, self.desc_thresh,
            self.ratio, res.data_ptr(), canvas.data_ptr(), pin.data_ptr())
        ent = self._graph_entry(key) if self._graph_mode else None
        if ent is not None:       # replay on the caller's stream and wait: one library call
            cur = self._raw_stream()
            self.ctx.check(lib.pano_graph_launch_sync(c, ent[0], _lib._P(cur)))
            self.last_graphs.append(ent[0])
            cyl, colnz = ent[1]
            # the next identical call skips all of the above (run()'s fast path)
            self._fast = (self._fast_key, (ent[0], cyl, colnz, off_bb, off_plan, nhead, canvas, ent[2]))
        elif self._graph_mode:
            cyl, colnz = self._replay(key, seg)
            T.cuda.current_stream(self.device).synchronize()
        else:
            cyl, colnz = seg()
            self.ctx.sync()
        head = self._head_np[:nhead]                                     # the one sync point
        return cyl, colnz, head, off_bb, off_plan, canvas

    # ------------------------------------------------------------------ whole run
    def run(self, frames_dev, focals, margin: int = 15, timers: bool = False,
            graph: bool = False, device_plan: bool = True) -> StitchResult:
        """run_panorama's numeric body.  device_plan (default): one launch chain and one host
        read per stitch; the host-planned form (two reads) runs when the plan reports a
        canvas above capacity or a column covered by three frames, or with device_plan=False.

        The reference has no keypoint limit: a frame with more keypoints than the capacity
        (the pair records say PANO_E_OVERFLOW) re-runs the stitch once with the capacity grown
        to fit, and the Stitcher keeps the larger capacity.  The returned panorama and canvas
        are views of buffers the next run() on this Stitcher reuses: clone them to keep them."""
        try:
            return self._run(frames_dev, focals, margin, graph, device_plan)
        except PanoError as e:
            if e.code != _lib.PANO_E_OVERFLOW or self.method != "sift":
                raise
            need = self.grown_cap()
            if need is None:
                raise
            self.cap = need
            self.release_graphs()
            return self._run(frames_dev, focals, margin, graph, device_plan)

    def grown_cap(self):
        """The capacity the last SIFT features call needed (power of two >= the largest frame
        count), or None when no count exceeded the capacity (an internal-stage overflow, which
        a larger keypoint capacity does not fix)."""
        counts = self._buf.get("counts")
        if counts is None:
            return None
        c = counts.cpu().numpy()
        if (c < 0).any() or c.max() <= self.cap:
            return None
        return 1 << int(np.ceil(np.log2(int(c.max()))))

    def _use_slot(self, sl):
        """Make output slot sl current: its buffers, graph fast path and pinned head."""
        if sl == self._slot:
            return
        self._slot_state[self._slot] = (self._fast, self._fast_key, self._head_np)
        self._fast, self._fast_key, self._head_np = self._slot_state.pop(sl, (None, None, None))
        self._slot = sl

    def run_sequence(self, items, margin: int = 15):
        """Generator: run(..., graph=True) over a sequence of stitches -- items: (frames_dev,
        focals) pairs, e.g. consecutive frame sets of a video or one set re-stitched -- with two
        in flight: stitch i + 1 is launched before the host reads stitch i's head and builds its
        result, so the GPU does not idle while the host finishes a stitch (the host gap between
        synchronous run() calls).  Stitches alternate between two output slots; a
        yielded result stays valid until the generator is resumed (run()'s rule: until the next
        call).  A stitch the replay cannot finish (first use of a slot, a capacity or plan
        overflow, a missing match) drains the pipeline and goes through run().

        Graphs are keyed on the frame buffer's address.  When every item is the same resident
        buffer (one set re-stitched) the graphs replay on it directly.  When the items are
        distinct buffers (a video's frame sets), each slot owns a staging buffer: the item's
        frames are copied into it on the stream (a device copy, ~3 us per 10 MB) and the slot's
        graph, captured once on the staging buffer, replays for every item of that shape --
        no re-capture per buffer."""
        items = list(items)
        T = self.torch
        inflight = None                  # (index, slot, event, replay state)
        # host items (pinned uint8 frames, SURVEY 8(d)'s wall: frames on the host): uploaded into
        # the slot's staging buffer on the stream, right before the slot's graph replays
        on_host = any(f.device.type == "cpu" for f, _ in items)
        shared = not on_host and len({(f.data_ptr(), tuple(f.shape)) for f, _ in items}) <= 1
        dev = T.device("cuda", self.device) if isinstance(self.device, int) else T.device(self.device)

        def src_of(i):
            frames_dev = items[i][0]
            if shared:
                return frames_dev
            stg = self._stage.get(i % 2)
            if stg is None or stg.shape != frames_dev.shape or stg.dtype != frames_dev.dtype:
                stg = self._stage[i % 2] = T.empty(frames_dev.shape, dtype=frames_dev.dtype, device=dev)
            return stg

        def launch(i):
            sl = i % 2
            self._use_slot(sl)
            frames_dev, focals = items[i]
            src = src_of(i)
            fast = self._fast
            if (fast is None or fast[0] != self._fast_key_of(src, focals)
                    or fast[1][7] != self.ctx.generation()):
                return None
            if src is not frames_dev:
                if on_host:
                    # the upload on a copy stream: it overlaps the running stitch i - 1 (the
                    # slot's previous reader, stitch i - 2, has finished: its result was read)
                    cs = self._copy_stream()
                    with T.cuda.stream(cs):
                        src.copy_(frames_dev, non_blocking=True)
                        up = T.cuda.Event()
                        up.record(cs)
                    T.cuda.current_stream(self.device).wait_event(up)
                else:
                    src.copy_(frames_dev, non_blocking=True)  # same stream as the replay
            g = fast[1][0]
            self.ctx.check(self.ctx.lib.pano_graph_launch_stream(self.ctx.h, g, _lib._P(self._raw_stream())))
            ev = T.cuda.Event()
            ev.record()
            return (i, sl, ev, fast[1])

        def finish(job):
            i, sl, ev, state = job
            _, cyl, colnz, off_bb, off_plan, nhead, canvas, _ = state
            t0 = time.perf_counter()
            ev.synchronize()
            head = self._slot_head(sl)[:nhead]
            hdr = int(head[off_plan:off_plan + 4].view(np.int32)[0])
            if hdr != _lib.PANO_OK or head[:off_bb].view(np.int32).reshape(-1, 16)[:, 15].any():
                return None
            self._use_slot(sl)
            return self._from_head(head, off_bb, off_plan, canvas, cyl, colnz, margin, True, {}, t0)

        try:
            i = 0
            while i < len(items) or inflight is not None:
                nxt = launch(i) if i < len(items) else None
                if i < len(items) and nxt is None:
                    # not replayable yet: drain, then the synchronous path (captures the graph)
                    if inflight is not None:
                        job, inflight = inflight, None
                        r = finish(job)
                        yield r if r is not None else self._rerun(items, job[0], margin, src_of)
                    yield self._rerun(items, i, margin, src_of)
                    i += 1
                    continue
                if inflight is not None:
                    job, inflight = inflight, None
                    r = finish(job)
                    if r is None:
                        # drain the launched successor, redo this stitch synchronously, then
                        # re-issue the successor
                        if nxt is not None:
                            nxt[2].synchronize()
                        yield self._rerun(items, job[0], margin, src_of)
                        if nxt is not None:
                            i = nxt[0]
                            continue
                    else:
                        yield r
                inflight = nxt
                i += 1
        finally:
            if inflight is not None:
                inflight[2].synchronize()
            self._use_slot(0)

    def _copy_stream(self):
        """A private stream for the host-item uploads and downloads of run_sequence /
        StitchPool.run_sequence(to_host=True)."""
        if getattr(self, "_cstream", None) is None:
            self._cstream = self.torch.cuda.Stream(self.device)
        return self._cstream

    def _rerun(self, items, i, margin, src_of):
        self._use_slot(i % 2)
        src = src_of(i)
        if src is not items[i][0]:
            src.copy_(items[i][0], non_blocking=True)
        return self.run(src, items[i][1], margin=margin, graph=True)

    def _slot_head(self, sl):
        return self._head_np if sl == self._slot else self._slot_state[sl][2]

    def _fast_key_of(self, frames_dev, focals):
        return (frames_dev.data_ptr(), tuple(frames_dev.shape),
                np.asarray(focals, np.float64).tobytes(), self.canvas_cap, self.method, self.match,
                self.ratio, self.desc_thresh, self.ransac_thr, bytes(self.params), self.cap,
                self.max_points)

    def _run(self, frames_dev, focals, margin, graph, device_plan):
        t = {}
        tick = time.perf_counter
        t0 = tick()
        self.last_graphs = []
        n = frames_dev.shape[0]
        if device_plan and 2 <= n <= 256:
            self._graph_mode = graph
            # replay fast path: same frames buffer, focals and settings as the last replay
            fk = self._fast_key_of(frames_dev, focals) if graph else None
            fast = self._fast
            if fast is not None and fast[0] == fk and fast[1][7] == self.ctx.generation():
                g, cyl, colnz, off_bb, off_plan, nhead, canvas, _ = fast[1]
                cur = self._raw_stream()
                self.ctx.check(self.ctx.lib.pano_graph_launch_sync(self.ctx.h, g, _lib._P(cur)))
                self.last_graphs.append(g)
                head = self._head_np[:nhead]
            else:
                self._fast_key = fk
                cyl, colnz, head, off_bb, off_plan, canvas = self._planned(frames_dev, focals)
            return self._from_head(head, off_bb, off_plan, canvas, cyl, colnz, margin, graph, t, t0)
        cyl, colnz, recs_dev = self.records(frames_dev, focals, graph)
        recs = recs_dev.cpu().numpy().view(_lib.PAIR_NP).reshape(-1)   # sync point 1
        t["features_match_ransac"] = tick() - t0
        self._check_records(recs)
        return self._finish(cyl, colnz, recs, margin, graph, t, t0)

    def _from_head(self, head, off_bb, off_plan, canvas, cyl, colnz, margin, graph, t, t0):
        """The StitchResult of a device-planned stitch from its pinned head (records, crop box,
        plan header)."""
        tick = time.perf_counter
        head = head.copy()          # ONE read of the pinned head; the next run() reuses it
        recs = head[:off_bb].view(_lib.PAIR_NP).reshape(-1)
        hdr = head[off_plan:off_plan + 32].view(np.int32)
        t["features_match_ransac"] = tick() - t0
        status = head[:off_bb].view(np.int32).reshape(-1, 16)[:, 15]     # PAIR_NP.status
        if status.any():
            self._check_records(recs)
        if hdr[0] == _lib.PANO_E_NOMATCH:
            raise PanoError(_lib.PANO_E_NOMATCH, "a pair has no descriptor match")
        if hdr[0] == _lib.PANO_OK:
            if self.method == "sift" and not status.any():
                # the records' six doubles (dx dy xA yA xB yB) in one conversion
                rows = head[:off_bb].view(np.float64).reshape(-1, 8)[:, :6].tolist()
                shifts = [(r[0], r[1]) for r in rows]
                best_pairs = [((r[2], r[3]), (r[4], r[5])) for r in rows]
            else:
                shifts, best_pairs = self._shifts(recs)
            H, W = int(hdr[1]), int(hdr[2])
            # crop box: min of ymin / xmin and max of ymax / xmax over the partial boxes,
            # as one min over the sign-flipped columns
            slots = head[off_bb:off_bb + 16 * BBOX_SLOTS].view(np.int32).reshape(BBOX_SLOTS, 4)
            m = (slots * _BOX_SIGN).min(axis=0).tolist()
            bb = (m[0], -m[1], m[2], -m[3])
            return self._crop_planned(canvas, H, W, bb, margin, shifts, best_pairs, recs, t, t0)
        # PANO_E_OVERFLOW: composite with the host plan below, reusing the records
        return self._finish(cyl, colnz, recs, margin, graph, t, t0)

    @staticmethod
    def _check_records(recs):
        bad = np.nonzero(recs["status"] == _lib.PANO_E_OVERFLOW)[0]
        if len(bad):
            raise PanoError(_lib.PANO_E_OVERFLOW,
                            f"pairs {bad.tolist()}: a frame has more keypoints than the capacity")

    def _shifts(self, recs):
        """Per-pair moves and best pairs as the reference's Python values: floats of the
        float32 coordinates for SIFT, int() of them for Harris."""
        if np.any(recs["status"] != _lib.PANO_OK):
            # the reference's blend would fail on a None pair (image_stitching_sift.py:164)
            raise PanoError(_lib.PANO_E_NOMATCH, "a pair has no descriptor match")
        cols = [recs[k] for k in ("dx", "dy", "xA", "yA", "xB", "yB")]
        if self.method != "sift":
            cols = [np.trunc(c).astype(np.int64) for c in cols]
        dx, dy, xa, ya, xb, yb = (c.tolist() for c in cols)
        shifts = list(zip(dx, dy))
        best_pairs = [((a, b), (c, d)) for a, b, c, d in zip(xa, ya, xb, yb)]
        return shifts, best_pairs

    def _finish(self, cyl, colnz, recs, margin, graph, t, t0):
        self.ctx.sync()
        shifts, best_pairs = self._shifts(recs)
        corr = drift_correct(shifts)
        pxy = [(a[0], a[1], b[0], b[1]) for a, b in best_pairs]
        canvas, bb_dev = self.composite(cyl, colnz, corr, pxy, bbox=True, graph=graph)
        bb = bb_dev.cpu().numpy()                                        # sync point 2
        return self._crop(canvas, bb, margin, shifts, best_pairs, recs, t, t0)

    def _crop_planned(self, buf, H, W, bb, margin, shifts, best_pairs, recs, t, t0):
        """_crop on the device-planned canvas (an H x W x 3 view of the capacity buffer), with
        one strided view each for the canvas and the panorama."""
        if bb[1] < 0:
            y0, y1, x0, x1 = 0, H - 1, 0, W - 1
        else:
            y0 = max(0, bb[0] + margin)
            y1 = min(H - 1, bb[1] - margin)
            x0, x1 = bb[2], bb[3]
        # the two views of the same buffer and geometry are reused from the last call (a
        # replayed stitch usually has both): creating them costs more than the rest of run()
        vk = (buf.data_ptr(), H, W, y0, y1, x0, x1)
        views = self._views.get(vk)
        if views is None:
            canvas = buf.as_strided((H, W, 3), (W * 3, 3, 1))
            pano = canvas if (bb[1] < 0 or y0 > y1 or x0 > x1) else buf.as_strided(
                (y1 + 1 - y0, x1 + 1 - x0, 3), (W * 3, 3, 1), buf.storage_offset() + y0 * W * 3 + x0 * 3)
            if len(self._views) >= 8:
                self._views.clear()
            self._views[vk] = views = (canvas, pano)
        canvas, pano = views
        t["total"] = time.perf_counter() - t0
        return StitchResult(pano, canvas, shifts, best_pairs, recs, (y0, y1, x0, x1), t)

    def _crop(self, canvas, bb, margin, shifts, best_pairs, recs, t, t0):
        """rectangle_crop (image_stitching_sift.py:208-247) from the fused bbox."""
        tick = time.perf_counter
        H = canvas.shape[0]
        if bb[1] < 0:
            y0, y1, x0, x1 = 0, H - 1, 0, canvas.shape[1] - 1
            pano = canvas
        else:
            y0 = max(0, int(bb[0]) + margin)
            y1 = min(H - 1, int(bb[1]) - margin)
            x0, x1 = int(bb[2]), int(bb[3])
            pano = canvas if (y0 > y1 or x0 > x1) else canvas.as_strided(
                (y1 + 1 - y0, x1 + 1 - x0, 3), canvas.stride(), canvas.storage_offset() +
                y0 * canvas.stride(0) + x0 * 3)
        t["total"] = tick() - t0
        return StitchResult(pano, canvas, shifts, best_pairs, recs, (y0, y1, x0, x1), t)


class StitchPool:
    """A sequence of stitches over k Stitchers with PRIVATE libpano contexts (each its own
    scratch) and streams: stitch i runs on member i % k, so one stitch's latency-bound stages
    (the small blur octaves, the sort, the post-descriptor chain, the plan) overlap another's
    bandwidth-bound ones on the device.  Each member keeps its own run_sequence (two stitches
    in flight, graphs captured on its first items), so up to 2k stitches are in flight; the
    results come back in item order and are bit-identical to Stitcher.run's.  A yielded result
    stays valid until the generator is resumed (in fact until its member's next one, k items
    later).  Each member runs its blur tail on its own stream (PANO_CTX_TAIL_MAIN), so k
    members use k streams: k = 4 matches the process's 4 hardware queues (GPU_MAX_HW_QUEUES).
    Measured on MI355X: parrington 0.753 ms per stitch at k = 4, 0.772 at 3,
    0.835 at 2, 0.78 at 6 and 8, against 0.98 with one context.

    ``kw`` are Stitcher's arguments (method, cap, match, ...)."""

    def __init__(self, method: str = "sift", contexts: int = 4, device: int | None = None, **kw):
        import torch
        self.torch = torch
        dev = torch.cuda.current_device() if device is None else device
        if contexts < 1:
            raise PanoError(_lib.PANO_E_ARG, "StitchPool needs at least one context")
        self.members = [Stitcher(method, device=dev, ctx=_lib.Context(dev), **kw) for _ in range(contexts)]
        if contexts > 1:
            # the blur tail on each member's own stream: with another stitch filling the device
            # the side stream's fork / join edges cost more than the overlap it buys (bench A/B:
            # 0.832-0.837 against 0.839-0.842 ms per stitch)
            # and the distance GEMM without candidate splits (fewer, longer workgroups: 0.741-0.743
            # against 0.745-0.748 ms per stitch at four contexts)
            for st in self.members:
                st.ctx.set_flags(_lib.PANO_CTX_TAIL_MAIN | _lib.PANO_CTX_MATCH_WHOLE)
        self.streams = [torch.cuda.Stream(dev) for _ in range(contexts)]
        self.device = self.members[0].device

    def upload(self, frames):
        """Frames to the device (one buffer every member reads)."""
        return self.members[0].upload(frames)

    def run_sequence(self, items, margin: int = 15, to_host: bool = False):
        """Generator over StitchResults of items ((frames, focals) pairs) in order.

        Host-to-host form (SURVEY 8(d)'s wall: decoded frames on the host -> cropped panorama on
        the host): items whose frames are pinned host tensors are uploaded on their member's
        stream right before its stitch, and with to_host=True every panorama is copied to a
        pinned host buffer on the same stream (``result.host``, a numpy view valid until the
        member's next result, k items later).  The copies of one member overlap the other
        members' stitches on the device, so the PCIe legs leave the per-stitch rate."""
        T = self.torch
        items = list(items)
        k = len(self.members)
        cur = T.cuda.current_stream(self.device)
        for s in self.streams:
            s.wait_stream(cur)                   # inputs made on the caller's stream
        gens = []
        for m, (st, s) in enumerate(zip(self.members, self.streams)):
            with T.cuda.stream(s):
                gens.append(st.run_sequence(items[m::k], margin=margin))
        pins = [None] * k
        pending = None                           # (result, its download's event): yielded one item late
        try:
            for i in range(len(items)):
                m = i % k
                with T.cuda.stream(self.streams[m]):
                    r = next(gens[m])
                if not to_host:
                    yield r
                    continue
                # the stitch is complete (its head was read); the download goes on the member's
                # copy stream -- its own stream already holds the next stitch, which the copy must
                # not wait behind -- and later work on the member stream (the stitch that reuses
                # this canvas slot) waits for it.  The result is yielded one item later, when its
                # download has had the next item's host work to finish in (with one member, at once)
                # the crop's canvas rows are one contiguous byte range: one plain copy (no
                # device-side gather of the strided view), the host array a strided view of it
                cs = self.members[m]._copy_stream()
                pano, canvas = r.panorama, r.canvas
                row = canvas.stride(0)
                off = pano.storage_offset() - canvas.storage_offset()
                first, col0 = off // row, off % row
                nb = pano.shape[0] * row
                pin = pins[m]
                if pin is None or pin.numel() < nb:
                    pin = pins[m] = T.empty(max(nb, 1 << 20), dtype=T.uint8, pin_memory=True)
                with T.cuda.stream(cs):
                    pin[:nb].copy_(canvas.reshape(-1)[first * row:first * row + nb], non_blocking=True)
                    ev = T.cuda.Event()
                    ev.record(cs)
                self.streams[m].wait_event(ev)
                r.host = np.lib.stride_tricks.as_strided(pin.numpy()[col0:], shape=tuple(pano.shape),
                                                         strides=(row, pano.stride(1), pano.stride(2)),
                                                         writeable=False)
                if k == 1:
                    ev.synchronize()
                    yield r
                    continue
                if pending is not None:
                    pending[1].synchronize()
                    yield pending[0]
                pending = (r, ev)
            if pending is not None:
                pending[1].synchronize()
                yield pending[0]
        finally:
            for g, s in zip(gens, self.streams):
                with T.cuda.stream(s):
                    g.close()
            for s in self.streams:
                cur.wait_stream(s)

    def release_graphs(self):
        for st in self.members:
            st.release_graphs()
