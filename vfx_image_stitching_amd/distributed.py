"""Multi-GPU stitching: pairs shard across ranks, one gather of per-pair records.

SURVEY.md section 8(e): pairs are independent until drift correction / compositing, so

  1. rank r owns a contiguous range of pairs and the frames they touch (+1 boundary
     frame); it runs cylindrical projection, features, matching and RANSAC locally;
  2. ONE all_gather (RCCL over xGMI for backend "nccl", gloo on CPU tests) of the 64-byte
     pano_pair_rec records of every pair -- the only data-path exchange;
  3. every rank replays drift correction and the composite plan for the WHOLE sequence
     on the host (a few microseconds), then composites its own band of the canvas.
     Bands are independent when no column is covered by three frames (frame i never
     reaches frame i-2: true whenever |dx| > w/2, e.g. parrington / grail / synthetic);
     otherwise band compositing is refused (``BandError``).
  4. rectangle_crop needs the global bounding box, and rank 0 needs every band's place: ONE
     all_gather of 8 int64 per rank (box, owned columns, fallback flag);
  5. the owned bands go to rank 0 point to point (RCCL send / recv over xGMI), which places
     them into the final canvas and crops it: the panorama exists on rank 0 at the end of
     every step, as on one GPU.  If any rank's band is refused (a column covered by three
     frames, a band above its capacity), every rank sees it in the layout exchange and the
     frames go to rank 0 instead, which runs the sequential fold (the reference's blend order).

The host logic here is device-agnostic so it is unit-tested with gloo on the CPU; the
GPU work is the libpano calls of pipeline.Stitcher.
"""
from __future__ import annotations

import time

import numpy as np

from . import _lib
from ._lib import PanoError


class BandError(PanoError):
    """The device plan refused this rank's band.  ``plan_status`` is the global plan's status
    (PANO_OK when the global plan is fine and only the band split failed), ``band_status``
    the band plan's; ``records`` the gathered pair records (for a host-planned fallback)."""

    def __init__(self, msg, plan_status=_lib.PANO_OK, band_status=_lib.PANO_OK, records=None):
        super().__init__(_lib.PANO_E_UNSUPPORTED, msg)
        self.plan_status = int(plan_status)
        self.band_status = int(band_status)
        self.records = records


def shard_ranges(n_pairs: int, world: int):
    """Contiguous balanced pair ranges: rank r -> (first pair, pair count)."""
    base, extra = divmod(n_pairs, world)
    out, start = [], 0
    for r in range(world):
        c = base + (1 if r < extra else 0)
        out.append((start, c))
        start += c
    return out


def gather_records(local: "object", counts, group=None):
    """all_gather of fixed-size uint8 [P_max, 64] record blocks -> global PAIR_NP array."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    pmax = max(counts)
    buf = torch.zeros((pmax, 64), dtype=torch.uint8, device=local.device)
    buf[:local.shape[0]] = local
    out = torch.empty((world * pmax, 64), dtype=torch.uint8, device=local.device)
    dist.all_gather_into_tensor(out, buf, group=group)
    h = out.cpu().numpy().reshape(world, pmax, 64)
    recs = [h[r, :counts[r]] for r in range(world)]
    return np.ascontiguousarray(np.concatenate(recs)).view(_lib.PAIR_NP).reshape(-1)


def records_to_shifts(recs, integer=False):
    shifts, pairs = [], []
    for r in recs:
        if r["status"] != _lib.PANO_OK:
            raise PanoError(_lib.PANO_E_NOMATCH, "a pair has no descriptor match")
        cast = int if integer else float
        shifts.append((cast(r["dx"]), cast(r["dy"])))
        pairs.append(((cast(r["xA"]), cast(r["yA"])), (cast(r["xB"]), cast(r["yB"]))))
    return shifts, pairs


def global_plan(shifts_corr, pairs, n_frames, h, w):
    """pano_plan_composite over the whole sequence -> (steps list, first_xy, (H, W))."""
    lib = _lib.load()
    sh = np.ascontiguousarray(np.array(shifts_corr, np.float64).reshape(-1, 2))
    pr = np.ascontiguousarray(np.array([[a[0], a[1], b[0], b[1]] for a, b in pairs],
                                       np.float64).reshape(-1, 4))
    steps = (_lib.Step * max(n_frames - 1, 1))()
    first = np.zeros(2, np.int32)
    hw = np.zeros(2, np.int32)
    rc = lib.pano_plan_composite(_lib.f64p(sh), _lib.f64p(pr), n_frames, h, w, steps,
                                 _lib.i32p(first), _lib.i32p(hw))
    if rc:
        raise PanoError(rc, "pano_plan_composite")
    return list(steps)[:n_frames - 1], first.copy(), (int(hw[0]), int(hw[1]))


def frame_xy(steps, first, i):
    """Final-canvas top-left of frame i's content."""
    if i == 0:
        return int(first[0]), int(first[1])
    s = steps[i - 1]
    return int(s.frame_x), int(s.frame_y)


def check_bands(steps, first, w):
    """Band compositing is exact iff frame i never overlaps frame i-2 (see module doc)."""
    for i in range(2, len(steps) + 1):
        xi = frame_xy(steps, first, i)[0]
        xk = frame_xy(steps, first, i - 2)[0]
        if not (xi + w <= xk or xk + w <= xi):
            raise BandError(f"frames {i} and {i - 2} overlap: bands are not independent")


def last_cover(steps, first, w, i, n_frames):
    """Columns whose final value is written by frame i: its span minus frame i+1's span.

    With no column covered by three frames (check_bands), only frame i+1 can overwrite
    frame i, so a canvas column's final value is fixed by its LAST covering frame i and
    that frame's predecessor i-1.  Returns a list of disjoint [lo, hi) intervals.
    """
    lo, hi = frame_xy(steps, first, i)[0], frame_xy(steps, first, i)[0] + w
    if i + 1 >= n_frames:
        return [(lo, hi)]
    nlo = frame_xy(steps, first, i + 1)[0]
    nhi = nlo + w
    out = []
    if lo < min(hi, nlo):
        out.append((lo, min(hi, nlo)))
    if max(lo, nhi) < hi:
        out.append((max(lo, nhi), hi))
    return out


def owned_columns(steps, first, w, f0, count, n_frames):
    """Canvas columns a band of frames f0 .. f0+count composites to their final value.

    The band holds frames f0 .. f0+count and applies steps f0+1 .. f0+count, so it owns the
    columns whose last covering frame is in (f0, f0+count] -- plus frame 0's for the first
    band.  Returns one [lo, hi) interval (BandError if the union is not contiguous).
    """
    iv = []
    for i in range(f0 if f0 == 0 else f0 + 1, f0 + count + 1):
        iv.extend(last_cover(steps, first, w, i, n_frames))
    if not iv:
        return (0, 0)
    iv.sort()
    lo, hi = iv[0]
    for a, b in iv[1:]:
        if a > hi:
            raise BandError(f"band {f0}..{f0 + count} owns non-contiguous columns")
        hi = max(hi, b)
    return lo, hi


def band_plan(steps, first, w, H, f0, count, n_frames=None):
    """Local composite plan for frames f0 .. f0+count (rank's range incl. boundary frame).

    Returns (local_steps, local_first_xy, x_offset, band_width, owned (x0, x1)).
    The band starts from frame f0 as it stands before step f0+1 (its raw pixels in the
    columns the next frame can reach: frame f0+1 never meets frame f0-1) and applies
    global steps f0+1 .. f0+count.  Owned columns: see owned_columns.
    """
    if n_frames is None:
        n_frames = len(steps) + 1
    xs = [frame_xy(steps, first, f0 + k)[0] for k in range(count + 1)]
    x_lo, x_hi = min(xs), max(xs) + w
    loc = (_lib.Step * max(count, 1))()
    for k in range(count):
        g = steps[f0 + k]
        s = loc[k]
        for name, _ in _lib.Step._fields_:
            setattr(s, name, getattr(g, name))
        s.frame_x = g.frame_x - x_lo
        s.canvas_x = g.canvas_x - x_lo
    fx, fy = frame_xy(steps, first, f0)
    first_loc = np.array([fx - x_lo, fy], np.int32)
    own_lo, own_hi = owned_columns(steps, first, w, f0, count, n_frames)
    assert x_lo <= own_lo and own_hi <= x_hi
    return loc, first_loc, x_lo, x_hi - x_lo, (own_lo, own_hi)


def local_records(stitcher, frames_dev, focals, graph=False):
    """Cylindrical projection, features, matching and RANSAC of one rank's frames."""
    cyl, colnz, recs_dev = stitcher.records(frames_dev, focals, graph)
    return recs_dev, cyl, colnz


def composite_band(stitcher, cyl, colnz, recs, pair_start, check=True):
    """Drift + global plan from ALL records, then this rank's band of the canvas.

    Returns (owned band view [H, own_hi-own_lo, 3] on device, own_lo, (H, W)).
    """
    import torch
    n_local, h, w = cyl.shape[0], cyl.shape[1], cyl.shape[2]
    from .pipeline import drift_correct
    shifts, pairs = records_to_shifts(recs, integer=stitcher.method != "sift")
    n_frames = len(shifts) + 1
    steps, first, (H, W) = global_plan(drift_correct(shifts), pairs, n_frames, h, w)
    if check:
        check_bands(steps, first, w)
    loc, first_loc, x0, bw, (own_lo, own_hi) = band_plan(steps, first, w, H, pair_start,
                                                         n_local - 1, n_frames)
    band = stitcher._get("band", (H, bw, 3), torch.uint8)
    ctx = stitcher.ctx
    ctx.check(ctx.lib.pano_composite(ctx.h, _lib.ptr(cyl), _lib.ptr(colnz), n_local, h, w, loc,
                                     _lib.i32p(first_loc), _lib.ptr(band), H, bw))
    return band[:, own_lo - x0:own_hi - x0], own_lo, (H, W)


NO_BOX = (1 << 30, -1, 1 << 30, -1)


def global_bbox(local_bbox, group=None):
    """rectangle_crop's box over all bands: elementwise min/max of [ymin ymax xmin xmax]
    (int64 tensor; a band with no pixel contributes NO_BOX).  One 4-int all_reduce."""
    import torch
    import torch.distributed as dist
    b = local_bbox.to(torch.int64).clone()
    # (-ymin, ymax, -xmin, xmax) under one MAX reduction
    v = torch.stack([-b[0], b[1], -b[2], b[3]])
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(v, op=dist.ReduceOp.MAX, group=group)
    v = v.cpu().numpy()
    return int(-v[0]), int(v[1]), int(-v[2]), int(v[3])


def rank_records(stitcher, frames_dev, focals, pmax, graph=False):
    """Segment 1 of a rank's step (the single-GPU launch chain up to the pair records):
    cylindrical projection, features, matching and RANSAC of the rank's frames, the records
    written into a zero-padded [pmax, 64] uint8 device block (what the all_gather moves).
    Returns (block, cyl, colnz)."""
    import torch
    st = stitcher
    n_local = frames_dev.shape[0]
    block = st._get("recs_block", (pmax, 64), torch.uint8)

    def seg():
        cyl, colnz = st.cylindrical(frames_dev, focals)
        feats = st.features(cyl)
        st.pair_records(feats, [(i, i + 1) for i in range(n_local - 1)], out=block[:n_local - 1])
        return cyl, colnz

    if not graph:
        block.zero_()
        cyl, colnz = seg()
        return block, cyl, colnz
    key = ("rank_records", frames_dev.data_ptr(), tuple(frames_dev.shape),
           np.asarray(focals, np.float64).tobytes(), pmax, st.method, st.match, bytes(st.params),
           st.cap, st.max_points, st.ransac_thr, st.desc_thresh, st.ratio)
    if st._graph_entry(key) is None:
        block.zero_()                      # padding rows stay zero in every replay
    cyl, colnz = st._replay(key, seg)
    return block, cyl, colnz


def _staged(t, group):
    """gloo moves host memory only: a device tensor in a gloo group (the multi-process tests on
    one GPU) is exchanged through a host copy.  RCCL ("nccl") moves device memory directly."""
    import torch.distributed as dist
    return t.is_cuda and dist.get_backend(group) == "gloo"


def all_gather_dev(out, inp, group=None):
    """all_gather_into_tensor(out, inp): device to device over RCCL; staged through host
    memory for a gloo group on device tensors."""
    import torch.distributed as dist
    if _staged(inp, group):
        o = out.cpu()
        dist.all_gather_into_tensor(o, inp.cpu(), group=group)
        out.copy_(o)
        return out
    dist.all_gather_into_tensor(out, inp, group=group)
    return out


def _p2p(ops_spec, group=None):
    """batch_isend_irecv of (op, tensor, peer) triples; gloo on device tensors goes through
    host copies (receives copied back after the wait)."""
    import torch.distributed as dist
    ops, back = [], []
    for op, t, peer in ops_spec:
        if _staged(t, group):
            h = t.cpu() if op is dist.isend else t.new_empty(t.shape, device="cpu")
            if op is dist.irecv:
                back.append((t, h))
            t = h
        ops.append(dist.P2POp(op, t, peer, group))
    if ops:
        for q in dist.batch_isend_irecv(ops):
            q.wait()
    for t, h in back:
        t.copy_(h)


def gather_blocks(block, group=None):
    """THE collective of a sharded stitch: all_gather_into_tensor of every rank's [pmax, 64]
    record block, device to device (RCCL over xGMI for backend "nccl"; gloo on CPU tensors)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        return block
    out = torch.empty((world * block.shape[0], 64), dtype=torch.uint8, device=block.device)
    return all_gather_dev(out, block, group)


def block_layout(pair_counts):
    """Where each rank's records sit: rank r's block of the gathered [world * pmax, 64] array
    starts at row r * pmax and its records land at global pair starts[r] (pair order)."""
    pmax = max(pair_counts)
    starts = np.concatenate([[0], np.cumsum(pair_counts)]).astype(np.int64)
    return pmax, starts


def compact_blocks(gathered, pair_counts):
    """The global [P, 64] record array from gathered blocks (torch; rank_band does the same
    with device copies inside its launch chain)."""
    import torch
    pmax, _ = block_layout(pair_counts)
    return torch.cat([gathered[r * pmax:r * pmax + c] for r, c in enumerate(pair_counts)])


def rank_band(stitcher, cyl, colnz, gathered, pair_counts, f0, margin=15, graph=False):
    """Segment 2 (device-planned, one host read): compact the gathered blocks into the global
    record array, pano_plan_device over the WHOLE sequence (drift correction + geometry),
    pano_band_plan for this rank's frames f0 .. f0 + n_local - 1, pano_composite_planned of its
    band, and one pinned copy of {records, crop-box partials, band info, plan header}.
    Returns (records PAIR_NP, band view [H, own_hi - own_lo, 3] on device, own_lo, (H, W),
    local crop box (ymin, ymax, xmin, xmax) in global columns or NO_BOX)."""
    import torch
    S = rank_band_launch(stitcher, cyl, colnz, gathered, pair_counts, f0, graph)
    torch.cuda.current_stream(stitcher.device).synchronize()      # the one host read
    return rank_band_finish(S, S["pin"].numpy()[:S["nhead"]])


def rank_band_launch(stitcher, cyl, colnz, gathered, pair_counts, f0, graph=False):
    """rank_band's launches, nothing read back: the global plan, this rank's band plan and
    composite, the band's layout row (pano_band_layout_row, 8 int64 at S["row"]) and the
    pinned copy of the head.  Returns the state rank_band_finish parses."""
    import torch
    from .pipeline import BBOX_SLOTS
    st = stitcher
    lib, c = st.ctx.lib, st.ctx.h
    n_local, h, w = cyl.shape[0], cyl.shape[1], cyl.shape[2]
    pmax, starts = block_layout(pair_counts)
    P = int(starts[-1])
    plan_bytes = int(lib.pano_plan_device_bytes())
    off_bb = P * 64
    off_band = off_bb + 16 * BBOX_SLOTS
    off_row = off_band + 16                      # the layout row: 8 int64 (8-byte aligned)
    off_gp = (off_row + 64 + 255) // 256 * 256
    off_lp = off_gp + (plan_bytes + 255) // 256 * 256
    res = st._get("band_result", (off_lp + plan_bytes,), torch.uint8)
    Hcap, Wcap = st.canvas_cap or (2 * h, (n_local + 2) * w)
    canvas = st._get("band_canvas", (Hcap * Wcap * 3,), torch.uint8)
    nhead = off_gp + 32
    world = len(pair_counts)
    npin = nhead + 64 * world                    # + the gathered layout table (run_rank)
    pin = st._buf.get("band_pin")
    if pin is None or pin.numel() < npin:
        if pin is not None and st._graphs:
            # graphs captured under an earlier key copy their head into the old block: drop
            # them (the key below also carries the pinned address)
            st.release_graphs()
        pin = torch.empty(max(npin, 4096), dtype=torch.uint8, pin_memory=True)
        st._buf["band_pin"] = pin

    def seg():
        for r, cnt in enumerate(pair_counts):
            if cnt:
                st.ctx.check(lib.pano_copy_async(c, _lib._P(res.data_ptr() + int(starts[r]) * 64),
                                                 _lib._P(gathered.data_ptr() + r * pmax * 64), cnt * 64))
        st.ctx.check(lib.pano_plan_device(c, _lib.ptr(res[:off_bb]), P + 1, h, w,
                                          int(st.method != "sift"), Hcap, 1 << 30,
                                          _lib.ptr(res[off_gp:off_lp])))
        st.ctx.check(lib.pano_band_plan(c, _lib.ptr(res[off_gp:off_lp]), f0, n_local, w, Wcap,
                                        _lib.ptr(res[off_lp:]), _lib.ptr(res[off_band:off_gp])))
        st.ctx.check(lib.pano_composite_planned(c, _lib.ptr(cyl), _lib.ptr(colnz), n_local, h, w,
                                                _lib.ptr(res[off_lp:]), _lib.ptr(canvas), Hcap, Wcap, 0,
                                                _lib.ptr(res[off_bb:off_band])))
        st.ctx.check(lib.pano_band_layout_row(c, _lib.ptr(res[off_gp:off_lp]), _lib.ptr(res[off_band:off_row]),
                                              _lib.ptr(res[off_bb:off_band]), _lib.ptr(res[off_row:off_row + 64])))
        st.ctx.check(lib.pano_copy_async(c, _lib._P(pin.data_ptr()), _lib.ptr(res), nhead))

    if graph:
        key = ("rank_band", cyl.data_ptr(), colnz.data_ptr(), tuple(cyl.shape), gathered.data_ptr(),
               tuple(pair_counts), f0, st.method, Hcap, Wcap, res.data_ptr(), canvas.data_ptr(),
               pin.data_ptr())
        st._replay(key, seg)
    else:
        seg()
    return {"st": st, "pin": pin, "nhead": nhead, "off_bb": off_bb, "off_band": off_band,
            "off_gp": off_gp, "row": res[off_row:off_row + 64].view(torch.int64).view(1, LAYOUT_INTS),
            "canvas": canvas, "f0": f0, "n_local": n_local, "Hcap": Hcap, "Wcap": Wcap}


def rank_band_finish(S, head):
    """rank_band's result from the pinned head (records, crop-box partials, band info, the
    global plan header); raises BandError when the plan or the band plan refused."""
    from .pipeline import BBOX_SLOTS
    st, off_bb, off_band, off_gp = S["st"], S["off_bb"], S["off_band"], S["off_gp"]
    f0, n_local, Hcap, Wcap, canvas = S["f0"], S["n_local"], S["Hcap"], S["Wcap"], S["canvas"]
    recs = head[:off_bb].view(_lib.PAIR_NP).reshape(-1).copy()
    st._check_records(recs)
    band = head[off_band:off_band + 16].view(np.int32)
    gst = head[off_gp:off_gp + 32].view(np.int32)
    if gst[0] == _lib.PANO_E_NOMATCH:
        raise PanoError(_lib.PANO_E_NOMATCH, "a pair has no descriptor match")
    if gst[0] != _lib.PANO_OK:
        raise BandError(f"global device plan status {int(gst[0])}: the canvas exceeds the capacity "
                        f"({Hcap} rows) or a column is covered by three frames",
                        plan_status=gst[0], band_status=band[0], records=recs)
    if band[0] != _lib.PANO_OK:
        raise BandError(f"band plan status {int(band[0])} for frames {f0}..{f0 + n_local - 1}: the "
                        "owned columns are not contiguous or wider than the band capacity "
                        f"({Wcap} columns)", plan_status=gst[0], band_status=band[0], records=recs)
    H, W, own_lo, own_hi = int(gst[1]), int(gst[2]), int(band[1]), int(band[2])
    bw = own_hi - own_lo
    view = canvas[:H * bw * 3].view(H, bw, 3)
    slots = head[off_bb:off_band].view(np.int32).reshape(BBOX_SLOTS, 4)
    box = (int(slots[:, 0].min()), int(slots[:, 1].max()), int(slots[:, 2].min()), int(slots[:, 3].max()))
    box = NO_BOX if box[1] < 0 else (box[0], box[1], box[2] + own_lo, box[3] + own_lo)
    return recs, view, own_lo, (H, W), box


LAYOUT_INTS = 8                # per rank: ymin ymax xmin xmax own_lo own_hi fallback plan-status


def _root(group):
    import torch.distributed as dist
    return dist.get_global_rank(group, 0) if group is not None else 0


def exchange_layout(box, own, fallback, group=None, device=None):
    """The layout collective of a sharded step: all_gather of LAYOUT_INTS int64 per rank --
    this rank's crop box (ymin, ymax, xmin, xmax in global columns, NO_BOX when its band has no
    pixel above the threshold), its owned columns [lo, hi) and whether its band was refused.
    Returns the int64 [world, LAYOUT_INTS] numpy table every rank then reads."""
    import torch
    import torch.distributed as dist
    row = torch.tensor([[*box, own[0], own[1], int(bool(fallback)), 0]], dtype=torch.int64, device=device)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        return row.cpu().numpy()
    out = torch.empty((world, LAYOUT_INTS), dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(out, row, group=group)
    return out.cpu().numpy()


def layout_box(layout):
    """The global crop box from the layout table: min / max over the ranks' boxes."""
    return (int(layout[:, 0].min()), int(layout[:, 1].max()), int(layout[:, 2].min()), int(layout[:, 3].max()))


def assemble_bands(owned, layout, canvas_hw, group=None, out=None):
    """The owned bands of every rank into rank 0's [H, W, 3] canvas: each rank != 0 sends its
    contiguous band to rank 0 (P2P; RCCL over xGMI on device tensors, gloo on CPU ones), rank 0
    receives them all in one batch and places them at their owned columns.  Returns the canvas
    on rank 0 and None elsewhere.  owned: this rank's [H, own_hi - own_lo, 3] uint8 band."""
    import torch
    import torch.distributed as dist
    H, W = canvas_hw
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if world > 1 else 0
    root = _root(group) if world > 1 else 0
    if rank != 0:
        if owned.numel():
            _p2p([(dist.isend, owned.contiguous(), root)], group)
        return None
    canvas = out if out is not None else torch.empty((H, W, 3), dtype=torch.uint8, device=owned.device)
    lo0, hi0 = int(layout[0, 4]), int(layout[0, 5])
    canvas[:, lo0:hi0].copy_(owned)
    ops, tmps = [], []
    for r in range(1, world):
        lo, hi = int(layout[r, 4]), int(layout[r, 5])
        if hi <= lo:
            continue
        t = torch.empty((H, hi - lo, 3), dtype=torch.uint8, device=owned.device)
        src = dist.get_global_rank(group, r) if group is not None else r
        ops.append((dist.irecv, t, src))
        tmps.append((lo, hi, t))
    _p2p(ops, group)
    for lo, hi, t in tmps:
        canvas[:, lo:hi].copy_(t)
    return canvas


def crop_box(box, H, W, margin):
    """rectangle_crop's rows / columns (image_stitching_sift.py:208-247) from a global box."""
    if box[1] < 0:
        return 0, H - 1, 0, W - 1
    return max(0, box[0] + margin), min(H - 1, box[1] - margin), box[2], box[3]


def fold_on_root(stitcher, cyl, colnz, recs, pair_counts, margin=15, group=None):
    """The fallback of a sharded step whose bands are not independent: every rank sends its
    cylindrical frames (all but its first, which the previous rank holds) to rank 0, which
    composites the whole sequence with the host plan (the sequential fold where three frames
    cover a column, exactly like Stitcher.run's own fallback).  Returns the StitchResult on
    rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist
    st = stitcher
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if rank != 0:
        if cyl.shape[0] > 1:
            _p2p([(dist.isend, cyl[1:].contiguous(), _root(group)),
                  (dist.isend, colnz[1:].contiguous(), _root(group))], group)
        return None
    parts_c, parts_z, ops = [cyl], [colnz], []
    for r in range(1, world):
        c = int(pair_counts[r])
        if c == 0:
            continue
        tc = torch.empty((c,) + tuple(cyl.shape[1:]), dtype=cyl.dtype, device=cyl.device)
        tz = torch.empty((c,) + tuple(colnz.shape[1:]), dtype=colnz.dtype, device=colnz.device)
        src = dist.get_global_rank(group, r) if group is not None else r
        ops += [(dist.irecv, tc, src), (dist.irecv, tz, src)]
        parts_c.append(tc)
        parts_z.append(tz)
    _p2p(ops, group)
    cyl_all = torch.cat(parts_c).contiguous()
    colnz_all = torch.cat(parts_z).contiguous()
    return st._finish(cyl_all, colnz_all, recs, margin, False, {}, time.perf_counter())


def run_rank(stitcher, frames_dev, focals, pair_start, pair_counts, group=None, margin=15,
             graph=False):
    """One rank's share of a sharded stitch (frames_dev = its pair range + boundary frame):
    the single-GPU launch chain (rank_records, rank_band: device planning, one host read)
    split around ONE all_gather of the 64-byte pair records, plus the crop box's 4-int
    all_reduce.  At world 1 it is Stitcher.run's device-planned stitch over the whole canvas.

    Returns dict(records=global PAIR_NP, band=device canvas of the owned band,
    bbox=global crop box (y0, y1, x0, x1), x_offset=band's first column in the final canvas,
    canvas_hw, and on rank 0 panorama / canvas: the cropped panorama and the whole canvas,
    assembled from every rank's band (None on the other ranks))."""
    import torch
    import torch.distributed as dist
    st = stitcher
    st.last_graphs = []
    st._graph_mode = graph
    pmax = max(pair_counts)
    block, cyl, colnz = rank_records(st, frames_dev, focals, pmax, graph)
    gathered = gather_blocks(block, group)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world > 1:
        return _run_rank_sharded(st, cyl, colnz, gathered, pair_start, pair_counts, group, margin, graph)
    try:
        recs, owned, own_lo, (H, W), box = rank_band(st, cyl, colnz, gathered, pair_counts,
                                                     pair_start, margin, graph)
        refused = None
    except BandError as e:
        if world == 1:
            # one rank holds every frame: composite with the host plan, as Stitcher.run does
            # when the device plan refuses (three frames over a column, a canvas above capacity)
            res = st._finish(cyl, colnz, e.records, margin, graph, {}, time.perf_counter())
            return {"records": res.records, "band": res.canvas, "x_offset": 0,
                    "canvas_hw": tuple(res.canvas.shape[:2]), "bbox": res.bbox,
                    "panorama": res.panorama, "canvas": res.canvas}
        refused, recs, owned, own_lo, box = e, e.records, None, 0, NO_BOX
    if world == 1:
        y0, y1, x0, x1 = crop_box(box, H, W, margin)
        canvas = owned                          # the whole canvas is rank 0's band
        pano = canvas if (y0 > y1 or x0 > x1) else canvas[y0:y1 + 1, x0:x1 + 1]
        return {"records": recs, "band": owned, "x_offset": own_lo, "canvas_hw": (H, W),
                "bbox": (y0, y1, x0, x1), "panorama": pano, "canvas": canvas}
    own = (own_lo, own_lo + (owned.shape[1] if owned is not None else 0))
    layout = exchange_layout(box, own, refused is not None, group, device=cyl.device)
    if layout[:, 6].any():
        # some band was refused: every rank saw it in the layout, so all take the fallback
        res = fold_on_root(st, cyl, colnz, recs, pair_counts, margin, group)
        if res is None:
            return {"records": recs, "band": None, "x_offset": 0, "canvas_hw": None, "bbox": None,
                    "panorama": None, "canvas": None}
        return {"records": res.records, "band": res.canvas, "x_offset": 0,
                "canvas_hw": tuple(res.canvas.shape[:2]), "bbox": res.bbox, "panorama": res.panorama,
                "canvas": res.canvas}
    y0, y1, x0, x1 = crop_box(layout_box(layout), H, W, margin)
    canvas = assemble_bands(owned, layout, (H, W), group, out=st._get("full_canvas", (H, W, 3), torch.uint8)
                            if dist.get_rank(group) == 0 else None)
    pano = None
    if canvas is not None:
        pano = canvas if (y0 > y1 or x0 > x1) else canvas[y0:y1 + 1, x0:x1 + 1]
    return {"records": recs, "band": owned, "x_offset": own_lo, "canvas_hw": (H, W),
            "bbox": (y0, y1, x0, x1), "panorama": pano, "canvas": canvas}


def _run_rank_sharded(st, cyl, colnz, gathered, pair_start, pair_counts, group, margin, graph):
    """run_rank at world > 1 with ONE host read per rank: the band segment is launched, its
    layout row (pano_band_layout_row: crop box, owned columns, refusal, plan status) goes
    through an all_gather on the device, and a single pinned read brings back the head
    (records, band, plan header) together with every rank's layout row.  Then the owned bands
    go to rank 0 (P2P), which places and crops them; a refused band anywhere sends every rank
    to the fold on rank 0 instead."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    S = rank_band_launch(st, cyl, colnz, gathered, pair_counts, pair_start, graph)
    lay = torch.empty((world, LAYOUT_INTS), dtype=torch.int64, device=cyl.device)
    all_gather_dev(lay, S["row"], group)
    pin, nhead = S["pin"], S["nhead"]
    st.ctx.check(st.ctx.lib.pano_copy_async(st.ctx.h, _lib._P(pin.data_ptr() + nhead), _lib.ptr(lay),
                                            64 * world))
    torch.cuda.current_stream(st.device).synchronize()            # the one host read
    raw = pin.numpy()
    layout = raw[nhead:nhead + 64 * world].view(np.int64).reshape(world, LAYOUT_INTS).copy()
    if (layout[:, 7] == _lib.PANO_E_NOMATCH).any():
        raise PanoError(_lib.PANO_E_NOMATCH, "a pair has no descriptor match")
    if layout[:, 6].any():
        # some band was refused: every rank sees it in the gathered layout, all take the fallback
        recs = raw[:S["off_bb"]].view(_lib.PAIR_NP).reshape(-1).copy()
        st._check_records(recs)
        res = fold_on_root(st, cyl, colnz, recs, pair_counts, margin, group)
        if res is None:
            return {"records": recs, "band": None, "x_offset": 0, "canvas_hw": None, "bbox": None,
                    "panorama": None, "canvas": None}
        return {"records": res.records, "band": res.canvas, "x_offset": 0,
                "canvas_hw": tuple(res.canvas.shape[:2]), "bbox": res.bbox, "panorama": res.panorama,
                "canvas": res.canvas}
    recs, owned, own_lo, (H, W), _ = rank_band_finish(S, raw[:nhead])
    y0, y1, x0, x1 = crop_box(layout_box(layout), H, W, margin)
    canvas = assemble_bands(owned, layout, (H, W), group, out=st._get("full_canvas", (H, W, 3), torch.uint8)
                            if dist.get_rank(group) == 0 else None)
    pano = None
    if canvas is not None:
        pano = canvas if (y0 > y1 or x0 > x1) else canvas[y0:y1 + 1, x0:x1 + 1]
    return {"records": recs, "band": owned, "x_offset": own_lo, "canvas_hw": (H, W),
            "bbox": (y0, y1, x0, x1), "panorama": pano, "canvas": canvas}

