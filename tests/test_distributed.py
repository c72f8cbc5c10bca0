"""Multi-GPU host logic on the CPU: pair shards, the record all_gather,
band ownership and the crop-box all_reduce -- world_size 2 over gloo.

The band compositing itself is checked on the GPU (test_gpu_parity.py::test_bands_*).
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

from vfx_image_stitching_amd import _lib
from vfx_image_stitching_amd import distributed as D
from vfx_image_stitching_amd.pipeline import drift_correct


def _plan(gold, h=512, w=384):
    shifts = [tuple(s["move"]) for s in gold["shifts"]]
    pairs = [tuple(tuple(p) for p in s["pair"]) for s in gold["shifts"]]
    steps, first, (H, W) = D.global_plan(drift_correct(shifts), pairs, len(shifts) + 1, h, w)
    return steps, first, H, W


@pytest.mark.parametrize("n_pairs,world", [(17, 1), (17, 2), (17, 8), (143, 8), (5, 8), (0, 3)])
def test_shard_ranges_balanced_and_contiguous(n_pairs, world):
    r = D.shard_ranges(n_pairs, world)
    assert len(r) == world
    assert sum(c for _, c in r) == n_pairs
    assert max(c for _, c in r) - min(c for _, c in r) <= 1
    pos = 0
    for s, c in r:
        assert s == pos
        pos += c
    if (n_pairs, world) == (17, 8):                     # 3,2,2,2,2,2,2,2
        assert [c for _, c in r] == [3, 2, 2, 2, 2, 2, 2, 2]


def _last_frame_per_column(steps, first, w, n, W):
    last = np.full(W, -1)
    for i in range(n):
        x = D.frame_xy(steps, first, i)[0]
        last[x:x + w] = i
    return last


@pytest.mark.parametrize("name", ["sift_parrington.json", "sift_grail.json",
                                  "harris_parrington.json", "harris_grail.json"])
@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_band_ownership_tiles_canvas(gold_json, name, world):
    """Owned column ranges partition [0, W) and each owned column's last covering frame
    and its predecessor are both inside the owning band."""
    gold = gold_json(name)
    steps, first, H, W = _plan(gold)
    n = len(steps) + 1
    w = 384
    D.check_bands(steps, first, w)
    last = _last_frame_per_column(steps, first, w, n, W)
    assert (last >= 0).all()
    covered = np.zeros(W, np.int32)
    for s, c in D.shard_ranges(n - 1, world):
        loc, first_loc, x0, bw, (lo, hi) = D.band_plan(steps, first, w, H, s, c, n)
        assert x0 <= lo <= hi <= x0 + bw
        covered[lo:hi] += 1
        seg = last[lo:hi]
        assert ((seg > s) | ((seg == 0) & (s == 0))).all()
        assert (seg <= s + c).all()
        # local plan = global plan shifted by the band origin
        for k in range(c):
            assert loc[k].frame_x + x0 == steps[s + k].frame_x
            assert loc[k].frame_y == steps[s + k].frame_y
    assert (covered == 1).all()


def test_check_bands_refuses_triple_coverage():
    """Small |dx| (< w/2): frames i and i-2 overlap -> band compositing is refused."""
    shifts = [(-100.0, 0.0)] * 4
    pairs = [((10.0, 10.0), (110.0, 10.0))] * 4
    steps, first, _ = D.global_plan(drift_correct(shifts), pairs, 5, 64, 384)
    with pytest.raises(D.BandError):
        D.check_bands(steps, first, 384)


# ---------------------------------------------------------------- gloo world_size 2

def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rec(dx, dy, n):
    r = np.zeros(1, _lib.PAIR_NP)
    r["dx"], r["dy"] = dx, dy
    r["xA"], r["yA"], r["xB"], r["yB"] = 10.0, 20.0, 10.0 - dx, 20.0 - dy
    r["n_matches"], r["votes"], r["status"] = n, n, _lib.PANO_OK
    return r


def _worker(rank, world, port, gold, q, h=512, w=384):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        shifts = [tuple(s["move"]) for s in gold["shifts"]]
        pairs = [s["pair"] for s in gold["shifts"]]
        shards = D.shard_ranges(len(shifts), world)
        s0, c = shards[rank]
        # 1. this rank's records (as pano_pair_shifts would write them) -> one all_gather
        local = np.concatenate([_rec(shifts[s0 + k][0], shifts[s0 + k][1], 100 + s0 + k)
                                for k in range(c)])
        for k in range(c):
            (xa, ya), (xb, yb) = pairs[s0 + k]
            local[k]["xA"], local[k]["yA"], local[k]["xB"], local[k]["yB"] = xa, ya, xb, yb
        t = torch.from_numpy(local.view(np.uint8).reshape(c, 64).copy())
        counts = [cc for _, cc in shards]
        recs = D.gather_records(t, counts)
        # the device path's form: zero-padded [pmax, 64] blocks, one all_gather_into_tensor,
        # compacted by the block layout -- the same global records
        pmax, starts = D.block_layout(counts)
        blk = torch.zeros((pmax, 64), dtype=torch.uint8)
        blk[:c] = t
        comp = D.compact_blocks(D.gather_blocks(blk), counts)
        assert list(starts) == [0] + list(np.cumsum(counts))
        assert np.array_equal(comp.numpy(), recs.view(np.uint8).reshape(-1, 64))
        # 2. every rank replays the same global plan and derives its band
        got_shifts, got_pairs = D.records_to_shifts(recs)
        steps, first, (H, W) = D.global_plan(drift_correct(got_shifts), got_pairs,
                                             len(got_shifts) + 1, h, w)
        D.check_bands(steps, first, w)
        _, _, _, _, (lo, hi) = D.band_plan(steps, first, w, H, s0, c, len(steps) + 1)
        spans = [None] * world
        dist.all_gather_object(spans, (lo, hi))
        # 3. crop box: rank 1 pretends its band is empty
        box = torch.tensor([5 + rank, 400 - rank, lo, hi - 1] if rank == 0 else list(D.NO_BOX),
                           dtype=torch.int64)
        g = D.global_bbox(box)
        q.put((rank, [(float(r["dx"]), float(r["dy"]), int(r["n_matches"])) for r in recs],
               spans, (H, W), g))
    finally:
        dist.destroy_process_group()


def _synthetic_gold(n_frames=144, w=1920, step=1229):
    """Ground-truth records of the synthetic config-5 sequence: dx = -step,
    dy = jitter difference, one true correspondence per pair."""
    from vfx_image_stitching_amd import data
    jit = np.random.default_rng(1).integers(-3, 4, n_frames)
    shifts = []
    for i in range(n_frames - 1):
        dx, dy = -float(step), float(jit[i] - jit[i + 1])
        xa, ya = 300.0, 500.0
        shifts.append({"move": [dx, dy], "pair": [[xa, ya], [xa - dx, ya - dy]]})
    return {"shifts": shifts}


@pytest.mark.parametrize("which", ["parrington", "synthetic_strong"])
def test_gloo_world2_gather_plan_bands_bbox(gold_json, which):
    """parrington: the 17 golden pairs; synthetic_strong: bench.py --scaling strong's shards of
    the 144-frame / 143-pair config-5 batch (72 + 71 pairs), whose bands must tile the whole
    canvas."""
    import torch.multiprocessing as mp
    if which == "parrington":
        gold, hw = gold_json("sift_parrington.json"), (512, 384)
    else:
        gold, hw = _synthetic_gold(), (1080, 1920)
        import bench
        assert [c for _, c in bench.strong_shards("synthetic", 2)] == \
            [c for _, c in D.shard_ranges(len(gold["shifts"]), 2)] == [72, 71]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, gold, q, *hw)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    shifts = [tuple(s["move"]) for s in gold["shifts"]]
    for rank, recs, spans, (H, W), g in out:
        assert [(a, b) for a, b, _ in recs] == [tuple(map(float, s)) for s in shifts]
        assert [n for _, _, n in recs] == list(range(100, 100 + len(shifts)))
        # the two bands tile the canvas exactly
        (l0, h0), (l1, h1) = spans
        assert sorted([l0, h0, l1, h1])[0] == 0 and max(h0, h1) == W
        assert min(h0, h1) == max(l0, l1)
        assert g == (5, 400, spans[0][0], spans[0][1] - 1)
        if which == "synthetic_strong":
            assert W >= 143 * 1229                       # the full 144-frame canvas
    assert out[0][1:] == out[1][1:]                      # identical replay on every rank


# ------------------------------------------------- panorama assembly at N > 1 (gloo, world 2)
def _assemble_worker(rank, world, port, q):
    """Each rank holds only its own band of the parrington canvas (the oracle's fold of the
    reference's golden shifts, cut at the rank's owned columns), exchanges the layout, sends its
    band to rank 0, and rank 0 crops: the panorama must be the reference's, byte for byte."""
    import torch
    import torch.distributed as dist
    from conftest import digest, load_json
    from oracle import stitch as ostitch
    from oracle.cv2_compat import bgr_to_gray_u8
    from vfx_image_stitching_amd import data
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        gold = load_json("sift_parrington.json")
        names, frames, focals, margin = data.load_set("parrington")
        shifts = [tuple(s["move"]) for s in gold["shifts"]]
        pairs = [tuple(tuple(p) for p in s["pair"]) for s in gold["shifts"]]
        h, w = frames.shape[1:3]
        steps, first, (H, W) = D.global_plan(drift_correct(shifts), pairs, len(frames), h, w)
        s0, c = D.shard_ranges(len(shifts), world)[rank]
        _, _, _, _, (lo, hi) = D.band_plan(steps, first, w, H, s0, c, len(frames))
        # this rank's band: the oracle's canvas at the owned columns (the rest is discarded)
        cyl = [ostitch.cylindrical(f, fl) for f, fl in zip(frames, focals)]
        mosaic = ostitch.compose(cyl, ostitch.drift_correct(shifts), pairs)
        assert mosaic.shape[:2] == (H, W)
        band = torch.from_numpy(np.ascontiguousarray(mosaic[:, lo:hi]))
        del mosaic
        ys, xs = np.nonzero(bgr_to_gray_u8(band.numpy()) > 0)
        box = (int(ys.min()), int(ys.max()), int(xs.min()) + lo, int(xs.max()) + lo) if ys.size else D.NO_BOX
        layout = D.exchange_layout(box, (lo, hi), False)
        canvas = D.assemble_bands(band, layout, (H, W))
        if rank == 0:
            y0, y1, x0, x1 = D.crop_box(D.layout_box(layout), H, W, margin)
            pano = canvas[y0:y1 + 1, x0:x1 + 1].numpy()
            q.put((rank, digest(pano), gold["pano_digest"], layout.tolist()))
        else:
            assert canvas is None
            q.put((rank, None, None, layout.tolist()))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_assembles_the_parrington_panorama():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_assemble_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0][1] == out[0][2], "assembled panorama differs from the reference's"
    assert out[0][3] == out[1][3]                               # every rank sees the same layout
    (l0, h0), (l1, h1) = sorted((r[4], r[5]) for r in out[0][3])   # the bands tile [0, W)
    assert l0 == 0 and h0 == l1 and h1 > h0


class _RootStitcher:
    """Stands in for Stitcher on rank 0 of the fallback: records what _finish received."""

    def _finish(self, cyl, colnz, recs, margin, graph, t, t0):
        return (cyl.clone(), colnz.clone(), len(recs), margin)


def _fold_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n_frames = 8
        counts = [c for _, c in D.shard_ranges(n_frames - 1, world)]
        s0 = sum(counts[:rank])
        # frame f is filled with the value f: the root must receive 0 .. n_frames - 1 in order
        fr = torch.arange(s0, s0 + counts[rank] + 1, dtype=torch.uint8)
        cyl = fr[:, None, None, None].expand(-1, 4, 5, 3).contiguous()
        colnz = fr[:, None].expand(-1, 5).contiguous()
        recs = np.zeros(n_frames - 1, _lib.PAIR_NP)
        layout = D.exchange_layout(D.NO_BOX, (0, 0), rank == 1)      # rank 1's band refused
        assert layout[:, 6].tolist() == [0, 1, 0][:world]
        res = D.fold_on_root(_RootStitcher(), cyl, colnz, recs, counts, 15)
        q.put((rank, None if res is None else (res[0][:, 0, 0, 0].tolist(), res[1][:, 0].tolist(),
                                               res[2], res[3])))
    finally:
        dist.destroy_process_group()


def test_gloo_world3_fallback_gathers_frames_to_root():
    """A refused band at world > 1: the layout exchange tells every rank, and the frames go to
    rank 0 in sequence order (each rank's first frame is its predecessor's last) for the
    sequential fold."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fold_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[1][1] is None and out[2][1] is None
    frames, colnz, nrec, margin = out[0][1]
    assert frames == list(range(8)) and colnz == list(range(8)) and nrec == 7 and margin == 15
