#!/usr/bin/env python3
"""Headline benchmark: Mpixels/s stitched, 18-image parrington, SIFT path, MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload parrington|grail|synthetic]
    python bench.py --gpus N ...        (N > 1: starts its own N rank processes, one per GPU)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (the same ranks)

A step = one whole stitch of one rank's sequence, inputs resident in HBM:
cylindrical projection -> SIFT features of every frame -> NN match (exact i8 MFMA) -> RANSAC
-> [N>1: all_gather of per-pair records] -> drift correction + composite plan -> composite
(band) -> crop bounding box [N>1: the band's 8-int layout row all_gathered on the device and
read back with the band head (one host read per rank), every band sent to rank 0 (RCCL P2P
over xGMI), which assembles the canvas and crops the panorama -- inside the timed step].

N = 1 (default): one stitch of the 18 parrington frames (BASELINE config 3, the headline);
the K timed stitches go through pipeline.StitchPool (--contexts, default 4): stitch i on a
private libpano context i % 4 with its own stream, so the device overlaps four stitches; every
stitch completes and is read back, and the last one is checked byte for byte against the
single-context stitch.  One context's run_sequence and synchronous run() over the same K
stitches are reported beside (`single_context_ms_per_step`, `run_ms_per_step`).
N > 1 (default): the north_star's scaling target, the synthetic 144-frame / 143-pair 1080p
batch with its pairs sharded over the ranks (strong scaling; the line
carries the committed N = 1 time of the same batch as `strong_n1_reference`), plus the weak
form as `weak_laps`: rank r stitches the parrington loop from frame 17 r, one panorama of N
laps.  --workload / --scaling choose either form explicitly.

value  = distinct input Mpx of the job / max-over-ranks seconds per step.
roofline: the dominant kernel, timed live with HIP events on the library's stream over the
timed region (libpano pano_prof_*), against its algorithmic bytes (DESIGN.md "Roofline").
cpu_baseline: the oracle (numpy restatement, bit-exact vs the reference) on rank 0 at N=1,
per-frame SIFT on a pool of single-threaded workers (one per host core it may use, <= 16),
the rest on one core; `cores` says how many.
pcie_inclusive: the same stitch with the frames uploaded from and the crop downloaded to
pinned host memory every step (never `value`).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
MFMA_BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (no sparsity)
MFMA_I8_PEAK_TOPS = 5000.0      # dense i8 MFMA: the bf16 cycles at twice the K (MI355X_MICROARCH.md)


def match_dtype(st):
    """The distance GEMM that ran: "i8" (u8 descriptors - 128 into v_mfma_i32_32x32x32_i8,
    the default), "bf16" or "f32"."""
    if st.match == "f32":
        return "f32"
    if st.match == "u8" and os.environ.get("PANO_MATCH_I8", "1") != "0":
        return "i8"
    return "bf16"
MFMA_F32_PEAK_TFLOPS = 157.3    # dense f32 MFMA
F32_VECTOR_PEAK_TFLOPS = 157.3  # MI355X f32 vector peak (v_pk_fma_f32), the blur's arithmetic


PMC_PROFILE_FRAMES = {"parrington": 18, "synthetic": 19}   # frames of the profiled step


def pmc_traffic(kernel, workload, method, n_frames):
    """HBM bytes PER STEP of a kernel class from the newest committed PMC traffic profile
    (tools/pmc_traffic.sh: separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes over the same
    SIFT step -- parrington, or the 19-frame synthetic 1080p one -- corrected per
    profiles/r01_fetch_calibration.txt).  A step of another frame count (the strong-scaling
    batch: 144 frames on one GPU) gets the profile's bytes scaled per frame -- every class
    here moves bytes in proportion to its frames -- and the source says so.  Per step, not per
    launch: the profile's launch count and the bench's need not agree (round 5's line mixed
    them), the step is the unit both count."""
    import glob
    if workload not in ("parrington", "synthetic") or method != "sift":
        return None, None
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_traffic_{workload}.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    c = d.get("classes", {}).get(kernel)
    if not c:
        return None, None
    per_step = c["hbm_bytes_per_step"]
    src = os.path.relpath(files[-1], ROOT)
    prof_frames = d.get("frames", PMC_PROFILE_FRAMES[workload])
    if n_frames != prof_frames:
        per_step *= n_frames / prof_frames
        src += f" (a {prof_frames}-frame step, scaled per frame to {n_frames} frames)"
    return per_step, src


def blur_f32_flops(st, n_frames):
    """Algorithmic f32 flops of the blur class per step: every Gaussian level output is a row
    pass of NT fused multiply-adds and a symmetric column pass of R + 1 fused multiply-adds and
    R pair additions (OpenCV's float32 filter), no tile-halo recompute."""
    import ctypes
    import math
    ctx = st.ctx
    p = st.params
    sig = p.sigma
    base = math.sqrt(max(sig * sig - (2 * p.assumed_blur) ** 2, 0.01))
    k = 2 ** (1.0 / p.num_intervals)
    sig_l = [sig] + [math.sqrt((k * k ** (i - 1) * sig) ** 2 - (k ** (i - 1) * sig) ** 2)
                     for i in range(1, p.num_intervals + 3)]
    buf = (ctypes.c_double * 64)()
    nt = ctypes.c_int()

    def flops_per_px(s):
        ctx.lib.pano_sift_taps(ctypes.c_double(s), buf, ctypes.byref(nt))
        n = nt.value
        r = (n - 1) // 2
        return 2 * n + 2 * (r + 1) + r
    no = ctypes.c_int32()
    hh, ww = ctypes.c_int32(), ctypes.c_int32()
    ctx.lib.pano_sift_level_shape(ctx.h, 0, ctypes.byref(hh), ctypes.byref(ww), ctypes.byref(no))
    fl = flops_per_px(base) * hh.value * ww.value
    for o in range(no.value):
        ctx.lib.pano_sift_level_shape(ctx.h, o, ctypes.byref(hh), ctypes.byref(ww), None)
        for l in range(1, p.num_intervals + 3):
            fl += flops_per_px(sig_l[l]) * hh.value * ww.value
    return fl * n_frames


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default=None, choices=["parrington", "grail", "synthetic"],
                    help="default: parrington at N = 1 (the headline config); at N > 1 the "
                         "north_star's scaling config, the synthetic 144-frame / 143-pair batch")
    ap.add_argument("--method", default="sift", choices=["sift", "harris"])
    ap.add_argument("--roofline-kernel", default="auto")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=0, help="frames of the CPU sample (0 = all)")
    ap.add_argument("--match", default=None, choices=["u8", "bf16", "f32"])
    ap.add_argument("--cap", type=int, default=0, help="keypoint capacity per frame (0 = auto)")
    ap.add_argument("--no-graph", dest="graph", action="store_false",
                    help="launch eagerly instead of replaying captured hipGraphs")
    ap.add_argument("--contexts", type=int, default=4,
                    help="N = 1 pipelined form: stitches dealt over this many private libpano "
                         "contexts (pipeline.StitchPool); 1 = one Stitcher's run_sequence")
    ap.add_argument("--no-pipeline", dest="pipeline", action="store_false",
                    help="N=1 graph mode: time one synchronous run() per step instead of "
                         "Stitcher.run_sequence (two stitches in flight)")
    ap.add_argument("--scaling", default=None, choices=["weak", "strong"],
                    help="weak: a fixed sequence per rank; strong: ONE fixed sequence (the set's "
                         "18 frames, or the synthetic 144-frame / 143-pair batch) whose pairs are "
                         "sharded over the ranks.  Default: weak at N = 1 (one parrington stitch), "
                         "strong at N > 1 (with --workload defaulting to synthetic: SURVEY 8(e))")
    ap.add_argument("--no-weak-laps", dest="weak_laps", action="store_false",
                    help="N > 1: skip the secondary weak-scaling parrington-laps measurement")
    return ap.parse_args()


def resolve_defaults(args, world):
    """N = 1: the headline (parrington, one stitch per step).  N > 1: the north_star's scaling
    target, >= 6x at 8 GPUs on the 144-pair synthetic batch -- the 143 pairs of config 5 sharded
    over the ranks, the panorama assembled on rank 0 inside every step (strong scaling)."""
    if args.workload is None:
        args.workload = "parrington" if world == 1 else "synthetic"
    if args.scaling is None:
        args.scaling = "strong" if (world > 1 and args.workload == "synthetic") else "weak"
    return args


SYNTH_PAIRS_PER_RANK = 18      # config 5: 8 ranks x 18 pairs ~ the 143-pair 144-frame loop


def synthetic_shards(world):
    """Pair ranges of the synthetic 144-frame sequence: 18 pairs per rank (weak scaling),
    the 143 pairs of SURVEY 8(d) config 5 at 8 ranks."""
    from vfx_image_stitching_amd import distributed as D
    return D.shard_ranges(min(143, SYNTH_PAIRS_PER_RANK * world), world)


SYNTH_FRAMES = 144             # config 5: the 144-frame synthetic batch, 143 stitched pairs


def strong_shards(name, world):
    """Strong scaling: the pairs of ONE fixed sequence over the ranks (contiguous, balanced;
    grail / parrington 17 pairs over 8 ranks = 3,2,...,2; synthetic 143 over 8 = 18 x 7 + 17)."""
    from vfx_image_stitching_amd import distributed as D
    n_pairs = SYNTH_FRAMES - 1 if name == "synthetic" else 17
    return D.shard_ranges(n_pairs, world)


def workload(name, rank, world, scaling="weak"):
    """-> (this rank's frames, focals, crop margin, (h, w), distinct frames of the job,
    per-rank pair counts).  Rank r holds the frames of its pairs plus the boundary frame."""
    from vfx_image_stitching_amd import data
    if scaling == "strong":
        shards = strong_shards(name, world)
        s, c = shards[rank]
        counts = [cc for _, cc in shards]
        if name == "synthetic":
            frames, focals, _ = data.synthetic_sequence(n_frames=SYNTH_FRAMES, h=1080, w=1920,
                                                        start=s, count=c + 1)
            return frames, focals, 15, (1080, 1920), SYNTH_FRAMES, counts
        names, frames, focals, margin = data.load_set(name)
        return frames[s:s + c + 1], focals[s:s + c + 1], margin, frames.shape[1:3], len(frames), counts
    if name == "synthetic":
        shards = synthetic_shards(world)
        s, c = shards[rank]
        # each rank generates only its own frames (the generator is window-independent)
        frames, focals, _ = data.synthetic_sequence(n_frames=SYNTH_FRAMES, h=1080, w=1920, start=s,
                                                    count=c + 1)
        counts = [cc for _, cc in shards]
        return frames, focals, 15, (1080, 1920), sum(counts) + 1, counts
    names, frames, focals, margin = data.load_set(name)
    n = len(frames)
    fr, fo = data.cyclic_sequence(frames, focals, start=(n - 1) * rank, count=n)
    return fr, fo, margin, frames.shape[1:3], world * (n - 1) + 1, [n - 1] * world


def kernel_bytes(name, st, n_frames, h, w):
    """Algorithmic HBM bytes of all launches of one kernel class in one step."""
    ctx = st.ctx
    import ctypes
    if name == "blur_level":
        # 3 P + 32 sum(Po) bytes per frame (gray in, 3 kept Gaussian
        # levels + 5 DoG per octave out); the class covers gray_frames, blur_fast, blur_tail
        no = ctypes.c_int32()
        hh, ww = ctypes.c_int32(), ctypes.c_int32()
        ctx.lib.pano_sift_level_shape(ctx.h, 0, ctypes.byref(hh), ctypes.byref(ww), ctypes.byref(no))
        spo = 0
        for o in range(no.value):
            ctx.lib.pano_sift_level_shape(ctx.h, o, ctypes.byref(hh), ctypes.byref(ww), None)
            spo += hh.value * ww.value
        return n_frames * (3 * h * w + 32 * spo), "GB/s"
    if name == "composite_step":
        return 9 * n_frames * h * w, "GB/s"
    if name in ("cyl_scatter", "cyl_gather"):
        return 6 * n_frames * h * w, "GB/s"
    if name in ("descriptor", "orientation"):
        # SURVEY 8(d) "S7+S9 upper bound": 12 sum(Po) bytes per frame (the three Gaussian
        # layers keypoints live on, read once); both classes are bounded by it
        tot = 0
        no = ctypes.c_int32()
        hh, ww = ctypes.c_int32(), ctypes.c_int32()
        ctx.lib.pano_sift_level_shape(ctx.h, 0, ctypes.byref(hh), ctypes.byref(ww), ctypes.byref(no))
        for o in range(no.value):
            ctx.lib.pano_sift_level_shape(ctx.h, o, ctypes.byref(hh), ctypes.byref(ww), None)
            tot += 12 * n_frames * hh.value * ww.value
        return tot, "GB/s"
    if name == "extrema_localize":
        tot = 0
        no = ctypes.c_int32()
        hh, ww = ctypes.c_int32(), ctypes.c_int32()
        ctx.lib.pano_sift_level_shape(ctx.h, 0, ctypes.byref(hh), ctypes.byref(ww), ctypes.byref(no))
        for o in range(no.value):
            ctx.lib.pano_sift_level_shape(ctx.h, o, ctypes.byref(hh), ctypes.byref(ww), None)
            tot += 20 * n_frames * hh.value * ww.value
        return tot, "GB/s"
    return None, None


def progress(msg):
    """One progress line on stderr (long runs: a line every phase, never on stdout, which holds
    only the JSON result)."""
    print(f"[bench rank {os.environ.get('RANK', '0')} {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """`python bench.py --gpus N` with no launcher: start N rank processes of this same command
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as torch.distributed.run would, rendezvous on
    127.0.0.1), wait for all of them and return the worst exit status.  Runs before anything in
    this process touches the GPU (children are started, never exec'd); rank 0 prints the line."""
    import subprocess
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port, HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        raise SystemExit(spawn_ranks(args.gpus))
    if os.environ.get("PANO_BENCH_SPAWN_PROBE") == "1":
        # tests/test_bench_spawn.py: what a spawned rank was given, before any GPU work
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE",
                                                         "MASTER_ADDR", "MASTER_PORT")}), flush=True)
        return
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # rehearsal of the N > 1 path on a one-GPU box (tests only, never a reported line): every
    # rank on cuda:0 over gloo (PANO_BENCH_REHEARSE=1); the real run is one rank per GPU, RCCL
    rehearse = os.environ.get("PANO_BENCH_REHEARSE") == "1"
    torch.cuda.set_device(0 if rehearse else local)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    args = resolve_defaults(args, world)

    from vfx_image_stitching_amd import distributed as D
    from vfx_image_stitching_amd.pipeline import Stitcher

    progress(f"workload {args.workload} ({args.scaling}), world {world}")
    frames, focals, margin, (h, w), distinct, counts = workload(args.workload, rank, world, args.scaling)
    n_local = len(frames)
    progress(f"{n_local} frames ready")
    cap = args.cap or (4096 if args.workload != "synthetic" else 65536)
    st = Stitcher(args.method, cap=cap, match=args.match)
    dev = st.upload(frames)                                   # resident in HBM
    pair_start = sum(counts[:rank])

    def step(graph=False):
        if world > 1:
            return D.run_rank(st, dev, focals, pair_start, counts, margin=margin, graph=graph)
        return st.run(dev, focals, margin=margin, graph=graph)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    progress("warm-up done")

    # pick the dominant kernel from one profiled (untimed) step
    ctx = st.ctx
    rk = args.roofline_kernel
    per_kernel = {}
    if rk == "auto":
        # per-class breakdown: one profiled (untimed) step per kernel class
        from vfx_image_stitching_amd._lib import KERNELS
        for k in KERNELS:
            ctx.prof_enable(k)
            step()
            r = ctx.prof_read(k)
            if r["launches"]:
                per_kernel[k] = r
        ctx.prof_enable(-1)
        rk = max(per_kernel, key=lambda k: per_kernel[k]["total_ms"])

    # timed region.  Eager: the dominant kernel's launches are bracketed by HIP events on the
    # library's stream.  hipGraph replay (default): the graphs are captured by an untimed step;
    # ROCm rejects timing events recorded inside graphs (hipErrorInvalidHandle), so the
    # dominant kernel is timed with the same events over K eager steps run right after.
    # N = 1 with graphs: the K stitches go through Stitcher.run_sequence, which launches stitch
    # k + 1 before the host finishes stitch k (every stitch still completes and is read back);
    # the same K stitches as synchronous run() calls are timed beside it (--no-pipeline: the
    # other way round).
    pipelined = world == 1 and args.graph and args.pipeline
    seq_beside = world == 1 and args.graph and not args.pipeline
    pool = None
    if args.graph:
        step(graph=True)
        if pipelined or seq_beside:
            for _ in st.run_sequence([(dev, focals)] * 3, margin=margin):   # both output slots
                pass
        if pipelined and args.contexts > 1 and n_local <= 32:
            # (a large batch -- the 144-frame strong form at N = 1 -- keeps one context: each
            # private context holds its own pyramid, ~70 GB at 144 x 1080p)
            # N = 1: the stitches dealt over private contexts (StitchPool): one stitch's
            # latency-bound stages overlap another's on the device; every member's graphs are
            # captured here, before the timed region
            from vfx_image_stitching_amd.pipeline import StitchPool
            pool = StitchPool(args.method, contexts=args.contexts, cap=cap, match=args.match)
            for _ in pool.run_sequence([(dev, focals)] * (4 * args.contexts + 2), margin=margin):
                pass
        torch.cuda.synchronize()
    else:
        ctx.prof_enable(rk)
        ctx.prof_read(rk)                                      # reset
    progress("timed region")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pool_pano = None
    if pool is not None:
        # the last result's panorama is copied to the host after the timed region (it stays
        # valid: nothing runs on its member afterwards); the first pageable device -> host copy
        # of a process pays ~50 ms of HIP staging setup, which is not the stitch's
        for r in pool.run_sequence([(dev, focals)] * args.steps, margin=margin):
            pool_pano = r.panorama
    elif pipelined:
        for _ in st.run_sequence([(dev, focals)] * args.steps, margin=margin):
            pass
    else:
        for _ in range(args.steps):
            step(graph=args.graph)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    ms_other = None
    if pipelined or seq_beside:
        # the same K stitches in the other form, for the record (not `value`)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if pipelined:
            for _ in range(args.steps):
                step(graph=True)
        else:
            for _ in st.run_sequence([(dev, focals)] * args.steps, margin=margin):
                pass
        torch.cuda.synchronize()
        ms_other = (time.perf_counter() - t1) / args.steps * 1e3
    ms_single = None
    if pool is not None:
        # one context's run_sequence over the same K stitches, for the record (not `value`)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in st.run_sequence([(dev, focals)] * args.steps, margin=margin):
            pass
        torch.cuda.synchronize()
        ms_single = (time.perf_counter() - t1) / args.steps * 1e3
    if args.graph:
        ctx.prof_enable(rk)
        ctx.prof_read(rk)
        for _ in range(args.steps):
            step()
    kr = ctx.prof_read(rk)
    ctx.prof_enable(-1)
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    ms_step = el / args.steps * 1e3
    mpx = distinct * h * w / 1e6
    progress(f"timed: {ms_step:.4f} ms per step; side measurements")
    value = mpx / (el / args.steps)

    # SURVEY 8(d) "wall": decoded uint8 frames on the host -> cropped uint8 panorama on the
    # host.  Same stitch, plus a pinned-host upload of the frames and a pinned-host download
    # of the cropped panorama inside every step (N = 1; reported beside `value`, never as it)
    pcie = jpg = None
    if world == 1:
        pcie = pcie_inclusive(st, frames, dev, focals, margin, args.steps, args.graph, mpx, pool)
        if args.workload in ("parrington", "grail") and args.scaling == "weak":
            jpg = jpeg_inclusive(st, args.workload, dev, focals, margin, args.steps, args.graph, mpx)

    roof = None
    byts, unit = kernel_bytes(rk, st, n_local, h, w)
    if kr["launches"]:
        per_step_ms = kr["total_ms"] / args.steps
        per_launch_ms = kr["total_ms"] / kr["launches"]
        launches_per_step = kr["launches"] / args.steps
        if byts is not None:
            per_launch_bytes = byts / launches_per_step
            ach = per_launch_bytes / (per_launch_ms * 1e-3) / 1e9
            traffic_step, tsrc = pmc_traffic(rk, args.workload, args.method, n_local)
            roof = {"bound": "hbm", "kernel": rk, "achieved": round(ach, 2), "peak": HBM_PEAK_GBS,
                    "timing": ("HIP events on the library stream, %d eager steps right after the "
                               "graph-replayed timed region" % args.steps) if args.graph
                    else "HIP events on the library stream over the timed region",
                    "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5),
                    "traffic": round(traffic_step / launches_per_step) if traffic_step else None,
                    "traffic_unit": "HBM bytes per launch (the PMC step's bytes / this step's launches)",
                    "traffic_per_step": round(traffic_step) if traffic_step else None,
                    "algorithmic_bytes_per_step": round(byts),
                    "traffic_over_algorithmic": round(traffic_step / byts, 3) if traffic_step else None,
                    "traffic_source": tsrc,
                    "algorithmic_bytes_per_launch": round(per_launch_bytes),
                    "avg_launch_ms": round(per_launch_ms, 5), "launches_per_step": launches_per_step,
                    "kernel_ms_per_step": round(per_step_ms, 4)}
            if rk == "blur_level" and args.method == "sift":
                fl = blur_f32_flops(st, n_local)
                tf = fl / (per_step_ms * 1e-3) / 1e12
                roof["f32_vector"] = {"note": "the blur's arithmetic: OpenCV's float32 FMA filter "
                                              "(DESIGN.md 4), its compute roofline",
                                      "achieved": round(tf, 2), "peak": F32_VECTOR_PEAK_TFLOPS,
                                      "unit": "TFLOP/s", "frac": round(tf / F32_VECTOR_PEAK_TFLOPS, 4)}
        else:
            roof = {"bound": "latency", "kernel": rk, "achieved": None, "peak": None, "unit": None,
                    "frac": None, "traffic": None, "avg_launch_ms": round(per_launch_ms, 5),
                    "launches_per_step": launches_per_step,
                    "kernel_ms_per_step": round(per_step_ms, 4)}

    # the one dense contraction (M1): the descriptor distance GEMM against the MFMA peak of
    # its input type.  Algorithmic flops = sum over pairs of 2 N_A N_B 128 with the actual
    # keypoint counts (tile padding not counted); time from the profiled eager step above.
    roof_match = None
    if args.method == "sift" and "dist_mfma" in per_kernel and per_kernel["dist_mfma"]["launches"]:
        cnt = st._buf["counts"].cpu().numpy().astype(np.float64)
        pairs = [(i, i + 1) for i in range(len(cnt) - 1)]
        fl = sum(2.0 * cnt[a] * cnt[b] * 128 for a, b in pairs)
        ms = per_kernel["dist_mfma"]["total_ms"]
        mdt = match_dtype(st)
        pk = {"f32": MFMA_F32_PEAK_TFLOPS, "bf16": MFMA_BF16_PEAK_TFLOPS, "i8": MFMA_I8_PEAK_TOPS}[mdt]
        tf = fl / (ms * 1e-3) / 1e12
        roof_match = {"bound": "mfma", "kernel": "dist_mfma", "dtype": mdt, "descriptors": st.match,
                      "achieved": round(tf, 2), "peak": pk, "unit": "TOPS" if mdt == "i8" else "TFLOP/s",
                      "frac": round(tf / pk, 5), "frac_of_bf16_peak": round(tf / MFMA_BF16_PEAK_TFLOPS, 5),
                      "flop_per_step": fl,
                      "mean_keypoints": round(float(cnt.mean()), 1),
                      "kernel_ms_per_step": round(ms, 4)}

    # SURVEY 8(d)'s whole-path roofline fraction: (sum of algorithmic bytes / 8.0 TB/s + the M1
    # flops / MFMA peak) / measured wall, bytes = 18 P + 64 sum(Po) per frame (C1, S1-S5, S7+S9,
    # B1), flops = sum over pairs of 2 N_A N_B 128 with the actual keypoint counts.  `frac`
    # prices the GEMM at the peak of the dtype it runs in (i8 MFMA, exact here); SURVEY's
    # formula prices it at the f32 MFMA peak (157.3 TF), carried as frac_survey_f32 -- above 1
    # where the exact i8 GEMM beats that floor outright (1080p).
    roof_path = None
    if args.method == "sift" and "blur_level" in per_kernel:
        spo_b, _ = kernel_bytes("extrema_localize", st, n_local, h, w)      # 20 sum(Po) n
        path_bytes = 18.0 * n_local * h * w + 64.0 * spo_b / 20.0
        fl = roof_match["flop_per_step"] if roof_match else 0.0
        mdt = match_dtype(st)
        pk = {"f32": MFMA_F32_PEAK_TFLOPS, "bf16": MFMA_BF16_PEAK_TFLOPS, "i8": MFMA_I8_PEAK_TOPS}[mdt]
        t_bytes = path_bytes / (HBM_PEAK_GBS * 1e9)
        wall = ms_step * 1e-3
        roof_path = {"formula": "SURVEY 8(d): (bytes / 8.0 TB/s + M1 flop / MFMA peak) / wall",
                     "bytes_per_step": round(path_bytes), "flop_per_step": fl, "gemm_dtype": mdt,
                     "floor_us": round((t_bytes + fl / (pk * 1e12)) * 1e6, 1),
                     "wall_us": round(wall * 1e6, 1),
                     "frac": round((t_bytes + fl / (pk * 1e12)) / wall, 4),
                     "frac_survey_f32": round((t_bytes + fl / (MFMA_F32_PEAK_TFLOPS * 1e12)) / wall, 4)}

    # correctness of what was timed: the single-GPU panorama against the reference's digest
    parity = None
    if world == 1 and args.workload != "synthetic" and len(frames) == 18:
        parity = check_parity(st, dev, focals, margin, args.workload, args.method, args.graph)
    if pool_pano is not None:
        # the pool's last timed stitch against the single-context stitch, byte for byte
        pool_pano = pool_pano.cpu().numpy()
        ref = st.run(dev, focals, margin=margin, graph=args.graph).panorama.cpu().numpy()
        same = ref.shape == pool_pano.shape and bool((ref == pool_pano).all())
        parity = dict(parity or {}, pool_matches_single_context=same)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if args.workload == "synthetic" and args.method == "sift":
            cpu = cpu_baseline_synthetic(h, w, distinct)
        elif len(frames) == 18:
            cpu = cpu_baseline(frames, focals, args.cpu_frames, args.method, h, w)

    # N > 1 strong: the same batch's N = 1 time from the committed single-GPU line (a different
    # box and run; the driver computes efficiency from its own per-N values), and the weak
    # parrington laps as a secondary measurement
    strong_ref = weak = None
    if world > 1 and args.scaling == "strong":
        strong_ref = strong_n1_reference(args.workload, args.method, ms_step)
    if world > 1 and args.weak_laps and args.method == "sift" and args.scaling == "strong":
        weak = weak_laps_secondary(args, rank, world)

    line = {
        "metric": "Mpixels/s stitched (18-img parrington, SIFT path)" if args.workload == "parrington"
        else f"Mpixels/s stitched ({args.workload}, {args.method})",
        "value": round(value, 3), "unit": "Mpx/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 4),
        "timed_form": (f"StitchPool.run_sequence ({args.contexts} private contexts, items round-robin)"
                       if pool is not None else "run_sequence" if pipelined else "run"),
        "pooled_ms_per_stitch": round(ms_step, 4) if pool is not None else None,
        "pooled_note": ("ms_per_step is the throughput of StitchPool (up to 2 stitches in flight per "
                        "context); single_context_ms_per_step is the one-context figure rounds 1-4 "
                        "reported as ms_per_step") if pool is not None else None,
        "single_context_ms_per_step": round(ms_single, 4) if ms_single is not None else None,
        "run_sequence_ms_per_step" if seq_beside else "run_ms_per_step":
            round(ms_other, 4) if ms_other is not None else None,
        "higher_is_better": True,
        "scaling": args.scaling, "vs_baseline": None,
        "dtype": ("u8 frames; f32 pyramid (OpenCV's float32 FMA blur order); match " +
                  {"f32": "f32 MFMA", "bf16": "bf16 MFMA, exact for integer descriptors",
                   "i8": "i8 MFMA on u8 descriptors - 128, exact integer distances"}[match_dtype(st)]
                  if args.method == "sift" else "u8 frames; f64 Harris response; f32 descriptors"),
        "data": "reference parrington JPEGs (packed under data/), decoded, resident in HBM"
        if args.workload != "synthetic" else "synthetic 1080p sequence (SURVEY 8d config 5)",
        "config": {"workload": f"{args.workload} {args.method} end-to-end: {distinct} frames "
                               f"{h}x{w}, {distinct - 1} pairs, {world} rank(s), this rank {n_local} "
                               f"frames ({args.scaling} scaling)",
                   "frames": distinct, "frame_hw": [h, w], "parallelism": f"pairs sharded x{world}",
                   "method": args.method, "match_gemm": st.match,
                   "assembly": "one canvas on one GPU" if world == 1 else
                   "bands sent to rank 0 (RCCL P2P), canvas assembled and cropped there, in the timed step",
                   "launch": "hipGraph replay" if args.graph else "eager"},
        "roofline": roof,
        "roofline_match": roof_match,
        "roofline_path": roof_path,
        "pcie_inclusive": pcie,
        "jpeg_inclusive": jpg,
        "cpu_baseline": cpu,
        "strong_n1_reference": strong_ref,
        "weak_laps": weak,
        "parity": parity,
        "kernels_ms_per_step": {k: round(v["total_ms"], 4) for k, v in per_kernel.items()},
    }
    if rehearse:
        line["rehearsal"] = ("PANO_BENCH_REHEARSE: every rank on cuda:0 over gloo (host-staged "
                             "exchanges) -- a path check, not a scaling measurement")
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def strong_n1_reference(workload, method, ms_step):
    """The committed N = 1 line of the same strong-scaling batch (profiles/r*_bench_<workload>
    _strong_n1.json, newest round): its ms_per_step and the speedup of this run over it."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_bench_{workload}_strong_n1.json")))
    if not files or method != "sift":
        return None
    try:
        ref = json.loads(open(files[-1]).read().strip().splitlines()[-1])
    except (ValueError, IndexError):
        return None
    n1 = ref.get("ms_per_step")
    if not n1:
        return None
    return {"ms_per_step_n1": n1, "source": os.path.relpath(files[-1], ROOT),
            "speedup": round(n1 / ms_step, 3),
            "note": "N = 1 time of the same batch from a committed single-GPU run (another box); "
                    "the driver computes scaling efficiency from its own per-N values"}


def weak_laps_secondary(args, rank, world):
    """N > 1: the weak-scaling form as a secondary number -- rank r stitches the parrington
    loop starting at frame 17 r, the job is one panorama of N laps assembled on rank 0; K steps,
    max over ranks (the same timing rules as the main line)."""
    import torch
    import torch.distributed as dist

    from vfx_image_stitching_amd import distributed as D
    from vfx_image_stitching_amd.pipeline import Stitcher
    frames, focals, margin, (h, w), distinct, counts = workload("parrington", rank, world, "weak")
    st = Stitcher("sift", cap=4096)
    dev = st.upload(frames)
    pair_start = sum(counts[:rank])

    def step(graph):
        return D.run_rank(st, dev, focals, pair_start, counts, margin=margin, graph=graph)
    for _ in range(max(1, args.warmup)):
        step(False)
    step(True)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    dist.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    mpx = distinct * h * w / 1e6
    return {"metric": "Mpixels/s stitched (parrington laps, weak scaling)", "unit": "Mpx/s",
            "value": round(mpx / (el / args.steps), 3), "ms_per_step": round(el / args.steps * 1e3, 4),
            "frames": distinct, "steps": args.steps, "scaling": "weak",
            "note": "rank r stitches the parrington loop from frame 17 r; one panorama of N laps "
                    "assembled on rank 0 per step"}


def pcie_inclusive(st, frames, dev, focals, margin, steps, graph, mpx, pool=None):
    """Host-to-host stitch rate: per step, the uint8 frames go pinned host -> HBM (into the
    resident input buffer), the stitch runs, and the crop's canvas rows come back to pinned
    host memory in one contiguous copy (the panorama is a view of them, as the device result
    is a view of the canvas); steps bracketed by synchronize like the timed region.  The H2D
    and D2H legs are also timed alone (HIP events) so a slow PCIe path shows as such."""
    import torch
    host_in = torch.from_numpy(np.ascontiguousarray(frames)).pin_memory()
    res = st.run(dev, focals, margin=margin, graph=graph)
    host_out = torch.empty(res.canvas.numel(), dtype=torch.uint8).pin_memory()

    def rows_of(res):
        """The canvas rows holding the crop, as one contiguous device range (flat uint8)."""
        pano = res.panorama
        base = res.canvas.reshape(-1)
        row = res.canvas.stride(0)
        first = (pano.storage_offset() - res.canvas.storage_offset()) // row
        return base[first * row:(first + pano.shape[0]) * row], pano

    flat, pano = rows_of(res)
    cur = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record(cur)
    dev.copy_(host_in, non_blocking=True)
    ev[1].record(cur)
    host_out[:flat.numel()].copy_(flat, non_blocking=True)
    ev[2].record(cur)
    torch.cuda.synchronize()
    h2d_ms, d2h_ms = ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])
    t0 = time.perf_counter()
    for _ in range(steps):
        dev.copy_(host_in, non_blocking=True)
        flat, pano = rows_of(st.run(dev, focals, margin=margin, graph=graph))
        host_out[:flat.numel()].copy_(flat, non_blocking=True)
        cur.synchronize()
    el = (time.perf_counter() - t0) / steps
    out = {"value": round(mpx / el, 3), "unit": "Mpx/s", "ms_per_step": round(el * 1e3, 4),
           "includes": "pinned H2D of the uint8 frames + stitch + pinned D2H of the crop's canvas "
                       "rows, per step (SURVEY 8(d) wall, JPEG I/O excluded)",
           "h2d_ms": round(h2d_ms, 4), "d2h_ms": round(d2h_ms, 4),
           "bytes_h2d": int(host_in.numel()), "bytes_d2h": int(flat.numel()),
           "panorama_bytes": int(pano.numel())}
    if pool is not None:
        # the same host-to-host stitches through the pool: each item's frames go pinned host ->
        # its member's staging buffer and its panorama -> pinned host on that member's stream,
        # so one member's PCIe legs overlap the other members' stitches (StitchPool.run_sequence
        # to_host); the last panorama is checked byte for byte against the device one
        ref = np.ascontiguousarray(pano.cpu().numpy())
        # every member's two output slots capture their graphs on the staging buffers first
        for _ in pool.run_sequence([(host_in, focals)] * (4 * len(pool.members) + 2), margin=margin, to_host=True):
            pass
        torch.cuda.synchronize()
        last = None
        t0 = time.perf_counter()
        for r in pool.run_sequence([(host_in, focals)] * steps, margin=margin, to_host=True):
            last = r.host
        torch.cuda.synchronize()
        el_p = (time.perf_counter() - t0) / steps
        out["pooled"] = {"value": round(mpx / el_p, 3), "unit": "Mpx/s", "ms_per_step": round(el_p * 1e3, 4),
                         "form": f"StitchPool.run_sequence(to_host=True), {len(pool.members)} contexts: "
                                 "per stitch pinned H2D of the frames and pinned D2H of the panorama "
                                 "on the member's stream, overlapping the other members' stitches",
                         "host_panorama_equals_device": bool(last is not None and last.shape == ref.shape
                                                             and (last == ref).all())}
    return out


def jpeg_inclusive(st, name, dev, focals, margin, steps, graph, mpx):
    """File-to-file rate: per step the frames' JPEG files (host bytes, the
    reference's cv2.imread input, image_stitching_sift.py:282) are decoded on the GPU straight
    into the resident frame buffer (pano_jpeg_decode: headers parsed on the host, entropy bytes
    uploaded once), the stitch runs, and the cropped panorama is encoded on the GPU into its
    JPEG file bytes (pano_jpeg_encode, cv2.imwrite at quality 95, :386).  The decode and the
    encode are also timed alone, with PIL's host decode / encode of the same data (what the
    harness otherwise runs, one core) beside them; the GPU decode must equal the resident
    PIL-decoded frames and the GPU file must equal PIL's q95 file byte for byte."""
    import io

    import torch
    from PIL import Image

    from vfx_image_stitching_amd import data, jpeg
    names, bufs = data.load_set_jpegs(name)
    if len(bufs) != dev.shape[0]:
        return None
    ref = dev.clone()
    out, st_ = jpeg.decode_batch(bufs, out=dev, status=True)
    dec_exact = bool(torch.equal(dev, ref)) and not bool(st_.any())
    sync = jpeg.last_stats(len(bufs))
    res = st.run(dev, focals, margin=margin, graph=graph)
    pano = res.panorama
    file_gpu = jpeg.encode(pano)
    pano_h = np.ascontiguousarray(pano.cpu().numpy())
    b = io.BytesIO()
    Image.fromarray(np.ascontiguousarray(pano_h[..., ::-1])).save(b, "JPEG", quality=95)
    enc_exact = file_gpu == b.getvalue()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        jpeg.decode_batch(bufs, out=dev, status=True)
    torch.cuda.synchronize()
    dec_ms = (time.perf_counter() - t0) / steps * 1e3
    t0 = time.perf_counter()
    for _ in range(steps):
        jpeg.encode(pano)
    enc_ms = (time.perf_counter() - t0) / steps * 1e3
    reps = max(1, steps // 4)
    t0 = time.perf_counter()
    for _ in range(reps):
        for bb in bufs:
            data.decode_jpeg(bb)
    pil_dec_ms = (time.perf_counter() - t0) / reps * 1e3
    t0 = time.perf_counter()
    for _ in range(reps):
        Image.fromarray(np.ascontiguousarray(pano_h[..., ::-1])).save(io.BytesIO(), "JPEG", quality=95)
    pil_enc_ms = (time.perf_counter() - t0) / reps * 1e3
    t0 = time.perf_counter()
    for _ in range(steps):
        jpeg.decode_batch(bufs, out=dev, status=True)
        r = st.run(dev, focals, margin=margin, graph=graph)
        jpeg.encode(r.panorama)
    el = (time.perf_counter() - t0) / steps
    return {"value": round(mpx / el, 3), "unit": "Mpx/s", "ms_per_step": round(el * 1e3, 4),
            "includes": "GPU decode of the frames' JPEG files (host bytes) + stitch + GPU encode of the "
                        "cropped panorama into its q95 JPEG file (host bytes), per step",
            "decode_ms": round(dec_ms, 4), "encode_ms": round(enc_ms, 4),
            "decode_bit_exact_vs_pil": dec_exact, "encode_bytes_equal_pil_q95": enc_exact,
            "jpeg_bytes_in": int(sum(len(x) for x in bufs)), "jpeg_bytes_out": len(file_gpu),
            "decode_sync": {"subsequences": int(sync[:, 0].sum()), "fix_candidates": int(sync[:, 1].sum()),
                            "serial_decodes": int(sync[:, 2].sum())},
            "pil_host_decode_ms": round(pil_dec_ms, 3), "pil_host_encode_ms": round(pil_enc_ms, 3),
            "pil_cores": 1}


def check_parity(st, dev, focals, margin, workload, method, graph):
    """Panorama of the benchmarked sequence vs the reference's (tests/golden digest), and its
    PSNR against the author's published panorama (real OpenCV; quality.compare_published)."""
    import hashlib
    path = os.path.join(ROOT, "tests", "golden", f"{method}_{workload}.json")
    if not os.path.exists(path):
        return None
    gold = json.load(open(path))
    pano = np.ascontiguousarray(st.run(dev, focals, margin=margin, graph=graph).panorama.cpu().numpy())
    h = hashlib.sha256()
    h.update(f"{pano.dtype.str}{pano.shape}".encode())
    h.update(pano.tobytes())
    ok = h.hexdigest() == gold["pano_digest"]
    out = {"panorama_bit_exact_vs_reference": ok, "shape": list(pano.shape),
           "psnr_db_vs_reference_run": "inf" if ok else None,
           "reference_run": "the reference's Python in the build container, OpenCV blur restated "
                            "(tests/golden/make_golden.py)"}
    pub = {"parrington": "sift_prtn_result.jpg", "grail": "sift_grail_result.jpg"}.get(workload)
    ppath = os.path.join(ROOT, "tests", "golden", "published", pub or "-")
    if method == "sift" and pub and os.path.exists(ppath):
        from vfx_image_stitching_amd import quality
        with open(ppath, "rb") as f:
            rep = quality.compare_published(pano, quality.decode_jpeg(f.read()))
        rep["published"] = f"reference Result/{pub} (real OpenCV, cv2.imwrite q95); ours q95 re-encoded"
        out["vs_published"] = rep
    return out


def _oracle_features(args):
    """Worker of cpu_baseline: the oracle's cylindrical projection + SIFT/Harris of one frame
    on one thread (spawned process; numpy single-threaded)."""
    frame, focal, method = args
    from threadpoolctl import threadpool_limits
    from oracle import harris as oharris
    from oracle import sift as osift
    from oracle import stitch as ostitch
    with threadpool_limits(1):
        cyl = ostitch.cylindrical(frame, focal)
        return osift.detect_and_describe(cyl) if method == "sift" else oharris.detect_and_describe(cyl)


def _warm_worker():
    """Pool initializer: every worker imports numpy / the oracle and loads its C blur before
    the timed region (first imports would otherwise land inside it)."""
    from oracle import cv2_compat, harris, sift, stitch  # noqa: F401
    from threadpoolctl import threadpool_limits  # noqa: F401
    cv2_compat._cv_blur_lib()


def _ready(_):
    time.sleep(0.2)                    # one short task per worker: all are up before t0
    return os.getpid()


def cpu_cores():
    """Host cores this process may use, capped at the box's CPU share (16)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:                                     # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(frames, focals, n, method, h, w):
    """The oracle (numpy restatement, bit-exact vs the reference) stitching the benchmarked
    sequence on the host cores: per-frame features in a process pool (one single-threaded
    worker per core, as the frames are independent), then matching, RANSAC, drift and the
    blend fold in this process.  n = frames of the sample (default: the whole sequence)."""
    import multiprocessing as mp
    from oracle import stitch as ostitch
    n = len(frames) if n <= 0 else min(n, len(frames))
    cores = cpu_cores()
    ctx = mp.get_context("spawn")                              # no fork of a HIP process
    k = min(cores, n)
    with ctx.Pool(k, initializer=_warm_worker) as pool:
        pool.map(_ready, range(k), chunksize=1)                              # every worker warm
        pool.map(_oracle_features, [(frames[0], focals[0], method)])        # numpy kernels warm
        t0 = time.perf_counter()
        feats = pool.map(_oracle_features, [(frames[i], focals[i], method) for i in range(n)])
        ostitch.stitch(list(frames[:n]), list(focals[:n]), method=method, margin=15, features=feats)
        el = time.perf_counter() - t0
    mpx = n * h * w / 1e6
    return {"value": round(mpx / el, 5), "unit": "Mpx/s", "cores": min(cores, n), "kind": "port",
            "sample": f"oracle end-to-end stitch of {n} frames ({n - 1} pairs): features in "
                      f"{min(cores, n)} single-threaded processes, the rest on one; {el:.1f} s",
            "reference_container_value": 0.00448,
            "reference_container_note": "the reference's own sift path, single-threaded, "
                                        "re-measured in the build container: 789.35 s for 18 "
                                        "frames (BASELINE.md)"}


def cpu_baseline_synthetic(h, w, n_frames_job):
    """the reference would need ~25 min per 1080p frame and ~50 min of NN
    loop per pair, so the oracle (bit-exact restatement, tests/test_oracle.py) runs ONE seeded
    pair -- frames 0 and 1 of the synthetic sequence: cylindrical + SIFT of both frames in two
    single-threaded processes, then the NN match and RANSAC on one core -- and the job time is
    that pair's wall time x the job's pairs (the reference computes a pair's two frames for
    every pair, image_stitching_sift.py:59-60), stated as extrapolated."""
    import multiprocessing as mp
    from threadpoolctl import threadpool_limits
    from oracle import stitch as ostitch
    from vfx_image_stitching_amd import data
    frames, focals, _ = data.synthetic_sequence(n_frames=SYNTH_FRAMES, h=h, w=w, start=0, count=2)
    ctx = mp.get_context("spawn")
    with ctx.Pool(2, initializer=_warm_worker) as pool:
        pool.map(_ready, range(2), chunksize=1)
        t0 = time.perf_counter()
        feats = pool.map(_oracle_features, [(frames[i], focals[i], "sift") for i in range(2)], chunksize=1)
        t1 = time.perf_counter()
        with threadpool_limits(1):
            (dx, dy), _ = ostitch.pair_shift_sift(*feats[0], *feats[1])
        el = time.perf_counter() - t0
    pairs = n_frames_job - 1
    job_s = el * pairs
    return {"value": round(n_frames_job * h * w / 1e6 / job_s, 6), "unit": "Mpx/s", "cores": 2,
            "kind": "port", "extrapolated": True,
            "sample": f"oracle on ONE seeded pair (config 5 frames 0, 1; {len(feats[0][0])} + "
                      f"{len(feats[1][0])} keypoints): features of both frames in 2 single-threaded "
                      f"processes ({t1 - t0:.1f} s), NN match + RANSAC on one core ({el - (t1 - t0):.1f} s); "
                      f"{el:.1f} s per pair x {pairs} pairs = {job_s:.0f} s extrapolated for the "
                      f"{n_frames_job}-frame job",
            "per_pair_s": round(el, 3), "pair_shift": [round(dx, 4), round(dy, 4)]}


if __name__ == "__main__":
    main()
