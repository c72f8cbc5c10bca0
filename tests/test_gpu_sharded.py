"""The N > 1 step end to end on ONE GPU: two (three) ranks as separate processes sharing the
card, over a gloo process group (gloo moves host memory, so distributed.py stages the device
tensors of the record all_gather, the layout all_gather and the band P2P through host copies;
with RCCL the same calls move device memory over xGMI).  Every rank runs
distributed.run_rank on its own pair shard of parrington -- rank_records, the record
all_gather, the band segment with its device layout row, ONE host read, the band P2P to rank
0 -- and rank 0's panorama must be the reference's (golden digest), eager and graph-replayed.
A capacity too small for the bands sends every rank to the fold on rank 0: same panorama.
"""
from __future__ import annotations

import os
import socket

import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q, force_fold):
    import torch
    import torch.distributed as dist
    from conftest import digest, load_json
    from vfx_image_stitching_amd import data
    from vfx_image_stitching_amd import distributed as D
    from vfx_image_stitching_amd.pipeline import Stitcher
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        gold = load_json("sift_parrington.json")
        names, frames, focals, margin = data.load_set("parrington")
        shards = D.shard_ranges(len(frames) - 1, world)
        s0, c = shards[rank]
        counts = [cc for _, cc in shards]
        st = Stitcher("sift")
        if force_fold:
            st.canvas_cap = (600, 700)            # the global plan fits no band: fold on rank 0
        dev = st.upload(frames[s0:s0 + c + 1])
        out = []
        for graph in ((False,) if force_fold else (False, True, True)):
            r = D.run_rank(st, dev, list(focals[s0:s0 + c + 1]), s0, counts, margin=margin, graph=graph)
            ok = None
            if rank == 0:
                ok = digest(r["panorama"].cpu().numpy()) == gold["pano_digest"]
            else:
                assert r["panorama"] is None
            out.append(ok)
        dist.barrier()
        q.put((rank, out, None))
    except Exception as e:                         # reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world,force_fold", [(2, False), (3, False), (2, True)])
def test_sharded_step_on_one_gpu_matches_reference(gpu, world, force_fold):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, force_fold)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for rank, out, err in res:
        assert err is None, f"rank {rank}:\n{err}"
    assert all(res[0][1]), res[0][1]               # rank 0's panorama == the reference's
