"""BASELINE config 5 at its stated size: the 144-frame / 143-pair synthetic 1080p batch
(SURVEY.md 8(d) "Config 5 generator"; the reference's per-pair loop,
/root/reference/image_stitching_sift.py:52-111) on ONE GPU, as ``bench.py --workload synthetic
--scaling strong`` times it, checked against:

* the generator's ground truth on every pair: dx = -1229 (the strip step), dy = the jitter
  difference, each within 1.5 px -- size-independent properties of the sequence;
* the oracle's golden for pairs 0 and 1 (tests/golden/synthetic_1080p.json) and for pairs 35,
  71, 107 and 142 (synthetic_1080p_spread.json), the oracle being pinned bit-exactly to the
  reference at the reference's own sizes: ransac move and match count at the bars of
  test_synthetic_1080p_vs_oracle_golden;
* the sharded form: each of the 8 strong-scaling shards (tools of distributed.py, what a rank
  runs before the record gather) gives byte-identical records to the matching slice of the
  whole-batch records.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_FRAMES, H, W, STEP = 144, 1080, 1920, 1229


@pytest.fixture(scope="module")
def batch(gpu):
    from vfx_image_stitching_amd import data
    from vfx_image_stitching_amd.pipeline import Stitcher
    frames, focals, jit = data.synthetic_sequence(n_frames=N_FRAMES, h=H, w=W)
    st = Stitcher("sift", cap=65536)
    dev = st.upload(frames)
    del frames
    res = st.run(dev, focals, margin=15)
    yield st, dev, focals, jit, res
    st.release_graphs()
    del dev, res
    # the shared context's scratch grew to the 144-frame 1080p pyramid (~70 GB): give it back
    st.ctx.release_scratch()


def test_config5_every_pair_recovers_the_generator_shift(batch):
    from vfx_image_stitching_amd import _lib
    _, _, _, jit, res = batch
    r = res.records
    assert len(r) == N_FRAMES - 1
    assert (r["status"] == _lib.PANO_OK).all()
    dy_true = np.diff(jit).astype(np.float64)
    err_x = np.abs(r["dx"] + STEP)
    err_y = np.abs(r["dy"] - dy_true)
    assert err_x.max() <= 1.5, (int(err_x.argmax()), float(err_x.max()))
    assert err_y.max() <= 1.5, (int(err_y.argmax()), float(err_y.max()))
    assert (r["n_matches"] > 1000).all()
    # the panorama: one loop of the strip, every frame's rows
    assert res.panorama.shape[1] >= (N_FRAMES - 1) * STEP
    assert res.panorama.shape[0] >= H // 2


def test_config5_first_pairs_equal_the_oracle_golden(batch, gold_json):
    _, _, _, _, res = batch
    r = res.records
    # the first pairs and the four spread over the sequence (make_golden_1080p_spread.py)
    pairs = gold_json("synthetic_1080p.json")["pairs"] + gold_json("synthetic_1080p_spread.json")["pairs"]
    assert len(pairs) == 6
    for want in pairs:
        p = want["pair"][0]
        assert abs(int(r[p]["n_matches"]) - want["n_matches"]) <= max(2, want["n_matches"] // 1000)
        assert abs(r[p]["dx"] - want["move"][0]) <= 1e-3 and abs(r[p]["dy"] - want["move"][1]) <= 1e-3, \
            (p, r[p], want)


def test_config5_shard_records_equal_the_whole_batch(batch):
    """Each rank of an 8-GPU strong-scaling run (143 pairs = 18 x 7 + 17) computes its records
    from its own frames (its pairs + the boundary frame): byte-identical to the whole batch's."""
    from vfx_image_stitching_amd import _lib
    from vfx_image_stitching_amd import distributed as D
    st, dev, focals, _, res = batch
    whole = res.records
    shards = D.shard_ranges(N_FRAMES - 1, 8)
    assert [c for _, c in shards] == [18] * 7 + [17]
    pmax = max(c for _, c in shards)
    for s, c in shards:
        block, _, _ = D.rank_records(st, dev[s:s + c + 1], focals[s:s + c + 1], pmax)
        got = block.cpu().numpy()
        assert not got[c:].any(), "padding rows of the block must stay zero"
        recs = got[:c].copy().view(_lib.PAIR_NP).reshape(-1)
        assert recs.tobytes() == whole[s:s + c].tobytes(), (s, c)
