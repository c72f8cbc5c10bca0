"""the visualiser's ratio-test matches + homography RANSAC
(sift_visualizeUI.py:247-273).

CPU: the oracle (oracle/homography.py) on known homographies, its degenerate cases and the
sampler's hash.  GPU: pano_pair_homography (csrc/homography.hip) against the oracle on the
same correspondences -- inlier counts, hypothesis choice and masks exact, H to 1e-9 relative
(the kernel contracts multiply-adds, numpy does not) -- and on real frames through the
two-image call the visualiser makes.  Parity with cv2.findHomography itself is unpinned
(OpenCV is absent; its sampler is random and it refines with Levenberg-Marquardt).
"""
from __future__ import annotations

import numpy as np
import pytest

from oracle import homography as ohom


def _known_h(rng):
    H = np.array([[1.02, 0.03, 35.0], [-0.02, 0.98, -12.0], [2e-5, -1e-5, 1.0]])
    H[:2, :2] += rng.normal(0, 0.01, (2, 2))
    return H


def _correspondences(seed, K=400, outlier_frac=0.3, noise=0.5, w=640, h=480):
    rng = np.random.default_rng(seed)
    H = _known_h(rng)
    S = np.c_[rng.uniform(0, w, K), rng.uniform(0, h, K)]
    D = ohom.perspective_transform(S, H) + rng.normal(0, noise, (K, 2))
    out = rng.random(K) < outlier_frac
    D[out] = np.c_[rng.uniform(0, w, out.sum()), rng.uniform(0, h, out.sum())]
    # float32 keypoint positions, as pano_kp carries them
    return H, S.astype(np.float32).astype(np.float64), D.astype(np.float32).astype(np.float64), ~out


# ------------------------------------------------------------------ CPU: oracle
def test_splitmix64_known_answer():
    # first outputs of the published SplitMix64 generator from state 0
    assert ohom.splitmix64(0) == 0xE220A8397B1DCDAF
    assert ohom.splitmix64(0x9E3779B97F4A7C15) == 0x6E789E6AA1B965F4


def test_oracle_recovers_known_homography():
    H0, S, D, inl = _correspondences(1)
    r = ohom.find_homography(S, D, thr=5.0, n_hyp=500, seed=3)
    assert r["status"] == "ok"
    H = r["H"].reshape(3, 3)
    grid = np.c_[np.repeat(np.arange(0, 640, 64), 8), np.tile(np.arange(0, 480, 60), 10)]
    err = np.abs(ohom.perspective_transform(grid, H) - ohom.perspective_transform(grid, H0)).max()
    assert err < 1.0, err
    # every true inlier within the threshold is found, and no far outlier
    true_in = inl & (ohom.reproj_err2(H0.reshape(-1), S, D) <= 25.0)
    assert r["mask"][true_in].mean() > 0.98
    assert r["inliers"] >= r["hyp_inliers"] * 0.98


def test_oracle_exact_correspondences_are_reproduced():
    H0, S, D, _ = _correspondences(2, K=60, outlier_frac=0.0, noise=0.0)
    r = ohom.find_homography(S, D, thr=1.0, n_hyp=50)
    assert r["inliers"] == 60
    np.testing.assert_allclose(r["H"].reshape(3, 3), H0, rtol=1e-4, atol=1e-6)


def test_oracle_degenerate_cases():
    rng = np.random.default_rng(0)
    # too few good matches: len(good) > MIN_MATCH_COUNT fails
    S = rng.uniform(0, 100, (10, 2))
    assert ohom.find_homography(S, S + 3, min_good=10)["status"] == "nomatch"
    # all points on one line: every sample has a collinear triple
    t = rng.uniform(0, 100, 40)
    S = np.c_[t, 2 * t + 1]
    r = ohom.find_homography(S, S + 3, n_hyp=64)
    assert r["status"] == "nomatch" and r["hyp_inliers"] == 0
    # a mirror image flips every triangle's orientation: rejected like cv2's checkSubset
    S = rng.uniform(0, 100, (40, 2))
    r = ohom.find_homography(S, np.c_[-S[:, 0], S[:, 1]], n_hyp=64)
    assert r["status"] == "nomatch"


def test_oracle_ratio_filter_and_knn2():
    rng = np.random.default_rng(5)
    a = rng.integers(0, 256, (50, 128))
    b = np.concatenate([a[:30] + rng.integers(-2, 3, (30, 128)), rng.integers(0, 256, (40, 128))])
    best, d1, d2 = ohom.knn2(a, b)
    assert (best[:30] == np.arange(30)).all()
    good = ohom.good_matches(best, d1, d2, ratio=0.7)
    assert set(range(30)) <= set(good.tolist())
    brute = ((a[:, None, :] - b[None]) ** 2).sum(-1)
    assert (d1 == brute.min(1)).all()


def test_ratio_boundary_is_the_float32_distance_form():
    """(1078, 2200): the squared form 1078 < 0.49 * 2200 is False (equal), the visualiser's
    float32 L2 form sqrt(1078) < 0.7 * sqrt(2200) is True; good_matches follows the latter."""
    best = np.array([0], np.int32)
    assert ohom.good_matches(best, np.array([1078], np.float32), np.array([2200], np.float32)).tolist() == [0]
    assert not 1078 < 0.49 * 2200


# ------------------------------------------------------------------ GPU: pano_pair_homography
def _device_pairs(torch, sets, cap):
    """Frames 2p (source points) and 2p+1 (destination points) with best = identity."""
    n = 2 * len(sets)
    kps = np.zeros((n, cap, 6), np.float32)
    counts = np.zeros(n, np.int32)
    best = np.full((len(sets), cap), -1, np.int32)
    d1 = np.zeros((len(sets), cap), np.float32)
    d2 = np.full((len(sets), cap), 1e6, np.float32)
    for p, (S, D) in enumerate(sets):
        K = len(S)
        kps[2 * p, :K, :2] = S
        kps[2 * p + 1, :K, :2] = D
        counts[2 * p] = counts[2 * p + 1] = K
        best[p, :K] = np.arange(K)
        d1[p, :K] = 10.0
    dev = lambda a: torch.from_numpy(a).cuda()
    return dev(kps.view(np.int32)), dev(counts), dev(best), dev(d1), dev(d2)


def _run_device(gpu, torch, kps, counts, best, d1, d2, cap, pairs, thr=5.0, n_hyp=2000, seed=0,
                min_good=10, ratio=0.7):
    from vfx_image_stitching_amd import _lib
    from vfx_image_stitching_amd._lib import ptr
    import ctypes
    P = len(pairs)
    recs = torch.zeros((P, _lib.HOMOGRAPHY_NP.itemsize), dtype=torch.uint8, device="cuda")
    mask = torch.zeros((P, cap), dtype=torch.uint8, device="cuda")
    hp = np.ascontiguousarray(np.array(pairs, np.int32).reshape(-1))
    gpu.check(gpu.lib.pano_pair_homography(gpu.h, ptr(kps), ptr(counts), cap, _lib.i32p(hp), P, ptr(best),
                                           ptr(d1), ptr(d2), 0.0, ratio, thr, n_hyp, ctypes.c_uint64(seed),
                                           min_good, ptr(recs), ptr(mask)))
    gpu.sync()
    return recs.cpu().numpy().view(_lib.HOMOGRAPHY_NP).reshape(-1), mask.cpu().numpy()


def _assert_rec_matches_oracle(rec, m, ref, K):
    assert int(rec["n_matches"]) == K
    status = {0: "ok", -4: "nomatch", -3: "overflow"}[int(rec["status"])]
    assert status == ref["status"]
    assert int(rec["hyp_inliers"]) == ref["hyp_inliers"]
    if status == "ok":
        assert int(rec["inliers"]) == ref["inliers"]
        np.testing.assert_array_equal(m[:K].astype(bool), ref["mask"])
        np.testing.assert_allclose(rec["H"], ref["H"], rtol=1e-9, atol=1e-12)


@pytest.mark.gpu
def test_pair_homography_vs_oracle_known_homographies(gpu):
    import torch
    sets, refs = [], []
    for seed, K, frac in [(11, 400, 0.3), (12, 1500, 0.5), (13, 37, 0.1), (14, 2048, 0.2)]:
        H0, S, D, _ = _correspondences(seed, K, frac)
        sets.append((S, D))
    cap = 2048
    dev = _device_pairs(torch, sets, cap)
    pairs = [(2 * p, 2 * p + 1) for p in range(len(sets))]
    recs, mask = _run_device(gpu, torch, *dev, cap, pairs, n_hyp=1000, seed=7)
    for p, (S, D) in enumerate(sets):
        ref = ohom.find_homography(S, D, thr=5.0, n_hyp=1000, seed=7, pair=p)
        _assert_rec_matches_oracle(recs[p], mask[p], ref, len(S))
        assert recs[p]["status"] == 0


@pytest.mark.gpu
def test_pair_homography_more_than_256_pairs(gpu):
    """Batches above one 256-pair chunk: the sample hash takes the GLOBAL pair index, so pair
    p + 256 draws its own hypotheses and matches the oracle at pair = p + 256."""
    import torch
    S, D = _correspondences(31, 60, 0.3)[1:3]
    P = 300
    sets = [(S, D)] * P
    cap = 64
    dev = _device_pairs(torch, sets, cap)
    recs, mask = _run_device(gpu, torch, *dev, cap, [(2 * p, 2 * p + 1) for p in range(P)], n_hyp=64,
                             seed=5)
    for p in (0, 1, 255, 256, 257, 299):
        ref = ohom.find_homography(S, D, thr=5.0, n_hyp=64, seed=5, pair=p)
        _assert_rec_matches_oracle(recs[p], mask[p], ref, len(S))


@pytest.mark.gpu
def test_pair_homography_ratio_boundary(gpu):
    """The kernel's ratio test at the (1078, 2200) boundary keeps the match (float32 L2 form)."""
    import torch
    S, D = _correspondences(41, 30, 0.0)[1:3]
    cap = 64
    kps, counts, best, d1, d2 = _device_pairs(torch, [(S, D)], cap)
    d1.fill_(1078.0)
    d2.fill_(2200.0)
    recs, _ = _run_device(gpu, torch, kps, counts, best, d1, d2, cap, [(0, 1)], n_hyp=64)
    assert int(recs["n_matches"][0]) == 30


@pytest.mark.gpu
def test_pair_homography_degenerate_and_overflow(gpu):
    import torch
    rng = np.random.default_rng(3)
    t = rng.choice(100, 40, replace=False).astype(np.float64)   # exact in float32: truly collinear
    line = np.c_[t, 2 * t + 1]
    few = rng.uniform(0, 100, (10, 2))
    ok = _correspondences(21, 200, 0.2)[1:3]
    cap = 256
    sets = [(line, line + 3), (few, few + 3), ok, ok]
    kps, counts, best, d1, d2 = _device_pairs(torch, sets, cap)
    counts[7] = cap + 5                      # frame 7 had more keypoints than the capacity
    recs, mask = _run_device(gpu, torch, kps, counts, best, d1, d2, cap,
                             [(0, 1), (2, 3), (4, 5), (6, 7)], n_hyp=256)
    assert recs["status"].tolist() == [-4, -4, 0, -3]
    assert not mask[0, :40].any() and not mask[1, :10].any()
    # an empty pair and a pair whose every match fails the ratio test
    kps2, counts2, best2, d12, d22 = _device_pairs(torch, [ok], cap)
    counts2[0] = 0
    recs2, _ = _run_device(gpu, torch, kps2, counts2, best2, d12, d22, cap, [(0, 1)])
    assert recs2["status"][0] == -4 and recs2["n_matches"][0] == 0
    kps3, counts3, best3, d13, d23 = _device_pairs(torch, [ok], cap)
    d23.fill_(11.0)                          # sqrt(10) < 0.7 sqrt(11) fails
    recs3, _ = _run_device(gpu, torch, kps3, counts3, best3, d13, d23, cap, [(0, 1)])
    assert recs3["status"][0] == -4 and recs3["n_matches"][0] == 0


def _gray(img):
    from oracle import cv2_compat
    return cv2_compat.bgr_to_gray_u8(img)


@pytest.mark.gpu
@pytest.mark.parametrize("pair", [(0, 1), (5, 6)])
def test_match_homography_parrington_vs_oracle(gpu, parrington, pair):
    from vfx_image_stitching_amd.homography import match_homography
    from vfx_image_stitching_amd import sift_impl
    names, frames, focals, _ = parrington
    g1, g2 = _gray(frames[pair[0]]), _gray(frames[pair[1]])
    kp1, kp2, res, outline = match_homography(g1, g2)
    _, des1 = sift_impl.compute_keypoints_and_descriptors(g1)
    _, des2 = sift_impl.compute_keypoints_and_descriptors(g2)
    assert len(des1) == len(kp1) and len(des2) == len(kp2)
    best, d1, d2 = ohom.knn2(des1, des2)
    good = ohom.good_matches(best, d1, d2, ratio=0.7)
    np.testing.assert_array_equal(res.good[:, 0], good)
    np.testing.assert_array_equal(res.good[:, 1], best[good])
    np.testing.assert_allclose(res.distance, np.sqrt(d1[good].astype(np.float64)), rtol=1e-6)
    S = np.array([kp1[i].pt for i in res.good[:, 0]], np.float32).astype(np.float64)
    D = np.array([kp2[j].pt for j in res.good[:, 1]], np.float32).astype(np.float64)
    ref = ohom.find_homography(S, D, thr=5.0, n_hyp=2000, seed=0, pair=0)
    assert res.status == "ok" == ref["status"]
    assert res.inliers == ref["inliers"] and res.hyp_inliers == ref["hyp_inliers"]
    np.testing.assert_array_equal(res.mask, ref["mask"])
    np.testing.assert_allclose(res.H.reshape(-1), ref["H"], rtol=1e-9, atol=1e-12)
    # consecutive frames of a panning sequence: mostly inliers, and the outline is the
    # query frame displaced sideways
    assert res.inliers >= 0.5 * len(res.good)
    h, w = g1.shape
    assert outline.shape == (4, 1, 2)
    assert np.abs(np.diff(outline[:, 0, 1][[0, 3]])) < 0.2 * h
