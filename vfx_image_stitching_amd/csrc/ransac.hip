// ransac.hip -- R1: match filtering + exhaustive translation voting.
//
//   compute_shift_sift  image_stitching_sift.py:74-82   accept i if best_dist < desc_thresh
//   ransac              image_stitching_sift.py:86-111  (= image_stitching_harris.py:242-271)
//
// Every accepted match is a hypothesis (no sampling): votes_m = #{j : (dx_j - dx_m)^2 +
// (dy_j - dy_m)^2 < thr} in double (Python floats; no contraction), and the FIRST maximum
// in match order wins (strict '>' at :107).  One 1024-thread workgroup per pair: an
// order-preserving compaction of the accepted rows, an LDS-tiled K x K vote, and a
// (votes desc, index asc) block reduction.
#include "pano_internal.h"

namespace {

constexpr int RB = 1024;

struct PairArg {
    int32_t a[256], b[256];
};

__device__ int block_excl_scan(int v, int *sh, int &total) {
    const int tid = threadIdx.x;
    sh[tid] = v;
    __syncthreads();
    for (int off = 1; off < RB; off <<= 1) {
        const int t = tid >= off ? sh[tid - off] : 0;
        __syncthreads();
        sh[tid] += t;
        __syncthreads();
    }
    total = sh[RB - 1];
    const int r = sh[tid] - v;
    __syncthreads();
    return r;
}

// Exclusive scan of one flag per thread over the RB-thread block: a wave ballot gives the
// in-wave prefix (popcount of the lanes below), one barrier publishes the wave totals.  The
// Hillis-Steele scan above takes 2 log2(RB) = 20 barriers per RB rows: pair_compact 10.4 us.
__device__ __forceinline__ int block_flag_scan(bool flag, int *wsum, int &total) {
    const unsigned long long m = __ballot(flag);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int below = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wv] = __popcll(m);
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < RB / 64; ++w) {
        const int t = wsum[w];
        base += w < wv ? t : 0;
        tot += t;
    }
    total = tot;
    __syncthreads();                     // wsum is rewritten by the next call
    return base + below;
}

// votes for every move of `mv[0..k)`, then first-max; results in *best_m, *best_v
__device__ void vote_argmax(const double2 *mv, int k, double thr, double2 *tile, int *ish,
                            int *best_m, int *best_v) {
    const int tid = threadIdx.x;
    int my_best_v = -1, my_best_m = 0x7fffffff;
    for (int m0 = 0; m0 < k; m0 += RB) {
        const int m = m0 + tid;
        const double2 me = m < k ? mv[m] : make_double2(0.0, 0.0);
        int votes = 0;
        for (int j0 = 0; j0 < k; j0 += RB) {
            __syncthreads();
            if (j0 + tid < k) tile[tid] = mv[j0 + tid];
            __syncthreads();
            const int nj = k - j0 < RB ? k - j0 : RB;
            for (int j = 0; j < nj; ++j) {
                const double ddx = tile[j].x - me.x;
                const double ddy = tile[j].y - me.y;
                const double d = ddx * ddx + ddy * ddy;
                votes += d < thr;
            }
        }
        if (m < k && votes > my_best_v) {   // m increases per thread: strict '>' keeps first
            my_best_v = votes;
            my_best_m = m;
        }
    }
    // block reduction: max votes, then min index
    __syncthreads();
    ish[tid] = my_best_v;
    ish[RB + tid] = my_best_m;
    __syncthreads();
    for (int off = RB / 2; off > 0; off >>= 1) {
        if (tid < off) {
            const int v2 = ish[tid + off], m2 = ish[RB + tid + off];
            const int v1 = ish[tid], m1 = ish[RB + tid];
            if (v2 > v1 || (v2 == v1 && m2 < m1)) {
                ish[tid] = v2;
                ish[RB + tid] = m2;
            }
        }
        __syncthreads();
    }
    *best_v = ish[0];
    *best_m = ish[RB];
    __syncthreads();
}

// Large K (1080p: thousands of matches per pair) makes the K x K vote the bulk of the work,
// so it is split over many workgroups: pair_compact (one workgroup per pair: the ordered
// compaction, K to HBM), pair_votes (grid = hypothesis chunks x pairs, LDS-tiled, votes to
// HBM), pair_select (one workgroup per pair: first maximum, record).
__global__ void __launch_bounds__(RB)
pair_compact(const pano_kp *__restrict__ kps, const int32_t *__restrict__ xy,
             const int32_t *__restrict__ counts, int cap, PairArg pairs,
             const int32_t *__restrict__ best, const float *__restrict__ d1,
             const float *__restrict__ d2, float desc_thresh, double ratio,
             double2 *__restrict__ moves, int32_t *__restrict__ midx, int32_t *__restrict__ kcount,
             int32_t *__restrict__ votes) {
    __shared__ int wsum[RB / 64];
    const int p = blockIdx.x, tid = threadIdx.x;
    const int fa = pairs.a[p], fb = pairs.b[p];
    const int NA = min(max(counts[fa], 0), cap);
    const int NB = min(max(counts[fb], 0), cap);
    const int32_t *bp = best + (size_t)p * cap;
    const float *p1 = d1 + (size_t)p * cap, *p2 = d2 + (size_t)p * cap;
    double2 *mv = moves + (size_t)p * cap;
    int32_t *mi = midx + (size_t)p * cap;
    int K = 0;
    for (int base = 0; base < NA; base += RB) {
        const int i = base + tid;
        int acc = 0;
        if (i < NA && bp[i] >= 0 && bp[i] < NB && p1[i] < desc_thresh)
            // the visualiser's test m.distance < ratio * n.distance (sift_visualizeUI.py:252-257):
            // FLANN / BFMatcher distances are float32 L2 norms, sqrtf of the exact squared
            // distance (correctly rounded), compared in Python doubles
            acc = ratio > 0.0 ? ((double)sqrtf(p1[i]) < ratio * (double)sqrtf(p2[i])) : 1;
        int tot;
        const int pos = block_flag_scan(acc != 0, wsum, tot);
        if (acc) {
            const int j = bp[i];
            double xa, ya, xb, yb;
            if (kps) {
                const pano_kp ka = kps[(size_t)fa * cap + i], kb = kps[(size_t)fb * cap + j];
                xa = ka.x; ya = ka.y; xb = kb.x; yb = kb.y;
            } else {
                xa = xy[((size_t)fa * cap + i) * 2];
                ya = xy[((size_t)fa * cap + i) * 2 + 1];
                xb = xy[((size_t)fb * cap + j) * 2];
                yb = xy[((size_t)fb * cap + j) * 2 + 1];
            }
            mv[K + pos] = make_double2(xa - xb, ya - yb);
            mi[K + pos] = i;
            if (votes) votes[(size_t)p * cap + K + pos] = 0;      // pair_votes accumulates
        }
        K += tot;
    }
    if (tid == 0) kcount[p] = K;
}

constexpr int VB = 256;   // hypotheses per pair_votes workgroup
constexpr int VJS = 8;    // splits of the match range per hypothesis chunk (grid.z)

// Votes of hypotheses m0 .. m0 + VB - 1 against the matches of split blockIdx.z: the K x K
// test has one dependent f64 chain per (m, j), so a workgroup per (hypothesis chunk, pair)
// left ~1.4 waves per SIMD and exposed the chain and LDS latency (1080p: 0.63 ms per step).
// Splitting the match range VJS ways gives VJS x the waves; four matches per iteration are
// four independent chains.  Partial counts are integer atomics into zeroed votes: exact.
// pair_select's work for pair p with NT threads: the record of an overflowed or match-less
// pair, else the first maximum of the votes (strict '>' in match order,
// image_stitching_sift.py:107) and its record.  vote(m) reads hypothesis m's count.
template <int NT, typename VOTE>
__device__ __forceinline__ void select_pair(int *ish, const pano_kp *__restrict__ kps,
                                            const int32_t *__restrict__ xy, const int32_t *__restrict__ counts,
                                            int cap, int fa, int fb, const int32_t *__restrict__ bp,
                                            const double2 *__restrict__ mv, const int32_t *__restrict__ mi, int K,
                                            VOTE vote, pano_pair_rec *__restrict__ rec) {
    const int tid = threadIdx.x;
    pano_pair_rec r{};
    r.n_matches = K;
    // a frame with more keypoints than the capacity (count > cap) or whose keypoint stages
    // overflowed (count -1) was matched on a truncated set: the pair's result is not the
    // reference's, so the record says so instead of carrying a silently different shift
    const int ca = counts[fa], cb = counts[fb];
    if (ca < 0 || cb < 0 || ca > cap || cb > cap) {
        if (tid == 0) {
            r.best = -1;
            r.status = PANO_E_OVERFLOW;
            *rec = r;
        }
        return;
    }
    if (K == 0) {
        if (tid == 0) {
            r.best = -1;
            r.status = PANO_E_NOMATCH;
            *rec = r;
        }
        return;
    }
    int my_v = -1, my_m = 0x7fffffff;
    for (int m = tid; m < K; m += NT) {
        const int v = vote(m);
        if (v > my_v) { my_v = v; my_m = m; }
    }
    ish[tid] = my_v;
    ish[NT + tid] = my_m;
    __syncthreads();
    for (int off = NT / 2; off > 0; off >>= 1) {
        if (tid < off) {
            const int v2 = ish[tid + off], m2 = ish[NT + tid + off];
            const int v1 = ish[tid], m1 = ish[NT + tid];
            if (v2 > v1 || (v2 == v1 && m2 < m1)) {
                ish[tid] = v2;
                ish[NT + tid] = m2;
            }
        }
        __syncthreads();
    }
    const int bm = ish[NT], bv = ish[0];
    if (tid == 0) {
        const int i = mi[bm];
        const int j = bp[i];
        if (kps) {
            const pano_kp ka = kps[(size_t)fa * cap + i], kb = kps[(size_t)fb * cap + j];
            r.xA = ka.x; r.yA = ka.y; r.xB = kb.x; r.yB = kb.y;
        } else {
            r.xA = xy[((size_t)fa * cap + i) * 2];
            r.yA = xy[((size_t)fa * cap + i) * 2 + 1];
            r.xB = xy[((size_t)fb * cap + j) * 2];
            r.yB = xy[((size_t)fb * cap + j) * 2 + 1];
        }
        r.dx = mv[bm].x;
        r.dy = mv[bm].y;
        r.votes = bv;
        r.best = bm;
        r.status = PANO_OK;
        *rec = r;
    }
}

typedef __attribute__((address_space(1))) int g_i32;

// pair_select folded into pair_votes (SEL, PANO_RANSAC_FOLD): each live workgroup drains its
// vote atomics (s_waitcnt vmcnt(0), barrier) and counts itself in on its pair with one
// device-scope add; the pair's last live workgroup reads the votes back with sc1 loads (device-
// scope atomics and sc1 loads meet at the device-coherent level: MI355X guide, visibility),
// runs pair_select's work and re-zeroes the counter.  A pair with no live vote workgroup (no
// match) gets its record from workgroup (0, p, 0).
struct SelArgs {
    const pano_kp *kps;
    const int32_t *xy, *counts, *best, *midx;
    PairArg pairs;
    pano_pair_rec *recs;
    int32_t *cnt;                        // [pair] arrivals (zero between launches)
};

template <bool SEL>
__global__ void __launch_bounds__(VB)
pair_votes(const double2 *__restrict__ moves, const int32_t *__restrict__ kcount, int cap,
           double thr, int32_t *__restrict__ votes, SelArgs sa) {
    __shared__ double2 tile[VB];
    __shared__ int ish[2 * VB];
    __shared__ int last;
    // grid (split, pair, hypothesis chunk): the chunks are sized by the capacity, and with
    // the chunk index outermost every live chunk 0 is dispatched before the empty ones
    const int p = blockIdx.y, tid = threadIdx.x;
    const int K = kcount[p];
    const int m0 = blockIdx.z * VB;
    const int jlo = (int)((long long)K * blockIdx.x / VJS), jhi = (int)((long long)K * (blockIdx.x + 1) / VJS);
    const double2 *mv = moves + (size_t)p * cap;
    if (m0 >= K || jlo >= jhi) {                      // whole workgroup
        if (SEL && K == 0 && blockIdx.x == 0 && blockIdx.z == 0)
            select_pair<VB>(ish, sa.kps, sa.xy, sa.counts, cap, sa.pairs.a[p], sa.pairs.b[p],
                            sa.best + (size_t)p * cap, mv, sa.midx + (size_t)p * cap, 0, [](int) { return 0; },
                            sa.recs + p);
        return;
    }
    const int m = m0 + tid;
    const double2 me = m < K ? mv[m] : make_double2(0.0, 0.0);
    int v = 0;
    for (int j0 = jlo; j0 < jhi; j0 += VB) {
        __syncthreads();
        if (j0 + tid < jhi) tile[tid] = mv[j0 + tid];
        __syncthreads();
        const int nj = jhi - j0 < VB ? jhi - j0 : VB;
        int j = 0;
        for (; j + 4 <= nj; j += 4) {
            int c[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const double ddx = tile[j + u].x - me.x;
                const double ddy = tile[j + u].y - me.y;
                c[u] = (ddx * ddx + ddy * ddy) < thr;
            }
            v += (c[0] + c[1]) + (c[2] + c[3]);
        }
        for (; j < nj; ++j) {
            const double ddx = tile[j].x - me.x;
            const double ddy = tile[j].y - me.y;
            v += (ddx * ddx + ddy * ddy) < thr;
        }
    }
    if (m < K && v) atomicAdd(&votes[(size_t)p * cap + m], v);
    if constexpr (SEL) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // every wave: its adds performed
        __syncthreads();
        if (tid == 0) {
            int splits = 0;                                   // live match-range splits of K
            for (int x = 0; x < VJS; ++x)
                splits += (int)((long long)K * x / VJS) < (int)((long long)K * (x + 1) / VJS);
            const int n_live = ((K + VB - 1) / VB) * splits;
            fold_release();
            last = __hip_atomic_fetch_add((g_i32 *)(sa.cnt + p), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                   n_live - 1;
        }
        __syncthreads();
        if (!last) return;
        fold_acquire();
        int32_t *vp = votes + (size_t)p * cap;
        select_pair<VB>(ish, sa.kps, sa.xy, sa.counts, cap, sa.pairs.a[p], sa.pairs.b[p],
                        sa.best + (size_t)p * cap, mv, sa.midx + (size_t)p * cap, K,
                        [&](int mm) {
                            return __hip_atomic_load((g_i32 *)(vp + mm), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        },
                        sa.recs + p);
        if (tid == 0) __hip_atomic_store((g_i32 *)(sa.cnt + p), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void __launch_bounds__(RB)
pair_select(const pano_kp *__restrict__ kps, const int32_t *__restrict__ xy,
            const int32_t *__restrict__ counts, int cap, PairArg pairs,
            const int32_t *__restrict__ best, const double2 *__restrict__ moves,
            const int32_t *__restrict__ midx, const int32_t *__restrict__ kcount,
            const int32_t *__restrict__ votes, pano_pair_rec *__restrict__ recs) {
    __shared__ int ish[2 * RB];
    const int p = blockIdx.x;
    const int32_t *vp = votes + (size_t)p * cap;
    select_pair<RB>(ish, kps, xy, counts, cap, pairs.a[p], pairs.b[p], best + (size_t)p * cap,
                    moves + (size_t)p * cap, midx + (size_t)p * cap, kcount[p], [&](int m) { return vp[m]; },
                    recs + p);
}

__global__ void __launch_bounds__(RB)
ransac_moves(const double2 *__restrict__ mv, int k, double thr, int32_t *__restrict__ out) {
    __shared__ int ish[2 * RB];
    __shared__ double2 tile[RB];
    if (k <= 0) {
        if (threadIdx.x == 0) { out[0] = -1; out[1] = 0; }
        return;
    }
    int bm, bv;
    vote_argmax(mv, k, thr, tile, ish, &bm, &bv);
    if (threadIdx.x == 0) { out[0] = bm; out[1] = bv; }
}

}  // namespace

int launch_pair_shifts(pano_ctx *ctx, const pano_kp *kps, const int32_t *xy_i32,
                       const int32_t *counts, int cap, const int32_t *h_pairs, int n_pairs,
                       const int32_t *best, const float *d1, const float *d2,
                       double desc_thresh, double ratio, double thr, pano_pair_rec *recs) {
    if (cap <= 0 || n_pairs <= 0 || (!kps && !xy_i32) || !counts || !best || !d1 ||
        (!d2 && ratio > 0) || !recs)
        return pano_fail(ctx, PANO_E_ARG, "pano_pair_shifts: bad arguments");
    const size_t need = (size_t)n_pairs * cap * (sizeof(double2) + 2 * sizeof(int32_t)) +
                        (size_t)n_pairs * sizeof(int32_t) + 256;
    int rc = pano_grow(ctx, &ctx->bscratch, &ctx->bscratch_bytes, need);
    if (rc) return rc;
    double2 *moves = (double2 *)ctx->bscratch;
    int32_t *midx = (int32_t *)(moves + (size_t)n_pairs * cap);
    int32_t *votes = midx + (size_t)n_pairs * cap;
    int32_t *kcount = votes + (size_t)n_pairs * cap;
    for (int p0 = 0; p0 < n_pairs; p0 += 256) {
        const int np = n_pairs - p0 < 256 ? n_pairs - p0 : 256;
        PairArg pa;
        for (int q = 0; q < np; ++q) {
            pa.a[q] = h_pairs[2 * (p0 + q)];
            pa.b[q] = h_pairs[2 * (p0 + q) + 1];
        }
        const size_t o = (size_t)p0 * cap;
        {
            PanoProf prof_(ctx, PK_PAIR_SHIFTS);
            pair_compact<<<np, RB, 0, ctx->stream>>>(
                kps, xy_i32, counts, cap, pa, best + o, d1 + o, d2 ? d2 + o : nullptr,
                (float)desc_thresh, ratio > 0 ? ratio : 0.0, moves + o, midx + o, kcount + p0, votes + o);
        }
        PANO_LAUNCH_CHECK(ctx, "pair_compact");
        static const bool fold_on = [] {              // pair_select folded into pair_votes
            const char *e = getenv("PANO_RANSAC_FOLD");
            return e ? atoi(e) != 0 : true;
        }();
        SelArgs sa{};
        if (fold_on) {
            const size_t need_c = 256 * sizeof(int32_t);
            if (need_c > ctx->sel_sync_bytes) {
                if (ctx->capturing) return pano_fail(ctx, PANO_E_UNSUPPORTED, "select counters inside a graph capture");
                PANO_HIP(ctx, hipMalloc((void **)&ctx->sel_sync, need_c));
                PANO_HIP(ctx, hipMemset(ctx->sel_sync, 0, need_c));     // each launch re-zeroes
                ctx->sel_sync_bytes = need_c;
            }
            sa.kps = kps;
            sa.xy = xy_i32;
            sa.counts = counts;
            sa.best = best + o;
            sa.midx = midx + o;
            sa.pairs = pa;
            sa.recs = recs + p0;
            sa.cnt = ctx->sel_sync;
        }
        {
            PanoProf prof_(ctx, PK_PAIR_SHIFTS);
            if (fold_on)
                pair_votes<true><<<dim3(VJS, np, (cap + VB - 1) / VB), VB, 0, ctx->stream>>>(moves + o, kcount + p0,
                                                                                            cap, thr, votes + o, sa);
            else
                pair_votes<false><<<dim3(VJS, np, (cap + VB - 1) / VB), VB, 0, ctx->stream>>>(moves + o, kcount + p0,
                                                                                             cap, thr, votes + o, sa);
        }
        PANO_LAUNCH_CHECK(ctx, "pair_votes");
        if (fold_on) continue;
        {
            PanoProf prof_(ctx, PK_PAIR_SHIFTS);
            pair_select<<<np, RB, 0, ctx->stream>>>(kps, xy_i32, counts, cap, pa, best + o, moves + o, midx + o,
                                                   kcount + p0, votes + o, recs + p0);
        }
        PANO_LAUNCH_CHECK(ctx, "pair_select");
    }
    return PANO_OK;
}

// Ordered compaction of the accepted matches of np pairs (desc_thresh, optional Lowe ratio):
// moves / midx [np][cap], kcount [np].  Shared with the homography path.
int launch_match_compact(pano_ctx *ctx, const pano_kp *kps, const int32_t *counts, int cap,
                         const int32_t *fa, const int32_t *fb, int np, const int32_t *best,
                         const float *d1, const float *d2, double desc_thresh, double ratio,
                         void *moves, int32_t *midx, int32_t *kcount) {
    if (np < 1 || np > 256) return pano_fail(ctx, PANO_E_ARG, "match compaction: 1..256 pairs");
    PairArg pa;
    for (int q = 0; q < np; ++q) {
        pa.a[q] = fa[q];
        pa.b[q] = fb[q];
    }
    {
        PanoProf prof_(ctx, PK_PAIR_SHIFTS);
        pair_compact<<<np, RB, 0, ctx->stream>>>(kps, nullptr, counts, cap, pa, best, d1, d2,
                                                desc_thresh > 0 ? (float)desc_thresh : INFINITY,
                                                ratio > 0 ? ratio : 0.0,
                                                (double2 *)moves, midx, kcount, nullptr);
    }
    PANO_LAUNCH_CHECK(ctx, "pair_compact");
    return PANO_OK;
}

int launch_ransac_translate(pano_ctx *ctx, const double *moves, int k, double thr,
                            int32_t *out) {
    if (k < 0 || (k > 0 && !moves) || !out) return pano_fail(ctx, PANO_E_ARG, "pano_ransac_translate");
    {
        PanoProf prof_(ctx, PK_PAIR_SHIFTS);
        ransac_moves<<<1, RB, 0, ctx->stream>>>((const double2 *)moves, k, thr, out);
    }
    PANO_LAUNCH_CHECK(ctx, "ransac_moves");
    return PANO_OK;
}
