// homography.hip -- SURVEY 8(f3): Lowe-ratio matches + homography RANSAC, the visualiser's
// path (sift_visualizeUI.py:247-266: FLANN kNN-2, `m.distance < 0.7 * n.distance`, then
// cv2.findHomography(src, dst, cv2.RANSAC, 5.0) when there are more than MIN_MATCH_COUNT = 10
// good matches).
//
// The neighbours are the EXACT brute-force kNN-2 of pano_match / pano_match_u8 (FLANN's
// randomised kd-trees are approximate), and the RANSAC is deterministic so that results
// are reproducible and testable against oracle/homography.py:
//   hypotheses  n_hyp 4-point samples of the good matches drawn by a counter-based hash
//               (splitmix64 of seed, pair, hypothesis, draw); samples with a collinear
//               triple or inconsistent triangle orientations between source and destination
//               are rejected (what cv2's HomographyEstimatorCallback::checkSubset rejects);
//   model       the 4-point DLT with h33 = 1: an 8 x 8 linear system solved in double by
//               Gaussian elimination with partial pivoting (singular -> rejected);
//   score       inliers = #{j : ||dst_j - H(src_j)||^2 <= thr^2} in double (cv2 compares
//               the squared reprojection error with thr^2 the same way); the first best
//               hypothesis wins;
//   refit       Hartley-normalised least squares over the winner's inliers (normal
//               equations of the linear DLT, 8 x 8, double), then the inliers recounted.
// cv2's refinement is Levenberg-Marquardt on the reprojection error and its sampling is
// random, so parity with cv2.findHomography itself is unpinned (OpenCV is not installed);
// the tests pin this kernel to its own restatement and to known homographies.
#include "pano_internal.h"

namespace {

constexpr int HB = 256;          // hypotheses per workgroup / threads per workgroup

struct PairArg {
    int32_t a[256], b[256];
};

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// Solve A x = b (n x n, row-major, in place) by Gaussian elimination with partial pivoting.
template <int N>
__device__ bool solve_gauss(double (&A)[N][N], double (&b)[N], double (&x)[N]) {
    double amax = 0.0;
    for (int i = 0; i < N; ++i)
        for (int j = 0; j < N; ++j) amax = fmax(amax, fabs(A[i][j]));
    if (!(amax > 0.0)) return false;
    for (int c = 0; c < N; ++c) {
        int p = c;
        for (int r = c + 1; r < N; ++r)
            if (fabs(A[r][c]) > fabs(A[p][c])) p = r;
        if (!(fabs(A[p][c]) > 1e-12 * amax)) return false;
        if (p != c) {
            for (int j = 0; j < N; ++j) { const double t = A[c][j]; A[c][j] = A[p][j]; A[p][j] = t; }
            const double t = b[c]; b[c] = b[p]; b[p] = t;
        }
        for (int r = c + 1; r < N; ++r) {
            const double f = A[r][c] / A[c][c];
            for (int j = c; j < N; ++j) A[r][j] -= f * A[c][j];
            b[r] -= f * b[c];
        }
    }
    for (int r = N - 1; r >= 0; --r) {
        double s = b[r];
        for (int j = r + 1; j < N; ++j) s -= A[r][j] * x[j];
        x[r] = s / A[r][r];
    }
    return true;
}

// 4-point DLT with h33 = 1: u = (h0 x + h1 y + h2) / (h6 x + h7 y + 1), v likewise.
__device__ bool dlt4(const double2 (&s)[4], const double2 (&d)[4], double (&H)[9]) {
    double A[8][8], b[8], h[8];
    for (int k = 0; k < 4; ++k) {
        const double x = s[k].x, y = s[k].y, u = d[k].x, v = d[k].y;
        double *r0 = A[2 * k], *r1 = A[2 * k + 1];
        r0[0] = x; r0[1] = y; r0[2] = 1; r0[3] = 0; r0[4] = 0; r0[5] = 0; r0[6] = -u * x; r0[7] = -u * y;
        r1[0] = 0; r1[1] = 0; r1[2] = 0; r1[3] = x; r1[4] = y; r1[5] = 1; r1[6] = -v * x; r1[7] = -v * y;
        b[2 * k] = u;
        b[2 * k + 1] = v;
    }
    if (!solve_gauss<8>(A, b, h)) return false;
    for (int i = 0; i < 8; ++i) H[i] = h[i];
    H[8] = 1.0;
    return true;
}

__device__ __forceinline__ double cross3(double2 a, double2 b, double2 c) {
    return (b.x - a.x) * (c.y - a.y) - (b.y - a.y) * (c.x - a.x);
}

// cv2 checkSubset for homographies: no collinear triple, and every triangle of the four
// points keeps its orientation from source to destination.
__device__ bool good_sample(const double2 (&s)[4], const double2 (&d)[4]) {
    const int tri[4][3] = {{0, 1, 2}, {1, 2, 3}, {2, 3, 0}, {3, 0, 1}};
    for (int t = 0; t < 4; ++t) {
        const double cs = cross3(s[tri[t][0]], s[tri[t][1]], s[tri[t][2]]);
        const double cd = cross3(d[tri[t][0]], d[tri[t][1]], d[tri[t][2]]);
        if (fabs(cs) < 1e-6 || fabs(cd) < 1e-6) return false;
        if ((cs > 0) != (cd > 0)) return false;
    }
    return true;
}

__device__ __forceinline__ double reproj_err2(const double (&H)[9], double2 s, double2 d) {
    const double w = H[6] * s.x + H[7] * s.y + H[8];
    const double u = (H[0] * s.x + H[1] * s.y + H[2]) / w;
    const double v = (H[3] * s.x + H[4] * s.y + H[5]) / w;
    const double du = u - d.x, dv = v - d.y;
    return du * du + dv * dv;
}

// Good matches of pair p as (src, dst) points, from pair_compact's ordered match indices.
__global__ void __launch_bounds__(256)
gather_points(const pano_kp *__restrict__ kps, int cap, PairArg pairs, const int32_t *__restrict__ best,
              const int32_t *__restrict__ midx, const int32_t *__restrict__ kcount,
              double2 *__restrict__ src, double2 *__restrict__ dst) {
    const int p = blockIdx.y, k = blockIdx.x * 256 + threadIdx.x;
    if (k >= kcount[p]) return;
    const int i = midx[(size_t)p * cap + k];
    const int j = best[(size_t)p * cap + i];
    const pano_kp a = kps[(size_t)pairs.a[p] * cap + i], b = kps[(size_t)pairs.b[p] * cap + j];
    src[(size_t)p * cap + k] = make_double2(a.x, a.y);
    dst[(size_t)p * cap + k] = make_double2(b.x, b.y);
}

// One hypothesis per thread: sample, model, inlier count over every good match (LDS tiles).
__global__ void __launch_bounds__(HB)
homography_hyp(const double2 *__restrict__ src, const double2 *__restrict__ dst,
               const int32_t *__restrict__ kcount, int cap, int n_hyp, int min_good,
               unsigned long long seed, double thr2, int32_t *__restrict__ score, int p0) {
    __shared__ double2 ts[HB], td[HB];
    const int p = blockIdx.y, tid = threadIdx.x;
    const int hyp = blockIdx.x * HB + tid;
    const int K = kcount[p];
    if (K <= min_good || K < 4) return;                   // uniform: no model for this pair
    const double2 *S = src + (size_t)p * cap, *D = dst + (size_t)p * cap;
    double H[9];
    bool ok = false;
    if (hyp < n_hyp) {
        int idx[4];
        int draw = 0;
        for (int q = 0; q < 4; ++q) {
            for (;;) {                                    // distinct indices, deterministic
                const unsigned long long r =
                    splitmix64(seed ^ ((unsigned long long)(p0 + p) << 48) ^ ((unsigned long long)hyp << 16) ^ (unsigned long long)draw++);
                const int c = (int)(r % (unsigned long long)K);
                bool dup = false;
                for (int e = 0; e < q; ++e) dup |= idx[e] == c;
                if (!dup) { idx[q] = c; break; }
            }
        }
        double2 s4[4], d4[4];
        for (int q = 0; q < 4; ++q) { s4[q] = S[idx[q]]; d4[q] = D[idx[q]]; }
        ok = good_sample(s4, d4) && dlt4(s4, d4, H);
    }
    int n_in = 0;
    for (int j0 = 0; j0 < K; j0 += HB) {
        __syncthreads();
        if (j0 + tid < K) { ts[tid] = S[j0 + tid]; td[tid] = D[j0 + tid]; }
        __syncthreads();
        const int nj = K - j0 < HB ? K - j0 : HB;
        if (ok)
            for (int j = 0; j < nj; ++j) n_in += reproj_err2(H, ts[j], td[j]) <= thr2;
    }
    if (hyp < n_hyp) score[(size_t)p * n_hyp + hyp] = ok ? n_in : -1;
}

// Per pair: the first best hypothesis, its inliers, the normalised least-squares refit over
// them, the refit's inliers (mask written when requested).  One workgroup per pair.
__global__ void __launch_bounds__(HB)
homography_select(const double2 *__restrict__ src, const double2 *__restrict__ dst,
                  const int32_t *__restrict__ kcount, int cap, int n_hyp, int min_good,
                  unsigned long long seed, double thr2, const int32_t *__restrict__ score,
                  const int32_t *__restrict__ counts, PairArg pairs,
                  pano_homography_rec *__restrict__ recs, uint8_t *__restrict__ mask, int p0) {
    __shared__ int sv[HB], si[HB];
    __shared__ double red[HB];
    __shared__ double Hs[9];
    __shared__ double M[8][9];                 // normal equations [A^T A | A^T b]
    const int p = blockIdx.x, tid = threadIdx.x;
    const int K = kcount[p];
    pano_homography_rec r{};
    r.n_matches = K;
    const double2 *S = src + (size_t)p * cap, *D = dst + (size_t)p * cap;
    // a frame whose keypoints did not fit the capacity was matched on a truncated set
    const int ca = counts[pairs.a[p]], cb = counts[pairs.b[p]];
    const bool overflow = ca < 0 || cb < 0 || ca > cap || cb > cap;
    if (overflow || K <= min_good || K < 4) {
        if (tid == 0) {
            r.status = overflow ? PANO_E_OVERFLOW : PANO_E_NOMATCH;
            for (int q = 0; q < 9; ++q) r.H[q] = 0.0;
            recs[p] = r;
        }
        if (mask) for (int j = tid; j < K; j += HB) mask[(size_t)p * cap + j] = 0;
        return;
    }
    // ---- first best hypothesis
    int bv = -1, bi = 0x7fffffff;
    for (int h = tid; h < n_hyp; h += HB) {
        const int v = score[(size_t)p * n_hyp + h];
        if (v > bv) { bv = v; bi = h; }
    }
    sv[tid] = bv;
    si[tid] = bi;
    __syncthreads();
    for (int off = HB / 2; off > 0; off >>= 1) {
        if (tid < off) {
            const int v2 = sv[tid + off], i2 = si[tid + off];
            if (v2 > sv[tid] || (v2 == sv[tid] && i2 < si[tid])) { sv[tid] = v2; si[tid] = i2; }
        }
        __syncthreads();
    }
    const int hv = sv[0], hi = si[0];
    if (hv < 4) {                                          // no valid model
        if (tid == 0) {
            r.status = PANO_E_NOMATCH;
            r.hyp_inliers = hv < 0 ? 0 : hv;
            for (int q = 0; q < 9; ++q) r.H[q] = 0.0;
            recs[p] = r;
        }
        if (mask) for (int j = tid; j < K; j += HB) mask[(size_t)p * cap + j] = 0;
        return;
    }
    // rebuild the winning hypothesis (same draws as homography_hyp)
    if (tid == 0) {
        int idx[4], draw = 0;
        for (int q = 0; q < 4; ++q) {
            for (;;) {
                const unsigned long long rr =
                    splitmix64(seed ^ ((unsigned long long)(p0 + p) << 48) ^ ((unsigned long long)hi << 16) ^ (unsigned long long)draw++);
                const int c = (int)(rr % (unsigned long long)K);
                bool dup = false;
                for (int e = 0; e < q; ++e) dup |= idx[e] == c;
                if (!dup) { idx[q] = c; break; }
            }
        }
        double2 s4[4], d4[4];
        for (int q = 0; q < 4; ++q) { s4[q] = S[idx[q]]; d4[q] = D[idx[q]]; }
        double H[9];
        dlt4(s4, d4, H);
        for (int q = 0; q < 9; ++q) Hs[q] = H[q];
    }
    __syncthreads();
    double H[9];
    for (int q = 0; q < 9; ++q) H[q] = Hs[q];
    // ---- Hartley normalisation over the inliers: centroids, mean distances -> sqrt(2)
    auto block_sum = [&](double v) {
        red[tid] = v;
        __syncthreads();
        for (int off = HB / 2; off > 0; off >>= 1) {
            if (tid < off) red[tid] += red[tid + off];
            __syncthreads();
        }
        const double s = red[0];
        __syncthreads();
        return s;
    };
    double sx = 0, sy = 0, dx = 0, dy = 0, cnt = 0;
    for (int j = tid; j < K; j += HB)
        if (reproj_err2(H, S[j], D[j]) <= thr2) {
            sx += S[j].x; sy += S[j].y; dx += D[j].x; dy += D[j].y; cnt += 1;
        }
    const double n_in = block_sum(cnt);
    const double msx = block_sum(sx) / n_in, msy = block_sum(sy) / n_in;
    const double mdx = block_sum(dx) / n_in, mdy = block_sum(dy) / n_in;
    double ds = 0, dd = 0;
    for (int j = tid; j < K; j += HB)
        if (reproj_err2(H, S[j], D[j]) <= thr2) {
            ds += sqrt((S[j].x - msx) * (S[j].x - msx) + (S[j].y - msy) * (S[j].y - msy));
            dd += sqrt((D[j].x - mdx) * (D[j].x - mdx) + (D[j].y - mdy) * (D[j].y - mdy));
        }
    const double ms = block_sum(ds) / n_in, md = block_sum(dd) / n_in;
    const double ks = ms > 0 ? 1.4142135623730951 / ms : 1.0, kd = md > 0 ? 1.4142135623730951 / md : 1.0;
    // ---- normal equations of the normalised linear DLT (h33' = 1) over the inliers: one
    // pass accumulates this thread's share of the 8 x 9 entries, then 72 block sums
    double acc[8][9];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int c = 0; c < 9; ++c) acc[a][c] = 0.0;
    for (int j = tid; j < K; j += HB) {
        if (!(reproj_err2(H, S[j], D[j]) <= thr2)) continue;
        const double x = (S[j].x - msx) * ks, y = (S[j].y - msy) * ks;
        const double u = (D[j].x - mdx) * kd, v = (D[j].y - mdy) * kd;
        const double r0[9] = {x, y, 1, 0, 0, 0, -u * x, -u * y, u};
        const double r1[9] = {0, 0, 0, x, y, 1, -v * x, -v * y, v};
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
            for (int c = 0; c < 9; ++c) acc[a][c] += r0[a] * r0[c] + r1[a] * r1[c];
    }
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int c = 0; c < 9; ++c) {
            const double s = block_sum(acc[a][c]);
            if (tid == 0) M[a][c] = s;
        }
    __syncthreads();
    if (tid == 0) {
        double A[8][8], b[8], h[8];
        for (int a = 0; a < 8; ++a) {
            for (int c = 0; c < 8; ++c) A[a][c] = M[a][c];
            b[a] = M[a][8];
        }
        if (solve_gauss<8>(A, b, h)) {
            // H = Td^-1 Hn Ts; Ts = [ks 0 -ks msx; 0 ks -ks msy; 0 0 1], Td likewise
            const double Hn[9] = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], 1.0};
            const double Ts[9] = {ks, 0, -ks * msx, 0, ks, -ks * msy, 0, 0, 1};
            const double Ti[9] = {1 / kd, 0, mdx, 0, 1 / kd, mdy, 0, 0, 1};
            double T1[9], T2[9];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    double s = 0;
                    for (int q = 0; q < 3; ++q) s += Hn[i * 3 + q] * Ts[q * 3 + j];
                    T1[i * 3 + j] = s;
                }
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    double s = 0;
                    for (int q = 0; q < 3; ++q) s += Ti[i * 3 + q] * T1[q * 3 + j];
                    T2[i * 3 + j] = s;
                }
            if (fabs(T2[8]) > 1e-300)
                for (int q = 0; q < 9; ++q) Hs[q] = T2[q] / T2[8];
        }
    }
    __syncthreads();
    for (int q = 0; q < 9; ++q) H[q] = Hs[q];
    double c2 = 0;
    for (int j = tid; j < K; j += HB) {
        const bool in = reproj_err2(H, S[j], D[j]) <= thr2;
        c2 += in;
        if (mask) mask[(size_t)p * cap + j] = in;
    }
    const double n_ref = block_sum(c2);
    if (tid == 0) {
        for (int q = 0; q < 9; ++q) r.H[q] = H[q];
        r.hyp_inliers = hv;
        r.inliers = (int)n_ref;
        r.status = PANO_OK;
        recs[p] = r;
    }
}

}  // namespace

int launch_pair_homography(pano_ctx *ctx, const pano_kp *kps, const int32_t *counts, int cap,
                           const int32_t *h_pairs, int n_pairs, const int32_t *best, const float *d1,
                           const float *d2, double desc_thresh, double ratio, double reproj_thr,
                           int n_hyp, unsigned long long seed, int min_good,
                           pano_homography_rec *recs, uint8_t *mask) {
    if (!kps || !counts || cap <= 0 || n_pairs <= 0 || !best || !d1 || (ratio > 0 && !d2) || !recs ||
        n_hyp < 1 || reproj_thr <= 0)
        return pano_fail(ctx, PANO_E_ARG, "pano_pair_homography: bad arguments");
    // ratio-test compaction (pano_pair_shifts' pair_compact), into this call's scratch
    const size_t mv_bytes = (size_t)n_pairs * cap * (sizeof(double2) + 2 * sizeof(int32_t)) +
                            (size_t)n_pairs * sizeof(int32_t) + 256;
    const size_t pt_bytes = 2 * (size_t)n_pairs * cap * sizeof(double2);
    const size_t sc_bytes = (size_t)n_pairs * n_hyp * sizeof(int32_t);
    int rc = pano_grow(ctx, &ctx->hmscratch, &ctx->hmscratch_bytes, mv_bytes + pt_bytes + sc_bytes + 512);
    if (rc) return rc;
    char *base = (char *)ctx->hmscratch;
    double2 *moves = (double2 *)base;
    int32_t *midx = (int32_t *)(moves + (size_t)n_pairs * cap);
    int32_t *kcount = midx + 2 * (size_t)n_pairs * cap;
    double2 *src = (double2 *)(base + ((mv_bytes + 255) & ~size_t(255)));
    double2 *dst = src + (size_t)n_pairs * cap;
    int32_t *score = (int32_t *)(dst + (size_t)n_pairs * cap);
    for (int p0 = 0; p0 < n_pairs; p0 += 256) {
        const int np = n_pairs - p0 < 256 ? n_pairs - p0 : 256;
        PairArg pa;
        for (int q = 0; q < np; ++q) {
            pa.a[q] = h_pairs[2 * (p0 + q)];
            pa.b[q] = h_pairs[2 * (p0 + q) + 1];
        }
        const size_t o = (size_t)p0 * cap;
        rc = launch_match_compact(ctx, kps, counts, cap, pa.a, pa.b, np, best + o, d1 + o,
                                  d2 ? d2 + o : nullptr, desc_thresh, ratio, moves + o, midx + o, kcount + p0);
        if (rc) return rc;
        {
            PanoProf prof_(ctx, PK_PAIR_SHIFTS);
            gather_points<<<dim3((cap + 255) / 256, np), 256, 0, ctx->stream>>>(
                kps, cap, pa, best + o, midx + o, kcount + p0, src + o, dst + o);
        }
        PANO_LAUNCH_CHECK(ctx, "gather_points");
        const double thr2 = reproj_thr * reproj_thr;
        {
            PanoProf prof_(ctx, PK_PAIR_SHIFTS);
            homography_hyp<<<dim3((n_hyp + HB - 1) / HB, np), HB, 0, ctx->stream>>>(
                src + o, dst + o, kcount + p0, cap, n_hyp, min_good, seed, thr2, score + (size_t)p0 * n_hyp, p0);
        }
        PANO_LAUNCH_CHECK(ctx, "homography_hyp");
        {
            PanoProf prof_(ctx, PK_PAIR_SHIFTS);
            homography_select<<<np, HB, 0, ctx->stream>>>(src + o, dst + o, kcount + p0, cap, n_hyp,
                                                          min_good, seed, thr2, score + (size_t)p0 * n_hyp,
                                                          counts, pa, recs + p0, mask ? mask + o : nullptr, p0);
        }
        PANO_LAUNCH_CHECK(ctx, "homography_select");
    }
    return PANO_OK;
}
