// match.hip -- M1 / H4: brute-force L2 nearest neighbour of descriptor rows.
//
//   SIFT  (image_stitching_sift.py:63-79): for each i, argmin_j ||dA_i - dB_j||^2 with a
//         strict '<' scan (first j wins ties).  Descriptors are integers in [0, 255], so
//         ||a||^2 + ||b||^2 - 2 a.b is an exact integer < 2^24 in f32 whatever the order:
//         the distance matrix is an MFMA GEMM with the argmin / second-min fused into the
//         epilogue.  Two exact variants:
//           bf16 (default, exact_int = 2): pack_rows -> bf16 rows + norms once per frame;
//                dist_bf16 loads MFMA fragments straight into registers (no LDS staging)
//                and runs v_mfma_f32_32x32x16_bf16 (integers 0..255 are exact in bf16);
//           f32  (exact_int = 1): dist_mfma, LDS-staged K chunks, v_mfma_f32_32x32x2_f32.
//   Harris (image_stitching_harris.py:219-240): float descriptors; numpy's np.dot(diff,
//         diff) is OpenBLAS sdot, whose summation order is reproduced exactly
//         (oracle/numerics.py::sdot_skx), one distance per thread.
//
// Workgroup tile: 128 (rows of A) x 128 (rows of B), 4 waves as 2 x 2, each wave 64 x 64 =
// 2 x 2 MFMA blocks of 32 x 32.  Per (row, column tile) the workgroup writes (best, index,
// second) partials; reduce_parts folds the column tiles in index order.
// Roofline unit M1 = 2*N*M*128 flop/pair.
#include "pano_internal.h"

#include <algorithm>

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int MT = 128;      // tile rows / cols
constexpr int KC = 32;       // K chunk
constexpr int LDA = KC + 1;  // padded LDS row (conflict-free column reads)

struct Part {
    float best;
    int32_t idx;
    float second;
};

__device__ __forceinline__ void merge(float &b, int &j, float &s, float b2, int j2, float s2) {
    if (b2 < b || (b2 == b && j2 < j)) {
        s = fminf(s2, b);
        b = b2;
        j = j2;
    } else {
        s = fminf(s, b2);
    }
}

__global__ void row_norms(const float *__restrict__ desc, const int32_t *__restrict__ counts,
                          int cap, int n_frames, float *__restrict__ norms) {
    const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (size_t)n_frames * cap) return;
    const float *d = desc + gid * PANO_DESC_DIM;
    float s = 0.0f;
    for (int k = 0; k < PANO_DESC_DIM; ++k) s = fmaf(d[k], d[k], s);   // exact: integers
    norms[gid] = s;
}

struct PairArg {
    int32_t a[256], b[256];
};

// Operand roles: C[j][i] = sum_k B[j][k] A[i][k], so in the 32 x 32 C layout (col = lane & 31,
// row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)) a lane owns ONE query row i and 16 candidate
// rows j: the argmin over j is a register fold, one lane^32 shuffle and one LDS merge of the
// two j-waves.  ELEM_BF16: the descriptors are staged as bf16 (exact for integers 0..255)
// and multiplied with v_mfma_f32_32x32x16_bf16 (K = 16 per issue, f32 accumulation exact
// below 2^24); otherwise v_mfma_f32_32x32x2_f32 in 4 K-chunks of 32.
typedef short bf16x8 __attribute__((ext_vector_type(8)));


__device__ __forceinline__ unsigned short f32_to_bf16_exact(float v) {
    return (unsigned short)(__float_as_uint(v) >> 16);   // exact for integers 0..255
}

__global__ void __launch_bounds__(256)
dist_mfma(const float *__restrict__ desc, const float *__restrict__ norms,
          const int32_t *__restrict__ counts, int cap, PairArg pairs, Part *__restrict__ parts,
          int n_jt) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ float nA[MT], nB[MT];
    __shared__ Part red[2][MT];
    const int p = blockIdx.z;
    const int fa = pairs.a[p], fb = pairs.b[p];
    int NA = counts[fa], NB = counts[fb];
    NA = min(max(NA, 0), cap);
    NB = min(max(NB, 0), cap);
    const int i0 = blockIdx.y * MT, j0 = blockIdx.x * MT;
    if (i0 >= NA || j0 >= NB) return;
    const float *dA = desc + (size_t)fa * cap * PANO_DESC_DIM;
    const float *dB = desc + (size_t)fb * cap * PANO_DESC_DIM;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wj = wv >> 1, wi = wv & 1;
    const int lr = lane & 31, lh = lane >> 5;
    if (tid < MT) nA[tid] = i0 + tid < NA ? norms[(size_t)fa * cap + i0 + tid] : 0.0f;
    else nB[tid - MT] = j0 + tid - MT < NB ? norms[(size_t)fb * cap + j0 + tid - MT] : 0.0f;
    f32x16 acc[2][2];   // [j block][i block]
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b)
            for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;

    {
        float *As = (float *)smem;          // [MT][LDA]
        float *Bs = As + MT * LDA;          // [MT][LDA]
        for (int k0 = 0; k0 < PANO_DESC_DIM; k0 += KC) {
            for (int q = tid; q < MT * KC / 4; q += 256) {
                const int row = q / (KC / 4), c4 = (q % (KC / 4)) * 4;
                float4 va = make_float4(0.f, 0.f, 0.f, 0.f), vb = va;
                if (i0 + row < NA) va = *(const float4 *)(dA + (size_t)(i0 + row) * PANO_DESC_DIM + k0 + c4);
                if (j0 + row < NB) vb = *(const float4 *)(dB + (size_t)(j0 + row) * PANO_DESC_DIM + k0 + c4);
                float *pa = As + row * LDA + c4;
                float *pb = Bs + row * LDA + c4;
                pa[0] = va.x; pa[1] = va.y; pa[2] = va.z; pa[3] = va.w;
                pb[0] = vb.x; pb[1] = vb.y; pb[2] = vb.z; pb[3] = vb.w;
            }
            __syncthreads();
#pragma unroll 4
            for (int kk = 0; kk < KC; kk += 2) {
                float fj[2], fi[2];
                for (int m = 0; m < 2; ++m) {
                    fj[m] = Bs[(wj * 64 + m * 32 + lr) * LDA + kk + lh];
                    fi[m] = As[(wi * 64 + m * 32 + lr) * LDA + kk + lh];
                }
                for (int a = 0; a < 2; ++a)
                    for (int b = 0; b < 2; ++b)
                        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(fj[a], fi[b], acc[a][b], 0, 0, 0);
            }
            __syncthreads();
        }
    }
    __syncthreads();
    // epilogue: per i (= lane & 31 of i block b), fold the wave's 64 j values
    for (int b = 0; b < 2; ++b) {
        const int il = wi * 64 + b * 32 + lr;          // tile-local i
        const float na = nA[il];
        float best = INFINITY, second = INFINITY;
        int bj = 0x7fffffff;
        for (int a = 0; a < 2; ++a) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int jl = wj * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
                if (j0 + jl < NB) {
                    const float d = (na + nB[jl]) - 2.0f * acc[a][b][r];
                    merge(best, bj, second, d, j0 + jl, INFINITY);
                }
            }
        }
        const float ob = __shfl_xor(best, 32);
        const int oj = __shfl_xor(bj, 32);
        const float os = __shfl_xor(second, 32);
        merge(best, bj, second, ob, oj, os);
        if (lh == 0) red[wj][il] = Part{best, bj, second};
    }
    __syncthreads();
    if (tid < MT) {
        Part x = red[0][tid];
        const Part y = red[1][tid];
        float bb = x.best, ss = x.second;
        int jj = x.idx;
        merge(bb, jj, ss, y.best, y.idx, y.second);
        const int gi = i0 + tid;
        if (gi < NA) parts[((size_t)p * n_jt + blockIdx.x) * cap + gi] = Part{bb, jj, ss};
    }
}

// ---------------------------------------------------------------- bf16 path (default)
// The distance is folded into the GEMM: with K extended from 128 to KA = 144 (one more
// 32x32x16 MFMA step), query rows are packed as  A' = [ a | 65536, 256, 1, 0 ... ]  and
// candidate rows as  B' = [ -2 b | c2, c1, c0, 0 ... ]  where ||b||^2 = c2 65536 + c1 256 + c0,
// so C = A'.B' = ||b||^2 - 2 a.b.  Every entry is a bf16-exact integer (|2b| <= 510 has 8
// significant bits, c* < 256, powers of two) and every partial sum is an integer < 2^21, so
// the f32 MFMA accumulation is exact in any order; ||a - b||^2 = ||a||^2 + C exactly, and the
// epilogue is a bare compare / select per element (||a||^2 is constant along the argmin).
// Rows past a frame's count (up to the 128-row padded stride) are packed as b = 0 with
// ||b||^2 = 2^22: never a best, and a second-best that large means "none" (reduce_parts).
constexpr int KA = 144;              // augmented K
constexpr int KS = KA / 16;          // MFMA K steps
constexpr float kPadNorm = 4194304.0f;

__device__ __forceinline__ unsigned short bf16_of_int(int v) {     // exact for |v| < 2^9
    return (unsigned short)(__float_as_uint((float)v) >> 16);
}

// 16 threads per row, 9 bf16 columns each (thread 15 also writes the augmentation).
__global__ void __launch_bounds__(256)
pack_rows(const float *__restrict__ desc, const int32_t *__restrict__ counts, int cap, int capP,
          int n_frames, unsigned short *__restrict__ pa, unsigned short *__restrict__ pb,
          float *__restrict__ norms) {
    const size_t gid = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t row = gid >> 4;
    const int part = (int)(gid & 15);
    if (row >= (size_t)n_frames * capP) return;
    const int f = (int)(row / capP), r = (int)(row % capP);
    int cnt = counts[f];
    cnt = min(max(cnt, 0), cap);
    const bool live = r < cnt;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    if (live) {
        const float4 *src = (const float4 *)(desc + ((size_t)f * cap + r) * PANO_DESC_DIM + part * 8);
        a = src[0];
        b = src[1];
    }
    float s = a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w + b.x * b.x + b.y * b.y + b.z * b.z +
              b.w * b.w;                                  // integers: exact in any order
    for (int d = 8; d > 0; d >>= 1) s += __shfl_xor(s, d, 16);
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    unsigned short ua[8], ub[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        ua[k] = f32_to_bf16_exact(v[k]);
        ub[k] = bf16_of_int(-2 * (int)v[k]);
    }
    unsigned short *da = pa + row * KA + part * 8, *db = pb + row * KA + part * 8;
    *(uint4 *)da = make_uint4(ua[0] | ua[1] << 16, ua[2] | ua[3] << 16, ua[4] | ua[5] << 16, ua[6] | ua[7] << 16);
    *(uint4 *)db = make_uint4(ub[0] | ub[1] << 16, ub[2] | ub[3] << 16, ub[4] | ub[5] << 16, ub[6] | ub[7] << 16);
    if (part == 0) {
        const int nb = live ? (int)s : (int)kPadNorm;
        unsigned short ta[16] = {}, tb[16] = {};
        ta[0] = (unsigned short)(__float_as_uint(65536.0f) >> 16);
        ta[1] = (unsigned short)(__float_as_uint(256.0f) >> 16);
        ta[2] = (unsigned short)(__float_as_uint(1.0f) >> 16);
        tb[0] = (nb >> 16) ? (unsigned short)(__float_as_uint((float)(nb >> 16)) >> 16) : 0;
        tb[1] = (unsigned short)(__float_as_uint((float)((nb >> 8) & 255)) >> 16);
        tb[2] = (unsigned short)(__float_as_uint((float)(nb & 255)) >> 16);
        uint4 *qa = (uint4 *)(pa + row * KA + 128), *qb = (uint4 *)(pb + row * KA + 128);
        for (int h = 0; h < 2; ++h) {
            qa[h] = make_uint4(ta[8 * h] | ta[8 * h + 1] << 16, ta[8 * h + 2] | ta[8 * h + 3] << 16,
                               ta[8 * h + 4] | ta[8 * h + 5] << 16, ta[8 * h + 6] | ta[8 * h + 7] << 16);
            qb[h] = make_uint4(tb[8 * h] | tb[8 * h + 1] << 16, tb[8 * h + 2] | tb[8 * h + 3] << 16,
                               tb[8 * h + 4] | tb[8 * h + 5] << 16, tb[8 * h + 6] | tb[8 * h + 7] << 16);
        }
        norms[row] = live ? s : 0.0f;
    }
}

// dist_bf16: workgroup = 128 query rows (4 waves as 2 (j) x 2 (i), each 64 x 64 = 2 x 2
// v_mfma_f32_32x32x16_bf16 blocks).  The query fragments stay in registers while the
// workgroup walks candidate tiles split, split + n_split, ... (the next tile's fragments are
// loaded while the current one is folded), so the partials are n_split per row, not one per
// tile.  Per element the fold is compare / select (plus min / max when SECOND).
template <bool SECOND>
__global__ void __launch_bounds__(256)
dist_bf16(const unsigned short *__restrict__ pa, const unsigned short *__restrict__ pb,
          const float *__restrict__ norms, const int32_t *__restrict__ counts, int cap, int capP,
          PairArg pairs, Part *__restrict__ parts, int n_split) {
    __shared__ Part red[2][MT];
    const int p = blockIdx.z;
    const int fa = pairs.a[p], fb = pairs.b[p];
    int NA = counts[fa], NB = counts[fb];
    NA = min(max(NA, 0), cap);
    NB = min(max(NB, 0), cap);
    const int i0 = blockIdx.y * MT;
    const int n_jt = (NB + MT - 1) / MT;
    if (i0 >= NA || (int)blockIdx.x >= n_jt) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wj = wv >> 1, wi = wv & 1;
    const int lr = lane & 31, lh = lane >> 5;
    const unsigned short *rA = pa + (size_t)fa * capP * KA;
    const unsigned short *rB = pb + (size_t)fb * capP * KA;
    bf16x8 fi[2][KS], fj[2][KS];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        const bf16x8 *qi = (const bf16x8 *)(rA + (size_t)(i0 + wi * 64 + m * 32 + lr) * KA + 8 * lh);
#pragma unroll
        for (int k = 0; k < KS; ++k) fi[m][k] = qi[2 * k];
    }
    auto load_b = [&](int jt) {
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const bf16x8 *qj = (const bf16x8 *)(rB + (size_t)(jt * MT + wj * 64 + m * 32 + lr) * KA + 8 * lh);
#pragma unroll
            for (int k = 0; k < KS; ++k) fj[m][k] = qj[2 * k];
        }
    };
    float best[2] = {INFINITY, INFINITY}, second[2] = {INFINITY, INFINITY};
    int bj[2] = {0x7fffffff, 0x7fffffff};
    int jt = blockIdx.x;
    load_b(jt);
    for (; jt < n_jt; jt += n_split) {
        f32x16 acc[2][2];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;
#pragma unroll
        for (int k = 0; k < KS; ++k)
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fj[a][k], fi[b][k], acc[a][b], 0, 0, 0);
        if (jt + n_split < n_jt) load_b(jt + n_split);      // in flight during the fold
        const int jb = jt * MT + wj * 64 + 4 * lh;
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int r = 0; r < 16; ++r) {   // j increasing within the lane: strict <
                    const float d = acc[a][b][r];
                    if (SECOND) second[b] = fminf(second[b], fmaxf(best[b], d));
                    const bool lt = d < best[b];
                    bj[b] = lt ? jb + a * 32 + (r & 3) + 8 * (r >> 2) : bj[b];
                    best[b] = lt ? d : best[b];
                }
    }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const float ob = __shfl_xor(best[b], 32);
        const int oj = __shfl_xor(bj[b], 32);
        const float os = __shfl_xor(second[b], 32);
        merge(best[b], bj[b], second[b], ob, oj, os);
        const int il = wi * 64 + b * 32 + lr;
        if (lh == 0) red[wj][il] = Part{best[b], bj[b], second[b]};
    }
    __syncthreads();
    if (tid < MT) {
        Part x = red[0][tid];
        const Part y = red[1][tid];
        float bb = x.best, ss = x.second;
        int jj = x.idx;
        merge(bb, jj, ss, y.best, y.idx, y.second);
        const int gi = i0 + tid;
        if (gi < NA) {
            const float na = norms[(size_t)fa * capP + gi];
            parts[((size_t)p * n_split + blockIdx.x) * cap + gi] = Part{na + bb, jj, na + ss};
        }
    }
}

// ---------------------------------------------------------------- u8 path (the Stitcher's)
// Descriptors as bytes [frames][cap][128] with exact squared norms (pano_sift_u8), so nothing
// is repacked between the descriptor kernel and the GEMM.  Workgroup = 256 query rows
// (8 waves: 4 row groups of 64 x 2 candidate halves of 64); every 128-row candidate tile is
// converted ONCE into LDS as the augmented bf16 row [b | c2, c1, c0, 0...] and read by all
// 256 query rows (the register-fragment form re-streamed each candidate row from L2 once per
// 128 query rows).  The next tile's bytes are in flight in registers while the current tile
// is multiplied.  Query fragments [-2 a | 65536, 256, 1, 0...] (|2a| <= 510: 8 significant
// bits, exact in bf16) are converted from bytes once, in registers, so C = ||b||^2 - 2 a.b
// exactly, as in dist_bf16.  Per element the fold is one min (the index is searched only
// when a 16-element block beats the running best), or compare / select with min / max when
// the second-best distance is wanted.
constexpr int QT = 256;              // query rows per workgroup
constexpr int BT = 128;              // candidate rows per LDS tile
constexpr int BKP = KA + 8;          // LDS row pitch (bf16): 304 B, rows 12 banks apart

__device__ __forceinline__ unsigned int bf16x2_of_ints(int v0, int v1) {
    // bf16 of small integers (8 significant bits): their f32 bits >> 16, exact
    return (__float_as_uint((float)v0) >> 16) | (__float_as_uint((float)v1) & 0xffff0000u);
}
// the four bytes of x as two dwords of bf16 pairs (v_cvt_f32_ubyte0..3 + two byte permutes)
__device__ __forceinline__ void bf16x4_of_u8x4(unsigned int x, unsigned int &lo, unsigned int &hi) {
    const float f0 = (float)(x & 255u), f1 = (float)((x >> 8) & 255u);     // v_cvt_f32_ubyte*
    const float f2 = (float)((x >> 16) & 255u), f3 = (float)(x >> 24);
    // selector 0x07060302: bytes 2, 3 of the second operand, then bytes 2, 3 of the first
    lo = __builtin_amdgcn_perm(__float_as_uint(f1), __float_as_uint(f0), 0x07060302u);
    hi = __builtin_amdgcn_perm(__float_as_uint(f3), __float_as_uint(f2), 0x07060302u);
}

template <bool SECOND>
__global__ void __launch_bounds__(512, 2)
dist_u8(const uint8_t *__restrict__ desc, const int32_t *__restrict__ norms,
        const int32_t *__restrict__ counts, int cap, PairArg pairs, Part *__restrict__ parts,
        int n_split) {
    __shared__ __attribute__((aligned(16))) unsigned short Bs2[2][BT * BKP];   // double buffer
    __shared__ Part red[2][QT];
    const int p = blockIdx.y;             // grid (split, pair, query tile): see launch_match_u8
    const int fa = pairs.a[p], fb = pairs.b[p];
    int NA = counts[fa], NB = counts[fb];
    NA = min(max(NA, 0), cap);
    NB = min(max(NB, 0), cap);
    const int i0 = blockIdx.z * QT;
    const int n_jt = (NB + BT - 1) / BT;
    if (i0 >= NA || (int)blockIdx.x >= n_jt) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wi = wv & 3, wj = wv >> 2;
    const int lr = lane & 31, lh = lane >> 5;
    const uint8_t *dA = desc + (size_t)fa * cap * PANO_DESC_DIM;
    const uint8_t *dB = desc + (size_t)fb * cap * PANO_DESC_DIM;
    // ---- query fragments, converted once: rows i0 + wi 64 + m 32 + lr, K step k holds
    // elements 16 k + 8 lh .. + 8
    bf16x8 fi[2][KS];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        const int row = i0 + wi * 64 + m * 32 + lr;
        const bool live = row < NA;
#pragma unroll
        for (int k = 0; k < KS - 1; ++k) {
            uint2 v = make_uint2(0u, 0u);
            if (live) v = *(const uint2 *)(dA + (size_t)row * PANO_DESC_DIM + 16 * k + 8 * lh);
            const unsigned int w[4] = {bf16x2_of_ints(-2 * (int)(v.x & 255), -2 * (int)((v.x >> 8) & 255)),
                                       bf16x2_of_ints(-2 * (int)((v.x >> 16) & 255), -2 * (int)(v.x >> 24)),
                                       bf16x2_of_ints(-2 * (int)(v.y & 255), -2 * (int)((v.y >> 8) & 255)),
                                       bf16x2_of_ints(-2 * (int)((v.y >> 16) & 255), -2 * (int)(v.y >> 24))};
            fi[m][k] = *(const bf16x8 *)w;
        }
        // augmentation [65536, 256, 1, 0, ...] on the lh = 0 half of the last K step
        const unsigned int a0 = (__float_as_uint(65536.0f) >> 16) | (__float_as_uint(256.0f) & 0xffff0000u);
        const unsigned int a1 = __float_as_uint(1.0f) >> 16;
        const unsigned int w[4] = {lh ? 0u : a0, lh ? 0u : a1, 0u, 0u};
        fi[m][KS - 1] = *(const bf16x8 *)w;
    }
    // ---- candidate tile staging: thread t converts row t % 128, bytes 32 (t / 128) .. + 32
    // (a wave writes 64 consecutive rows at one offset: rows 12 banks apart, conflict free)
    const int sr = tid & (BT - 1), sp = tid / BT;
    uint4 pre[2];
    int pre_norm = 0;
    auto fetch = [&](int jt) {
        const int row = jt * BT + sr;
        pre[0] = pre[1] = make_uint4(0u, 0u, 0u, 0u);
        pre_norm = (int)kPadNorm;               // past the count: never a best (reduce_parts)
        if (row < NB) {
            const uint4 *src = (const uint4 *)(dB + (size_t)row * PANO_DESC_DIM + 32 * sp);
            pre[0] = src[0];
            pre[1] = src[1];
            pre_norm = norms[(size_t)fb * cap + row];
        }
    };
    auto store = [&](unsigned short *Bs) {
        unsigned short *dst = Bs + sr * BKP + 32 * sp;
        const unsigned int *u = (const unsigned int *)pre;
        unsigned int o[16];
#pragma unroll
        for (int q = 0; q < 8; ++q) bf16x4_of_u8x4(u[q], o[2 * q], o[2 * q + 1]);
        uint4 *d4 = (uint4 *)dst;
#pragma unroll
        for (int q = 0; q < 4; ++q) d4[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
        if (sp == 0) {
            const int nb = pre_norm;                // ||b||^2 = c2 65536 + c1 256 + c0
            const unsigned int t0 = bf16x2_of_ints(nb >> 16, (nb >> 8) & 255);
            const unsigned int t1 = bf16x2_of_ints(nb & 255, 0);
            uint4 *aug = (uint4 *)(Bs + sr * BKP + 128);
            aug[0] = make_uint4(t0, t1, 0u, 0u);
            aug[1] = make_uint4(0u, 0u, 0u, 0u);
        }
    };
    float best[2] = {INFINITY, INFINITY}, second[2] = {INFINITY, INFINITY};
    int bj[2] = {0x7fffffff, 0x7fffffff};
    // Two LDS tiles: the MFMAs of tile t read one while the next tile (its bytes prefetched
    // into registers a tile earlier) is converted into the other, so the conversion VALU and
    // LDS stores run under the MFMAs, and one barrier per tile suffices.  (One workgroup per
    // CU: 180 VGPRs per lane allow two waves per SIMD.)
    int jt = blockIdx.x, cur = 0;
    fetch(jt);
    store(Bs2[0]);
    if (jt + n_split < n_jt) fetch(jt + n_split);
    for (; jt < n_jt; jt += n_split, cur ^= 1) {
        __syncthreads();        // tile jt complete in Bs2[cur]; every wave done with Bs2[cur ^ 1]
        const unsigned short *Bs = Bs2[cur];
        f32x16 acc[2][2];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;
#pragma unroll
        for (int k = 0; k < KS; ++k) {
            bf16x8 fj[2];
#pragma unroll
            for (int a = 0; a < 2; ++a)
                fj[a] = *(const bf16x8 *)(Bs + (wj * 64 + a * 32 + lr) * BKP + 16 * k + 8 * lh);
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fj[a], fi[b][k], acc[a][b], 0, 0, 0);
        }
        if (jt + n_split < n_jt) {
            store(Bs2[cur ^ 1]);
            if (jt + 2 * n_split < n_jt) fetch(jt + 2 * n_split);   // in flight for a tile
        }
        const int jb = jt * BT + wj * 64 + 4 * lh;
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                if (SECOND) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) {   // j increasing within the lane: strict <
                        const float d = acc[a][b][r];
                        second[b] = fminf(second[b], fmaxf(best[b], d));
                        const bool lt = d < best[b];
                        bj[b] = lt ? jb + a * 32 + (r & 3) + 8 * (r >> 2) : bj[b];
                        best[b] = lt ? d : best[b];
                    }
                } else {
                    // the block's minimum first (one op per element); its index only when it
                    // beats the running best, which happens ~ln(#blocks) times per row
                    float m = acc[a][b][0];
#pragma unroll
                    for (int r = 1; r < 16; ++r) m = fminf(m, acc[a][b][r]);
                    if (m < best[b]) {
                        int ri = 15;
#pragma unroll
                        for (int r = 14; r >= 0; --r) ri = acc[a][b][r] == m ? r : ri;   // first r
                        best[b] = m;
                        bj[b] = jb + a * 32 + (ri & 3) + 8 * (ri >> 2);
                    }
                }
            }
    }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const float ob = __shfl_xor(best[b], 32);
        const int oj = __shfl_xor(bj[b], 32);
        const float os = __shfl_xor(second[b], 32);
        merge(best[b], bj[b], second[b], ob, oj, os);
        const int il = wi * 64 + b * 32 + lr;
        if (lh == 0) red[wj][il] = Part{best[b], bj[b], second[b]};
    }
    __syncthreads();
    if (tid < QT) {
        Part x = red[0][tid];
        const Part y = red[1][tid];
        float bb = x.best, ss = x.second;
        int jj = x.idx;
        merge(bb, jj, ss, y.best, y.idx, y.second);
        const int gi = i0 + tid;
        if (gi < NA) {
            const float na = (float)norms[(size_t)fa * cap + gi];
            parts[((size_t)p * n_split + blockIdx.x) * cap + gi] = Part{na + bb, jj, na + ss};
        }
    }
}

// ---------------------------------------------------------------- i8 MFMA path (default)
// The descriptor bytes enter the i8 MFMA as b' = b - 128 (b ^ 0x80 read as int8), so no
// conversion at all, at twice the bf16 MFMA rate and K = 128 exactly (no augmentation):
//   a.b = a'.b' + 128 (sum a' + sum b') + 128^3,  sum a' = s_a - 128^2  (s = byte sum)
//   d(i, j) = ||a_i||^2 + ||b_j||^2 - 2 a.b = R_i + C_j - 2 a'.b',
//   R = ||a||^2 - 256 s_a,  C = ||b||^2 - 256 s_b + 2^22
// with a'.b' accumulated exactly in i32 (|a'.b'| <= 2^21): every distance is the exact
// integer the reference's np.dot gives, compared as integers (first index on ties).
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
constexpr int BPI = PANO_DESC_DIM + 16;          // LDS row pitch in bytes (rows 36 banks apart)
constexpr int kBig = 0x3fffffff;                 // "no distance" (padding rows, empty pairs)
// Packed distance keys: key = 32 (C_j - 2 a'.b') + idx(j), idx = the candidate's rank among
// the 32 rows one lane reads per tile (monotone in j).  One v_mad_i32_i24 forms the key from
// the accumulator and C32[j] = 32 C_j + idx(j) (LDS), so min / med3 on keys give the least
// distance with the first index, and the second-least distance, in one VALU op each.
// |32 (C - 2 a'.b')| < 2^29 + 2^27 for real rows; padding rows carry C = kPadC, whose keys
// (>= 2^30 - 2^27) never beat a real one; decoded distances >= kNone mean "no candidate".
constexpr int kPadC = 1 << 25;
constexpr int kNone = kPadC - (1 << 22);
__device__ __forceinline__ int key_idx(int j) { return ((j >> 5) & 1) * 16 + ((j >> 3) & 3) * 4 + (j & 3); }
__device__ __forceinline__ int med3_i32(int a, int b, int c) {
    int r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// c + a * b in one VALU op (|a|, |b| < 2^23 here: a'.b' is within +-2^21); b in an SGPR
// (-64 is not an inline constant, and VOP3 takes no literal)
__device__ __forceinline__ int mad_i24(int a, int b, int c) {
    int r;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(c));
    return r;
}

// R per descriptor row (rows past the frame's count: unused)
__global__ void __launch_bounds__(256)
row_consts(const uint8_t *__restrict__ desc, const int32_t *__restrict__ norms,
           const int32_t *__restrict__ counts, int cap, int32_t *__restrict__ cst) {
    const int f = blockIdx.x, row = blockIdx.y * 64 + (threadIdx.x >> 2), part = threadIdx.x & 3;   // (frame, block)
    const int n = min(max(counts[f], 0), cap);
    unsigned int sum = 0;
    if (row < n) {
        const uint4 *q = (const uint4 *)(desc + ((size_t)f * cap + row) * PANO_DESC_DIM + 32 * part);
        const uint4 v0 = q[0], v1 = q[1];
        const unsigned int w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) sum = __builtin_amdgcn_udot4(w[i], 0x01010101u, sum, false);
    }
    sum += __shfl_xor(sum, 1);
    sum += __shfl_xor(sum, 2);
    if (row < n && part == 0) cst[(size_t)f * cap + row] = norms[(size_t)f * cap + row] - 256 * (int)sum;
}

#ifndef PANO_I8_QLDS
#define PANO_I8_QLDS 1                   // query tile in LDS (0: in registers)
#endif
#ifndef PANO_I8_ABL
#define PANO_I8_ABL 0                    // timing ablations of the epilogue (wrong results): 1, 2
#endif
#ifndef PANO_I8_DBL
#define PANO_I8_DBL 0                    // 1: two accumulator sets per wave (epilogue beside the next MFMAs)
#endif
#ifndef PANO_I8_STAGGER
#define PANO_I8_STAGGER 1                // waves 4-7 run each tile's epilogue one barrier late
#endif
#ifndef PANO_I8_PRIO
#define PANO_I8_PRIO 0                   // 1: waves 4-7 at s_setprio 1 for the whole loop
#endif
#ifndef PANO_I8_WAVES
#define PANO_I8_WAVES 4                  // 4 waves per SIMD (two workgroups per CU): measured 2.87 -> 2.57 ms at 1080p
#endif
// The per-row constants R = |a|^2 - 256 sum(a) (query rows) and C = |b|^2 - 256 sum(b)
// (candidate rows) are formed while the rows are staged: the lanes staging one row sum its
// bytes with v_dot4_u32_u8 and a shuffle reduction (no separate row_consts launch; with
// PANO_I8_QLDS=0 the query rows stay in registers and row_consts still runs).
typedef __attribute__((address_space(1))) int g_i32;
typedef __attribute__((address_space(1))) float g_f32;

// reduce_parts folded into dist_i8 (fold != null): each workgroup stores its partial rows
// write-through (sc1), drains them (s_waitcnt vmcnt(0), barrier) and counts itself in on its
// (pair, query tile) with one device-scope add; the last of the tile's live splits reads every
// split's partials back with sc1 loads (MI355X guide, visibility, R1: no fence), merges them in
// split order -- reduce_parts' arithmetic -- writes best / d1 / d2 and re-zeroes the counter.
// Query tiles with no live split (past the count, or no candidates) get reduce_parts' "no
// candidate" rows from their split-0 workgroup.
struct MatchFold {
    int32_t *cnt;                        // [pair][query tile] arrivals (zero between launches)
    int32_t *best;
    float *d1, *d2;
};

template <bool SECOND>
__global__ void __launch_bounds__(512, PANO_I8_WAVES)
dist_i8(const uint8_t *__restrict__ desc, const int32_t *__restrict__ norms, const int32_t *__restrict__ cst,
        const int32_t *__restrict__ counts, int cap, PairArg pairs, Part *__restrict__ parts,
        int n_split, MatchFold fold) {
    __shared__ __attribute__((aligned(16))) unsigned char Bs2[2][BT * BPI];
    __shared__ __attribute__((aligned(16))) int Cs2[3][BT];   // C32 of tile t in Cs2[t % 3] (a lagging epilogue reads t - 1)
#if PANO_I8_QLDS
    // the query tile (B operand of every MFMA) in LDS, sign-flipped once: read per tile
    // instead of held in 32 VGPRs (register pressure spilled the staging state to scratch
    // inside the tile loop)
    __shared__ __attribute__((aligned(16))) unsigned char Qs[QT * BPI];
    // R of query row r sits in the row's pitch padding (bytes 128..131), so the workgroup's
    // LDS stays within half a CU (two workgroups per CU)
    auto rq = [&](int r) -> int & { return *(int *)(Qs + r * BPI + PANO_DESC_DIM); };
#endif
    struct IPart { int best, idx, second; };
    __shared__ IPart red[2][QT];
    const int p = blockIdx.y;             // grid (split, pair, query tile): see launch_match_u8
    const int fa = pairs.a[p], fb = pairs.b[p];
    int NA = counts[fa], NB = counts[fb];
    NA = min(max(NA, 0), cap);
    NB = min(max(NB, 0), cap);
    const int i0 = blockIdx.z * QT;
    const int n_jt = (NB + BT - 1) / BT;
    if (i0 >= NA || (int)blockIdx.x >= n_jt) {
        if (fold.cnt && blockIdx.x == 0 && (i0 >= NA || n_jt == 0)) {
            for (int t = threadIdx.x; t < QT && i0 + t < cap; t += 512) {
                const size_t o = (size_t)p * cap + i0 + t;
                fold.best[o] = -1;
                fold.d1[o] = INFINITY;
                if (fold.d2) fold.d2[o] = INFINITY;
            }
        }
        return;
    }
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wi = wv & 3, wj = wv >> 2;
    const int lr = lane & 31, lh = lane >> 5;
    const uint8_t *dA = desc + (size_t)fa * cap * PANO_DESC_DIM;
    const uint8_t *dB = desc + (size_t)fb * cap * PANO_DESC_DIM;
    // query fragments (B operand): rows i0 + wi 64 + m 32 + lr, K step k = bytes 32 k + 16 lh
#if PANO_I8_QLDS
    for (int e = tid; e < QT * (PANO_DESC_DIM / 16); e += 512) {   // 16-byte pieces, 8 lanes a row
        const int r = e >> 3, q = e & 7, row = i0 + r;
        uint4 v = make_uint4(0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u);
        if (row < NA) v = *(const uint4 *)(dA + (size_t)row * PANO_DESC_DIM + 16 * q);
        *(uint4 *)(Qs + r * BPI + 16 * q) = make_uint4(v.x ^ 0x80808080u, v.y ^ 0x80808080u,
                                                       v.z ^ 0x80808080u, v.w ^ 0x80808080u);
        unsigned int sum = 0;
        sum = __builtin_amdgcn_udot4(v.x, 0x01010101u, sum, false);
        sum = __builtin_amdgcn_udot4(v.y, 0x01010101u, sum, false);
        sum = __builtin_amdgcn_udot4(v.z, 0x01010101u, sum, false);
        sum = __builtin_amdgcn_udot4(v.w, 0x01010101u, sum, false);
        sum += __shfl_xor(sum, 1);
        sum += __shfl_xor(sum, 2);
        sum += __shfl_xor(sum, 4);
        if (q == 0 && row < NA) rq(r) = norms[(size_t)fa * cap + row] - 256 * (int)sum;
    }
    auto qfrag = [&](int m, int k) {
        return *(const i32x4 *)(Qs + (wi * 64 + m * 32 + lr) * BPI + 32 * k + 16 * lh);
    };
#else
    i32x4 fi[2][4];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        const int row = i0 + wi * 64 + m * 32 + lr;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint4 v = make_uint4(0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u);
            if (row < NA) v = *(const uint4 *)(dA + (size_t)row * PANO_DESC_DIM + 32 * k + 16 * lh);
            fi[m][k] = i32x4{(int)(v.x ^ 0x80808080u), (int)(v.y ^ 0x80808080u), (int)(v.z ^ 0x80808080u),
                             (int)(v.w ^ 0x80808080u)};
        }
    }
    auto qfrag = [&](int m, int k) { return fi[m][k]; };
#endif
    // candidate tile staging: four adjacent lanes copy one row (thread t: row t / 4, bytes
    // 32 (t % 4) .. + 32), with the sign flip; the row's C from their byte sums
#if PANO_I8_QLDS
    const int sr = tid >> 2, sp = tid & 3;
#else
    const int sr = tid & (BT - 1), sp = tid / BT;
#endif
    // fetch only issues the loads (the next tile's, a tile ahead); store, one tile later,
    // forms C from them, so no wait on a load sits right behind its issue
    uint4 pre[2];
    int pre_c = kPadC;
    auto fetch = [&](int jt) {
        const int row = jt * BT + sr;
        pre[0] = pre[1] = make_uint4(0u, 0u, 0u, 0u);
        pre_c = kPadC;                                  // past the count: never a best
        if (row < NB) {
            const uint4 *src = (const uint4 *)(dB + (size_t)row * PANO_DESC_DIM + 32 * sp);
            pre[0] = src[0];
            pre[1] = src[1];
#if PANO_I8_QLDS
            pre_c = norms[(size_t)fb * cap + row];      // |b|^2; the byte sum is taken in store
#else
            if (sp == 0) pre_c = cst[(size_t)fb * cap + row] + (1 << 22);
#endif
        }
    };
    auto store = [&](int buf, int cbuf) {
#if PANO_I8_QLDS
        unsigned int sum = 0;
        const unsigned int w[8] = {pre[0].x, pre[0].y, pre[0].z, pre[0].w, pre[1].x, pre[1].y, pre[1].z, pre[1].w};
#pragma unroll
        for (int i = 0; i < 8; ++i) sum = __builtin_amdgcn_udot4(w[i], 0x01010101u, sum, false);
        sum += __shfl_xor(sum, 1);
        sum += __shfl_xor(sum, 2);
        if (pre_c != kPadC) pre_c = pre_c - 256 * (int)sum + (1 << 22);
#endif
        uint4 *d4 = (uint4 *)(Bs2[buf] + sr * BPI + 32 * sp);
#pragma unroll
        for (int q = 0; q < 2; ++q)
            d4[q] = make_uint4(pre[q].x ^ 0x80808080u, pre[q].y ^ 0x80808080u, pre[q].z ^ 0x80808080u,
                               pre[q].w ^ 0x80808080u);
        if (sp == 0) Cs2[cbuf][sr] = PANO_I8_DBL ? -(pre_c * 32 + key_idx(sr))   // -C32: max form
                                                 : pre_c * 32 + key_idx(sr);     // C32: the key's base
    };
    int best[2] = {kBig, kBig}, second[2] = {kBig, kBig};
    int bj[2] = {0x7fffffff, 0x7fffffff};
    i32x16 acc[2][2];
    // the epilogue of one tile: its least / second-least key per query row folded into the
    // running state (keys are unique per lane; tiles come in increasing j, so strict < keeps
    // the first index on a tie)
    auto epilogue = [&](const i32x16 (&acc)[2][2], const int *Cs, int jt_e) {
        const int jb = jt_e * BT + wj * 64 + 4 * lh;
#if PANO_I8_DBL
        // negated keys -key = 64 a'.b' - C32 = (acc << 6) + (-C32): ONE v_lshl_add_u32 (a plain
        // op the scheduler can place between MFMAs), folded with max / med3
        int tb[2] = {(int)0x80000000, (int)0x80000000}, ts[2] = {(int)0x80000000, (int)0x80000000};
#else
        int tb[2] = {0x7fffffff, 0x7fffffff}, ts[2] = {0x7fffffff, 0x7fffffff};
#endif
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            // C32 of this lane's 16 candidate rows: rows (r & 3) + 8 (r >> 2) + 4 lh of block a
            int cj[16];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int4 c4 = *(const int4 *)(&Cs[wj * 64 + a * 32 + 8 * g + 4 * lh]);
                cj[4 * g] = c4.x; cj[4 * g + 1] = c4.y; cj[4 * g + 2] = c4.z; cj[4 * g + 3] = c4.w;
            }
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
#if PANO_I8_ABL == 1                                       // timing ablation: 1 VALU op per distance
                    tb[b] = min(tb[b], acc[a][b][r]);
                    continue;
#elif PANO_I8_ABL == 2                                     // timing ablation: no epilogue VALU
                    if (r == 0) tb[b] = min(tb[b], acc[a][b][0] + cj[0]);
                    continue;
#endif
#if PANO_I8_DBL
                    const int nkey = (int)(((unsigned)acc[a][b][r] << 6) + (unsigned)cj[r]);
                    if (SECOND) ts[b] = med3_i32(tb[b], nkey, ts[b]);
                    tb[b] = max(tb[b], nkey);
#else
                    const int key = mad_i24(acc[a][b][r], -64, cj[r]);
                    if (SECOND) ts[b] = med3_i32(tb[b], key, ts[b]);
                    tb[b] = min(tb[b], key);
#endif
                }
        }
#if PANO_I8_DBL
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            tb[b] = -tb[b];
            ts[b] = -ts[b];
        }
#endif
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int d1 = tb[b] >> 5, idx = tb[b] & 31;   // arithmetic shift: floor(key / 32)
            const int j = jb + (idx >> 4) * 32 + ((idx >> 2) & 3) * 8 + (idx & 3);
            if (SECOND) {
                const int d2 = ts[b] >> 5;
                second[b] = d1 < best[b] ? min(best[b], d2) : min(second[b], d1);
            }
            bj[b] = d1 < best[b] ? j : bj[b];
            best[b] = min(best[b], d1);
        }
    };
    // Stagger (MI355X_MICROARCH "two waves per SIMD", item 9): a SIMD holds waves w and w + 4
    // of a workgroup, which would otherwise reach their MFMAs and their VALU epilogues
    // together.  Waves 4-7 pass each tile's barrier before that tile's epilogue, the others
    // after it (the same number of barriers; the accumulators wait across it), so one wave's
    // epilogue runs beside its partner's MFMAs.  C32 is triple-buffered: a late epilogue of
    // tile t runs while tile t + 2 is staged.
    // the 16 MFMAs of one candidate tile (buffer Bs) into the accumulator set A
    auto mma = [&](i32x16 (&A)[2][2], const unsigned char *Bs) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            i32x4 fj[2], fq[2];
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                fj[a] = *(const i32x4 *)(Bs + (wj * 64 + a * 32 + lr) * BPI + 32 * k + 16 * lh);
                fq[a] = qfrag(a, k);
            }
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    A[a][b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fj[a], fq[b], k == 0 ? i32x16{} : A[a][b], 0, 0, 0);
        }
    };
#if PANO_I8_DBL
    // Two accumulator sets per wave: tile i's epilogue (VALU) is scheduled between the MFMAs
    // of tile i + 1 in the same wave (sched_group_barrier: 1 MFMA, 6 VALU), instead of after
    // them behind a dependency on the last MFMA.  Tile i of this workgroup sits in Bs2[i & 1]
    // and its C32 in Cs2[i % 3]; tile i + 2 is stored into tile i's buffer during step i (every
    // wave read tile i before the previous step's barrier) and fetched a step before that.
    i32x16 acc2[2][2];
    int jt = blockIdx.x, ti = 0;
    fetch(jt);
    store(0, 0);
    if (jt + n_split < n_jt) {
        fetch(jt + n_split);
        store(1, 1);
        if (jt + 2 * n_split < n_jt) fetch(jt + 2 * n_split);
    }
    __syncthreads();
    mma(acc, Bs2[0]);
    auto step = [&](i32x16 (&X)[2][2], i32x16 (&Y)[2][2]) -> bool {
        const bool more = jt + n_split < n_jt;
        // tile i + 1's MFMAs (past the last tile: the stale buffer, results unused) with tile
        // i's epilogue interleaved
        mma(Y, Bs2[(ti + 1) & 1]);
        epilogue(X, Cs2[ti % 3], jt);
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
        }
        if (jt + 2 * n_split < n_jt) {
            store(ti & 1, (ti + 2) % 3);
            if (jt + 3 * n_split < n_jt) fetch(jt + 3 * n_split);
        }
        __syncthreads();
        jt += n_split;
        ++ti;
        return more;
    };
    for (;;) {
        if (!step(acc, acc2)) break;
        if (!step(acc2, acc)) break;
    }
#else
    const bool lag = PANO_I8_STAGGER && wj == 1;
#if PANO_I8_PRIO
    if (wj == 1) __builtin_amdgcn_s_setprio(1);   // MI355X_MICROARCH two waves per SIMD, item 4
#endif
    int jt = blockIdx.x, cur = 0, c3 = 0;
    fetch(jt);
    store(0, 0);
    if (jt + n_split < n_jt) fetch(jt + n_split);
    __syncthreads();                // tile jt complete in buffer cur
    for (; jt < n_jt; jt += n_split, cur ^= 1, c3 = c3 == 2 ? 0 : c3 + 1) {
        mma(acc, Bs2[cur]);
        if (jt + n_split < n_jt) {
            store(cur ^ 1, c3 == 2 ? 0 : c3 + 1);
            if (jt + 2 * n_split < n_jt) fetch(jt + 2 * n_split);
        }
        // past this barrier: tile jt + n_split complete in cur ^ 1, every wave done with cur
        if (lag) __syncthreads();
        epilogue(acc, Cs2[c3], jt);
        if (!lag) __syncthreads();
    }
#endif
    auto imerge = [](int &b, int &j, int &s, int b2, int j2, int s2) {
        if (b2 < b || (b2 == b && j2 < j)) {
            s = min(s2, b);
            b = b2;
            j = j2;
        } else {
            s = min(s, b2);
        }
    };
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const int ob = __shfl_xor(best[b], 32), oj = __shfl_xor(bj[b], 32), os = __shfl_xor(second[b], 32);
        imerge(best[b], bj[b], second[b], ob, oj, os);
        const int il = wi * 64 + b * 32 + lr;
        if (lh == 0) red[wj][il] = IPart{best[b], bj[b], second[b]};
    }
    __syncthreads();
    if (tid < QT) {
        IPart x = red[0][tid];
        const IPart y = red[1][tid];
        imerge(x.best, x.idx, x.second, y.best, y.idx, y.second);
        const int gi = i0 + tid;
        if (gi < NA) {
#if PANO_I8_QLDS
            const int ra = rq(tid);
#else
            const int ra = cst[(size_t)fa * cap + gi];
#endif
            const float db = x.best >= kNone ? INFINITY : (float)(ra + x.best);
            const float ds = x.second >= kNone ? INFINITY : (float)(ra + x.second);
            Part *q = parts + ((size_t)p * n_split + blockIdx.x) * cap + gi;
            if (fold.cnt) {
                __hip_atomic_store((g_f32 *)&q->best, db, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store((g_i32 *)&q->idx, x.idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store((g_f32 *)&q->second, ds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                *q = Part{db, x.idx, ds};
            }
        }
    }
    if (!fold.cnt) return;
    __shared__ int last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");          // every wave: its partials landed
    __syncthreads();
    int32_t *cnt = fold.cnt + (size_t)p * gridDim.z + blockIdx.z;
    if (tid == 0) {
        fold_release();
        last = __hip_atomic_fetch_add((g_i32 *)cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               min(n_split, n_jt) - 1;
    }
    __syncthreads();
    if (!last) return;
    fold_acquire();
    if (tid < QT && i0 + tid < cap) {
        const int gi = i0 + tid;
        float b = INFINITY, s = INFINITY;
        int j = -1;
        if (gi < NA) {                           // reduce_parts, reading the partials sc1
            j = 0x7fffffff;
            const int nt = min(n_jt, n_split);
            for (int t = 0; t < nt; ++t) {
                Part *q = parts + ((size_t)p * n_split + t) * cap + gi;
                merge(b, j, s, __hip_atomic_load((g_f32 *)&q->best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                      __hip_atomic_load((g_i32 *)&q->idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                      __hip_atomic_load((g_f32 *)&q->second, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            }
            if (s >= kPadNorm) s = INFINITY;
        }
        const size_t o = (size_t)p * cap + gi;
        fold.best[o] = j;
        fold.d1[o] = b;
        if (fold.d2) fold.d2[o] = s;
    }
    if (tid == 0) __hip_atomic_store((g_i32 *)cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void reduce_parts(const Part *__restrict__ parts, const int32_t *__restrict__ counts,
                             int cap, PairArg pairs, int n_jt, int32_t *__restrict__ best,
                             float *__restrict__ d1, float *__restrict__ d2) {
    const int p = blockIdx.x;                         // grid (pair, row block)
    const int i = blockIdx.y * blockDim.x + threadIdx.x;
    if (i >= cap) return;
    int NA = counts[pairs.a[p]], NB = counts[pairs.b[p]];
    NA = min(max(NA, 0), cap);
    NB = min(max(NB, 0), cap);
    float b = INFINITY, s = INFINITY;
    int j = -1;
    if (i < NA) {
        j = 0x7fffffff;
        const int nt = min((NB + MT - 1) / MT, n_jt);
        for (int t = 0; t < nt; ++t) {
            const Part q = parts[((size_t)p * n_jt + t) * cap + i];
            merge(b, j, s, q.best, q.idx, q.second);
        }
        if (NB == 0) j = -1;
        if (s >= kPadNorm) s = INFINITY;      // only padding rows: no real second candidate
    }
    best[(size_t)p * cap + i] = j;
    d1[(size_t)p * cap + i] = b;
    if (d2) d2[(size_t)p * cap + i] = s;
}

// ---------------------------------------------------------------- Harris (float descriptors)
__device__ float sdot_skx_diff(const float *a, const float *b) {
    float a16[4][16];
    for (int k = 0; k < 4; ++k)
        for (int j = 0; j < 16; ++j) a16[k][j] = 0.0f;
    for (int i = 0; i < 128; i += 64)
        for (int k = 0; k < 4; ++k)
            for (int j = 0; j < 16; ++j) {
                const float t = a[i + 16 * k + j] - b[i + 16 * k + j];
                a16[k][j] = fmaf(t, t, a16[k][j]);
            }
    float v[8];
    for (int j = 0; j < 8; ++j) {
        const float s0 = a16[0][j] + a16[0][j + 8];
        const float s1 = a16[1][j] + a16[1][j + 8];
        const float s2 = a16[2][j] + a16[2][j + 8];
        const float s3 = a16[3][j] + a16[3][j + 8];
        v[j] = ((s0 + s1) + s2) + s3;
    }
    float h[4];
    for (int j = 0; j < 4; ++j) h[j] = v[j] + v[j + 4];
    return (h[0] + h[1]) + (h[2] + h[3]);
}

__global__ void __launch_bounds__(256)
dist_direct(const float *__restrict__ desc, const int32_t *__restrict__ counts, int cap,
            PairArg pairs, int32_t *__restrict__ best, float *__restrict__ d1,
            float *__restrict__ d2) {
    __shared__ float arow[PANO_DESC_DIM];
    __shared__ float rb[256];
    __shared__ int rj[256];
    __shared__ float rs[256];
    const int p = blockIdx.y, i = blockIdx.x, tid = threadIdx.x;
    const int fa = pairs.a[p], fb = pairs.b[p];
    int NA = counts[fa], NB = counts[fb];
    NA = min(max(NA, 0), cap);
    NB = min(max(NB, 0), cap);
    if (i >= cap) return;
    if (i >= NA) {
        if (tid == 0) {
            best[(size_t)p * cap + i] = -1;
            d1[(size_t)p * cap + i] = INFINITY;
            d2[(size_t)p * cap + i] = INFINITY;
        }
        return;
    }
    if (tid < PANO_DESC_DIM) arow[tid] = desc[((size_t)fa * cap + i) * PANO_DESC_DIM + tid];
    __syncthreads();
    float b = INFINITY, s = INFINITY;
    int j = 0x7fffffff;
    for (int jj = tid; jj < NB; jj += 256) {
        const float d = sdot_skx_diff(arow, desc + ((size_t)fb * cap + jj) * PANO_DESC_DIM);
        merge(b, j, s, d, jj, INFINITY);
    }
    rb[tid] = b;
    rj[tid] = j;
    rs[tid] = s;
    __syncthreads();
    if (tid == 0) {
        float B = INFINITY, Sx = INFINITY;
        int J = 0x7fffffff;
        for (int t = 0; t < 256; ++t) merge(B, J, Sx, rb[t], rj[t], rs[t]);
        best[(size_t)p * cap + i] = NB > 0 ? J : -1;
        d1[(size_t)p * cap + i] = B;
        d2[(size_t)p * cap + i] = Sx;
    }
}

}  // namespace

int match_set_attributes(pano_ctx *) { return PANO_OK; }

int launch_match_u8(pano_ctx *ctx, const uint8_t *desc, const int32_t *norms, const int32_t *counts,
                    int cap, const int32_t *h_pairs, int n_pairs, int32_t *best, float *d1, float *d2) {
    if (cap <= 0 || n_pairs <= 0 || !desc || !norms || !counts || !best || !d1)
        return pano_fail(ctx, PANO_E_ARG, "pano_match_u8: bad arguments");
    const int n_qt = (cap + QT - 1) / QT, n_bt = (cap + BT - 1) / BT;
    for (int p0 = 0; p0 < n_pairs; p0 += 256) {
        const int np = n_pairs - p0 < 256 ? n_pairs - p0 : 256;
        PairArg pa;
        for (int q = 0; q < np; ++q) {
            pa.a[q] = h_pairs[2 * (p0 + q)];
            pa.b[q] = h_pairs[2 * (p0 + q) + 1];
        }
        // query tiles x candidate splits x pairs: at least ~2 workgroups per CU even when
        // each pair is small (parrington); large pairs walk their candidate tiles in-kernel
        static const int target_wgs = [] {
            const char *e = getenv("PANO_MATCH_WGS");   // fewest workgroups the splits aim at
            return e ? std::max(1, atoi(e)) : 1024;
        }();
        const int tw = (ctx->flags_opt & PANO_CTX_MATCH_WHOLE) ? 1 : target_wgs;
        const int n_split = std::max(1, std::min(n_bt, (tw + n_qt * np - 1) / (n_qt * np)));
        const size_t part_bytes = ((size_t)np * n_split * cap * sizeof(Part) + 255) & ~size_t(255);
        int rc = pano_grow(ctx, &ctx->mscratch, &ctx->mscratch_bytes, part_bytes);
        if (rc) return rc;
        Part *parts = (Part *)ctx->mscratch;
        int32_t *bp = best + (size_t)p0 * cap;
        float *p1 = d1 + (size_t)p0 * cap, *p2 = d2 ? d2 + (size_t)p0 * cap : nullptr;
        // (split, pair, query tile): the dispatcher walks x, then y fastest, so every pair's
        // live query tiles (the low ones; the grid is sized by the capacity) go out before the
        // empty tail -- with the tile index outermost each pair's empty tiles were dispatched
        // ahead of the next pair's live ones (the same for row_consts and reduce_parts)
        dim3 grid(n_split, np, n_qt);
        static const bool use_i8 = [] {
            const char *e = getenv("PANO_MATCH_I8");     // 1 (default): i8 MFMA; 0: bf16 MFMA
            return e ? atoi(e) != 0 : true;
        }();
        if (use_i8) {
            int nf = 0;
            for (int q = 0; q < 2 * np; ++q) nf = std::max(nf, h_pairs[2 * p0 + q] + 1);
            const size_t cst_bytes = (size_t)nf * cap * sizeof(int32_t);
            rc = pano_grow(ctx, &ctx->mscratch, &ctx->mscratch_bytes, part_bytes + cst_bytes);
            if (rc) return rc;
            parts = (Part *)ctx->mscratch;
            int32_t *cst = (int32_t *)((char *)ctx->mscratch + part_bytes);
            if (!PANO_I8_QLDS) {   // the row constants are formed in dist_i8's staging otherwise
                {
                    PanoProf prof_(ctx, PK_NORMS);
                    row_consts<<<dim3(nf, (cap + 63) / 64), 256, 0, ctx->stream>>>(desc, norms, counts, cap, cst);
                }
                PANO_LAUNCH_CHECK(ctx, "row_consts");
            }
            // reduce_parts folded in (PANO_MATCH_FOLD, default 1; 0: the separate launch)
            static const bool fold_on = [] {
                const char *e = getenv("PANO_MATCH_FOLD");
                return e ? atoi(e) != 0 : true;
            }();
            MatchFold mf{};
            if (fold_on) {
                const size_t need = (size_t)256 * n_qt * sizeof(int32_t);
                if (need > ctx->match_sync_bytes) {
                    if (ctx->capturing)
                        return pano_fail(ctx, PANO_E_UNSUPPORTED, "match counters grown inside a graph capture");
                    if (ctx->match_sync) {
                        PANO_HIP(ctx, hipStreamSynchronize(ctx->stream));
                        (void)hipFree(ctx->match_sync);
                        ctx->match_sync = nullptr;
                        ctx->match_sync_bytes = 0;
                        ++ctx->generation;
                    }
                    PANO_HIP(ctx, hipMalloc((void **)&ctx->match_sync, need));
                    PANO_HIP(ctx, hipMemset(ctx->match_sync, 0, need));   // each launch re-zeroes
                    ctx->match_sync_bytes = need;
                }
                mf.cnt = ctx->match_sync;
                mf.best = bp;
                mf.d1 = p1;
                mf.d2 = p2;
            }
            {
                PanoProf prof_(ctx, PK_DIST_MFMA);
                if (p2)
                    dist_i8<true><<<grid, 512, 0, ctx->stream>>>(desc, norms, cst, counts, cap, pa, parts, n_split, mf);
                else
                    dist_i8<false><<<grid, 512, 0, ctx->stream>>>(desc, norms, cst, counts, cap, pa, parts, n_split, mf);
            }
            PANO_LAUNCH_CHECK(ctx, "dist_i8");
            if (fold_on) continue;
        } else {
            {
                PanoProf prof_(ctx, PK_DIST_MFMA);
                if (p2)
                    dist_u8<true><<<grid, 512, 0, ctx->stream>>>(desc, norms, counts, cap, pa, parts, n_split);
                else
                    dist_u8<false><<<grid, 512, 0, ctx->stream>>>(desc, norms, counts, cap, pa, parts, n_split);
            }
            PANO_LAUNCH_CHECK(ctx, "dist_u8");
        }
        dim3 g2(np, (cap + 255) / 256);
        {
            PanoProf prof_(ctx, PK_REDUCE);
            reduce_parts<<<g2, 256, 0, ctx->stream>>>(parts, counts, cap, pa, n_split, bp, p1, p2);
        }
        PANO_LAUNCH_CHECK(ctx, "reduce_parts");
    }
    return PANO_OK;
}

int launch_match(pano_ctx *ctx, const float *desc, const int32_t *counts, int cap,
                 const int32_t *h_pairs, int n_pairs, int exact_int, int32_t *best, float *d1,
                 float *d2) {
    if (cap <= 0 || n_pairs <= 0 || !desc || !counts || !best || !d1 || (!d2 && exact_int != 2))
        return pano_fail(ctx, PANO_E_ARG, "pano_match: bad arguments");
    int n_frames = 0;
    for (int q = 0; q < 2 * n_pairs; ++q) n_frames = h_pairs[q] + 1 > n_frames ? h_pairs[q] + 1 : n_frames;
    for (int p0 = 0; p0 < n_pairs; p0 += 256) {
        const int np = n_pairs - p0 < 256 ? n_pairs - p0 : 256;
        PairArg pa;
        for (int q = 0; q < np; ++q) {
            pa.a[q] = h_pairs[2 * (p0 + q)];
            pa.b[q] = h_pairs[2 * (p0 + q) + 1];
        }
        int32_t *bp = best + (size_t)p0 * cap;
        float *p1 = d1 + (size_t)p0 * cap, *p2 = d2 ? d2 + (size_t)p0 * cap : nullptr;
        if (!exact_int) {
            dim3 grid(cap, np);
            {
                PanoProf prof_(ctx, PK_DIST_DIRECT);
                dist_direct<<<grid, 256, 0, ctx->stream>>>(desc, counts, cap, pa, bp, p1, p2);
            }
            PANO_LAUNCH_CHECK(ctx, "dist_direct");
            continue;
        }
        const int n_t = (cap + MT - 1) / MT;
        const size_t norm_bytes = ((size_t)n_frames * n_t * MT * sizeof(float) + 255) & ~size_t(255);
        dim3 g2(np, (cap + 255) / 256);                      // reduce_parts: (pair, row block)
        if (exact_int == 2) {
            // query tiles x candidate splits x pairs: enough workgroups to fill the GPU even
            // when each pair is small; large pairs walk their candidate tiles in-kernel
            const int capP = n_t * MT;
            const int n_split = std::max(1, std::min(n_t, (4096 + n_t * np - 1) / (n_t * np)));
            const size_t part_bytes = ((size_t)np * n_split * cap * sizeof(Part) + 255) & ~size_t(255);
            const size_t pk_bytes = (size_t)n_frames * capP * KA * sizeof(unsigned short);
            int rc = pano_grow(ctx, &ctx->mscratch, &ctx->mscratch_bytes,
                               norm_bytes + part_bytes + 2 * pk_bytes);
            if (rc) return rc;
            float *norms = (float *)ctx->mscratch;
            Part *parts = (Part *)((char *)ctx->mscratch + norm_bytes);
            unsigned short *pka = (unsigned short *)((char *)ctx->mscratch + norm_bytes + part_bytes);
            unsigned short *pkb = (unsigned short *)((char *)pka + pk_bytes);
            const size_t rows = (size_t)n_frames * capP;
            {
                PanoProf prof_(ctx, PK_NORMS);
                pack_rows<<<(unsigned)((rows * 16 + 255) / 256), 256, 0, ctx->stream>>>(
                    desc, counts, cap, capP, n_frames, pka, pkb, norms);
            }
            PANO_LAUNCH_CHECK(ctx, "pack_rows");
            dim3 grid(n_split, n_t, np);
            {
                PanoProf prof_(ctx, PK_DIST_MFMA);
                if (p2)
                    dist_bf16<true><<<grid, 256, 0, ctx->stream>>>(pka, pkb, norms, counts, cap, capP,
                                                                   pa, parts, n_split);
                else
                    dist_bf16<false><<<grid, 256, 0, ctx->stream>>>(pka, pkb, norms, counts, cap, capP,
                                                                    pa, parts, n_split);
            }
            PANO_LAUNCH_CHECK(ctx, "dist_bf16");
            {
                PanoProf prof_(ctx, PK_REDUCE);
                reduce_parts<<<g2, 256, 0, ctx->stream>>>(parts, counts, cap, pa, n_split, bp, p1, p2);
            }
            PANO_LAUNCH_CHECK(ctx, "reduce_parts");
            continue;
        }
        const size_t part_bytes = (size_t)np * n_t * cap * sizeof(Part);
        int rc = pano_grow(ctx, &ctx->mscratch, &ctx->mscratch_bytes, norm_bytes + part_bytes);
        if (rc) return rc;
        float *norms = (float *)ctx->mscratch;
        Part *parts = (Part *)((char *)ctx->mscratch + norm_bytes);
        const size_t rows = (size_t)n_frames * cap;
        {
            PanoProf prof_(ctx, PK_NORMS);
            row_norms<<<(unsigned)((rows + 255) / 256), 256, 0, ctx->stream>>>(desc, counts, cap, n_frames, norms);
        }
        PANO_LAUNCH_CHECK(ctx, "row_norms");
        {
            dim3 grid(n_t, n_t, np);
            const size_t sm = 2 * (size_t)MT * LDA * sizeof(float);
            PanoProf prof_(ctx, PK_DIST_MFMA);
            dist_mfma<<<grid, 256, sm, ctx->stream>>>(desc, norms, counts, cap, pa, parts, n_t);
        }
        PANO_LAUNCH_CHECK(ctx, "dist_mfma");
        {
            PanoProf prof_(ctx, PK_REDUCE);
            reduce_parts<<<g2, 256, 0, ctx->stream>>>(parts, counts, cap, pa, n_t, bp, p1, p2);
        }
        PANO_LAUNCH_CHECK(ctx, "reduce_parts");
    }
    return PANO_OK;
}
