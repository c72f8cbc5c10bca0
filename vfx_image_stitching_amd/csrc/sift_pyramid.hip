// sift_pyramid.hip -- S1..S4 of sift_impl.py: base image, Gaussian and DoG pyramids.
//
//   generate_base_image      sift_impl.py:45-56   gray(u8) -> x2 INTER_LINEAR -> blur(s0)
//   generate_gaussian_images sift_impl.py:82-97   5 cascaded blurs / octave, next octave =
//                                                 INTER_NEAREST 1/2 of level n_lvl-3
//   generate_DoG_images      sift_impl.py:100-111 G[s+1] - G[s]
//
// One launch per (octave, level) blurs ALL frames of the batch (grid.z = frame).  A work-
// group owns a 64 x 64 output tile: it stages the (64+2r)^2 input tile in LDS through a
// mode-specific loader (BGR->gray->x2 bilinear for the base, nearest 1/2 of the previous
// octave for level 1 of octave o>0, plain for the rest), runs the row pass into a second
// LDS tile and the column pass to HBM, writing the DoG level in the same epilogue.
//
// Exactness (oracle/cv2_compat.py, oracle/cv_blur.c): the arithmetic is OpenCV
// 4.x's float32 separable filter, which the author's published SIFT panoramas pin (grail
// pixel-identical).  Taps are getGaussianKernelBitExact's, cast to f32.  Row pass
// (RowVec_32f): s = x0*k0, then s = fma(x_i, k_i, s) for i = 1..n-1 in f32.  Column pass
// (SymmColumnVec_32f): s = S0*kc, then s = fma(S[+i] + S[-i], k_i, s) for i = 1..r outward,
// the pair sum rounded to f32 first.  One rounding per operation, so any thread / tile /
// register mapping that keeps this per-output operation order is bit-identical.  The x2
// bilinear upsample of integer gray levels is exact.
#include "pano_internal.h"
#include "cas_taps.h"

#include <algorithm>
#include <cstring>
#include <utility>

namespace {

constexpr int TX = 64;
constexpr int TY = 64;
constexpr int TXP = TX + 1;   // odd trow pitch: row-pass stores are conflict-free

struct Taps {
    float k[PANO_MAX_TAPS];
    int n;
};

enum Mode { MODE_BASE = 0, MODE_LEVEL = 1, MODE_DOWN = 2, MODE_BASEF = 3 };   // BASEF: f32 gray input

struct LoadArgs {
    const uint8_t *gray;  // MODE_BASE: [n][sh][sw] u8 gray (cvtColor BGR2GRAY)
    const float *grayf;   // MODE_BASEF: [n][sh][sw] f32 gray (generate_base_image on any f32 image)
    const float *src;     // MODE_LEVEL: [n][H][W]; MODE_DOWN: [n][sh][sw]
    int sh, sw;           // source size (BASE: gray size; DOWN: previous octave size)
    double ifx, ify;      // DOWN: 1 / (dst / src), OpenCV resizeNN
};

// OpenCV INTER_LINEAR source index and f32 weight for destination d (cv2_compat._linear_map).
__device__ __forceinline__ void lin_map(int d, int src_n, int &s0, int &s1, float &w1) {
    double fx = (d + 0.5) * 0.5 - 0.5;   // inv_scale = 2 -> scale = 0.5
    int sx = (int)floor(fx);
    fx -= sx;
    if (sx < 0) { fx = 0.0; sx = 0; }
    if (sx >= src_n - 1) { fx = 0.0; sx = src_n - 1; }
    s0 = sx;
    s1 = sx + 1 < src_n ? sx + 1 : src_n - 1;
    w1 = (float)fx;
}

// BORDER_REFLECT_101 with the in-range case first (interior tiles never take the slow path).
__device__ __forceinline__ int reflect_fast(int i, int n) {
    return (unsigned)i < (unsigned)n ? i : reflect101(i, n);
}

// Tile staging.  Wave w stages tile rows w, w + NW, ... with lane = column (lane and
// 64 + lane): every row quantity (source row, reflection, bilinear row weights) is computed
// once per row in scalar registers (the row index is readfirstlane'd), every column
// quantity once per lane, so a staged element costs its load(s) and an LDS store.
struct ColMap {          // per-lane column part of a stager
    int c0, c1;          // source column(s)
    float w1;            // MODE_BASE: bilinear weight of c1
};

template <int MODE> struct Stager;

template <> struct Stager<MODE_LEVEL> {   // plain: source = previous level of this octave
    const float *base;
    int W, H;
    __device__ Stager(const LoadArgs &a, int f, int H_, int W_) : base(a.src + (size_t)f * H_ * W_), W(W_), H(H_) {}
    __device__ __forceinline__ ColMap col(int x) const { return ColMap{reflect_fast(x, W), 0, 0.f}; }
    __device__ __forceinline__ float get(int y, const ColMap &c) const {
        return base[(size_t)reflect_fast(y, H) * W + c.c0];
    }
};

template <> struct Stager<MODE_DOWN> {    // OpenCV INTER_NEAREST 1/2 of the previous octave
    const float *base;
    int W, H, sh, sw;
    double ifx, ify;
    __device__ Stager(const LoadArgs &a, int f, int H_, int W_)
        : base(a.src + (size_t)f * a.sh * a.sw), W(W_), H(H_), sh(a.sh), sw(a.sw), ifx(a.ifx), ify(a.ify) {}
    __device__ __forceinline__ ColMap col(int x) const {
        const int t = (int)floor(reflect_fast(x, W) * ifx);
        return ColMap{t < sw - 1 ? t : sw - 1, 0, 0.f};
    }
    __device__ __forceinline__ float get(int y, const ColMap &c) const {
        int sy = (int)floor(reflect_fast(y, H) * ify);
        sy = sy < sh - 1 ? sy : sh - 1;
        return base[(size_t)sy * sw + c.c0];
    }
};

template <> struct Stager<MODE_BASE> {    // gray (u8) -> x2 INTER_LINEAR, exact
    const uint8_t *fr;
    int W, H, sh, sw;
    __device__ Stager(const LoadArgs &a, int f, int H_, int W_)
        : fr(a.gray + (size_t)f * a.sh * a.sw), W(W_), H(H_), sh(a.sh), sw(a.sw) {}
    __device__ __forceinline__ ColMap col(int x) const {
        ColMap c;
        lin_map(reflect_fast(x, W), sw, c.c0, c.c1, c.w1);
        return c;
    }
    __device__ __forceinline__ float get(int y, const ColMap &c) const {
        int y0, y1;
        float wy;
        lin_map(reflect_fast(y, H), sh, y0, y1, wy);
        const uint8_t *r0 = fr + (size_t)y0 * sw, *r1 = fr + (size_t)y1 * sw;
        const float g00 = r0[c.c0], g01 = r0[c.c1];
        const float g10 = r1[c.c0], g11 = r1[c.c1];
        const float wx0 = 1.0f - c.w1;
        const float h0 = g00 * wx0 + g01 * c.w1;
        const float h1 = g10 * wx0 + g11 * c.w1;
        return h0 * (1.0f - wy) + h1 * wy;
    }
};

// f32 gray -> x2 INTER_LINEAR (the stage function generate_base_image on a caller's f32
// image): the same expression as Stager<MODE_BASE>; exact for integer-valued inputs, the
// reference's OpenCV rounding otherwise unpinned.
template <> struct Stager<MODE_BASEF> {
    const float *fr;
    int W, H, sh, sw;
    __device__ Stager(const LoadArgs &a, int f, int H_, int W_)
        : fr(a.grayf + (size_t)f * a.sh * a.sw), W(W_), H(H_), sh(a.sh), sw(a.sw) {}
    __device__ __forceinline__ ColMap col(int x) const {
        ColMap c;
        lin_map(reflect_fast(x, W), sw, c.c0, c.c1, c.w1);
        return c;
    }
    __device__ __forceinline__ float get(int y, const ColMap &c) const {
        int y0, y1;
        float wy;
        lin_map(reflect_fast(y, H), sh, y0, y1, wy);
        const float *r0 = fr + (size_t)y0 * sw, *r1 = fr + (size_t)y1 * sw;
        const float wx0 = 1.0f - c.w1;
        const float h0 = r0[c.c0] * wx0 + r0[c.c1] * c.w1;
        const float h1 = r1[c.c0] * wx0 + r1[c.c1] * c.w1;
        return h0 * (1.0f - wy) + h1 * wy;
    }
};

// Stage the (ih x iw) input tile whose top-left source pixel is (y0 - R, x0 - R) into
// t[ih][IWP] (iw <= 128).  NW waves; all of a lane's loads are issued before its stores.
template <int MODE, int NW, int RPW>
__device__ __forceinline__ void stage_tile(const LoadArgs &la, int f, int H, int W, int x0, int y0,
                                           int R, int ih, int iw, int IWP, float *t) {
    const Stager<MODE> sg(la, f, H, W);
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool has1 = 64 + lane < iw;
    const ColMap m0 = sg.col(x0 - R + lane);
    const ColMap m1 = sg.col(x0 - R + (has1 ? 64 + lane : lane));
    float v0[RPW], v1[RPW];
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
        const int ty = wv + NW * k;
        if (ty < ih) {
            v0[k] = sg.get(y0 - R + ty, m0);
            v1[k] = has1 ? sg.get(y0 - R + ty, m1) : 0.0f;
        }
    }
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
        const int ty = wv + NW * k;
        if (ty < ih) {
            if (lane < iw) t[ty * IWP + lane] = v0[k];   // iw < 64 (narrow tile): stay in the row
            if (has1) t[ty * IWP + 64 + lane] = v1[k];
        }
    }
}

// Interior tiles of MODE_LEVEL (no reflection: the whole (64 + 2R)^2 input window lies inside
// the plane, W % 4 == 0): 16-byte aligned loads over the 4-aligned superset of each row,
// scattered into the same LDS layout as stage_tile.  A quarter of the load instructions and
// no per-row reflection arithmetic (the interior is ~80 % of the tiles at octave 0).
template <int R, int NTHR, int TYT = TY, int TXT = TX>
__device__ __forceinline__ void stage_interior(const float *__restrict__ plane, int W, int x0, int y0,
                                               int IWP, float *t) {
    constexpr int IW = TXT + 2 * R, IH = TYT + 2 * R;
    const int xa = (x0 - R) & ~3, off = (x0 - R) - xa;    // off in 0..3, wave-uniform
    const int nq = (off + IW + 3) >> 2;                   // float4 per row
    constexpr int MAXQ = (IH * ((IW + 6) / 4) + NTHR - 1) / NTHR;
    const float *rowp = plane + (size_t)(y0 - R) * W + xa;
    float4 v[MAXQ];
    int rr[MAXQ], cc[MAXQ];
#pragma unroll
    for (int k = 0; k < MAXQ; ++k) {
        const int idx = (int)threadIdx.x + NTHR * k;
        const int r = idx / nq, q = idx - r * nq;
        rr[k] = r;
        cc[k] = 4 * q - off;                               // tile column of element 0 (>= -3)
        if (r < IH) v[k] = *(const float4 *)(rowp + (size_t)r * W + 4 * q);
    }
#pragma unroll
    for (int k = 0; k < MAXQ; ++k) {
        if (rr[k] >= IH) continue;
        const float e[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
        float *dst = t + rr[k] * IWP + cc[k];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (cc[k] + j >= 0 && cc[k] + j < IW) dst[j] = e[j];
    }
}

// Interior tiles of MODE_BASE (the x2 INTER_LINEAR source window lies inside the gray frame,
// no reflection, no clamping): the tile's gray source patch (<= 47 x 47 bytes) is loaded once
// into LDS as floats, then every staged element is the same f32 bilinear expression as
// Stager<MODE_BASE>::get over four LDS reads instead of four byte loads from global memory.
constexpr int kPatch = 48;                 // patch columns capacity
constexpr int kPatchP = kPatch + 1;        // odd pitch
constexpr int kPatchR = 72;                // patch rows capacity
template <int R, int NTHR, int TYT = TY>
__device__ __forceinline__ void stage_base_interior(const LoadArgs &la, int f, int x0, int y0, int IWP,
                                                    float *t, float *patch) {
    constexpr int IW = TX + 2 * R, IH = TYT + 2 * R;
    static_assert(IH / 2 + 3 <= kPatchR && IW / 2 + 3 <= kPatch, "patch capacity");
    const uint8_t *fr = la.gray + (size_t)f * la.sh * la.sw;
    int p0, p1, q0, q1;
    float w_unused;
    lin_map(y0 - R, la.sh, p0, p1, w_unused);               // first source row / column
    lin_map(x0 - R, la.sw, q0, q1, w_unused);
    const int np = IH / 2 + 3, nq = IW / 2 + 3;             // covers the window (+ slack)
    for (int i = threadIdx.x; i < np * kPatch; i += NTHR) {
        const int r = i / kPatch, c = i - r * kPatch;
        if (c < nq && p0 + r < la.sh && q0 + c < la.sw)       // slack rows past the frame: unread
            patch[r * kPatchP + c] = (float)fr[(size_t)(p0 + r) * la.sw + q0 + c];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int NW = NTHR / 64;
    // per-lane columns (lane, 64 + lane): patch column of c0 and the weight of c1
    int cA, cB;
    float wA, wB;
    {
        int a0, a1;
        lin_map(x0 - R + lane, la.sw, a0, a1, wA);
        cA = a0 - q0;
        const int xb = 64 + lane < IW ? 64 + lane : lane;
        lin_map(x0 - R + xb, la.sw, a0, a1, wB);
        cB = a0 - q0;
    }
    for (int ty = wv; ty < IH; ty += NW) {
        int r0, r1;
        float wy;
        lin_map(y0 - R + ty, la.sh, r0, r1, wy);
        const float *P0 = patch + (r0 - p0) * kPatchP, *P1 = P0 + kPatchP;
        {
            const float g00 = P0[cA], g01 = P0[cA + 1], g10 = P1[cA], g11 = P1[cA + 1];
            const float wx0 = 1.0f - wA;
            const float h0 = g00 * wx0 + g01 * wA;
            const float h1 = g10 * wx0 + g11 * wA;
            t[ty * IWP + lane] = h0 * (1.0f - wy) + h1 * wy;
        }
        if (64 + lane < IW) {
            const float g00 = P0[cB], g01 = P0[cB + 1], g10 = P1[cB], g11 = P1[cB + 1];
            const float wx0 = 1.0f - wB;
            const float h0 = g00 * wx0 + g01 * wB;
            const float h1 = g10 * wx0 + g11 * wB;
            t[ty * IWP + 64 + lane] = h0 * (1.0f - wy) + h1 * wy;
        }
    }
}

// Every tile of MODE_BASE (interior and edge alike): the gray source rows / columns the
// tile's reflected x2 INTER_LINEAR window reads form one contiguous patch (lin_map is monotone
// and BORDER_REFLECT_101 folds the window back inside [0, H) x [0, W)), loaded once into LDS as
// floats -- all of a thread's byte loads issued before its LDS stores -- then every staged
// element is Stager<MODE_BASE>::get's f32 bilinear expression over four LDS reads at its own
// (clamped) source indices.  Replaces, for the edge tiles (a third of parrington's octave-0
// tiles), stage_tile's four global byte loads and f64 row map per element.
template <int R, int NTHR, int TYT = TY>
__device__ __forceinline__ void stage_base_patch(const LoadArgs &la, int f, int H, int W, int x0, int y0,
                                                 int ih, int iw, int IWP, float *t, float *patch) {
    static_assert((TYT + 2 * R) / 2 + 3 <= kPatchR && (TX + 2 * R) / 2 + 3 <= kPatch, "patch capacity");
    const uint8_t *fr = la.gray + (size_t)f * la.sh * la.sw;
    int p0, pl, q0, ql, u;
    float w_unused;
    lin_map(max(y0 - R, 0), la.sh, p0, u, w_unused);                  // patch rows [p0, pl]
    lin_map(min(y0 - R + ih - 1, H - 1), la.sh, u, pl, w_unused);
    lin_map(max(x0 - R, 0), la.sw, q0, u, w_unused);                  // patch columns [q0, ql]
    lin_map(min(x0 - R + iw - 1, W - 1), la.sw, u, ql, w_unused);
    const int np = pl - p0 + 1, nq = ql - q0 + 1;
    constexpr int MAXP = (kPatchR * kPatch + NTHR - 1) / NTHR;
    uint8_t v[MAXP];
#pragma unroll
    for (int k = 0; k < MAXP; ++k) {
        const int i = (int)threadIdx.x + NTHR * k, r = i / kPatch, c = i - r * kPatch;
        v[k] = (r < np && c < nq) ? fr[(size_t)(p0 + r) * la.sw + q0 + c] : (uint8_t)0;
    }
#pragma unroll
    for (int k = 0; k < MAXP; ++k) {
        const int i = (int)threadIdx.x + NTHR * k, r = i / kPatch, c = i - r * kPatch;
        if (r < np && c < nq) patch[r * kPatchP + c] = (float)v[k];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int NW = NTHR / 64;
    // per-lane columns (lane, 64 + lane): patch columns of c0, c1 and the weight of c1
    int cA0, cA1, cB0, cB1;
    float wA, wB;
    {
        int a0, a1;
        lin_map(reflect_fast(x0 - R + min(lane, iw - 1), W), la.sw, a0, a1, wA);
        cA0 = a0 - q0;
        cA1 = a1 - q0;
        const int xb = 64 + lane < iw ? 64 + lane : min(lane, iw - 1);
        lin_map(reflect_fast(x0 - R + xb, W), la.sw, a0, a1, wB);
        cB0 = a0 - q0;
        cB1 = a1 - q0;
    }
    for (int ty = wv; ty < ih; ty += NW) {
        int r0, r1;
        float wy;
        lin_map(reflect_fast(y0 - R + ty, H), la.sh, r0, r1, wy);
        const float *P0 = patch + (r0 - p0) * kPatchP, *P1 = patch + (r1 - p0) * kPatchP;
        if (lane < iw) {
            const float g00 = P0[cA0], g01 = P0[cA1], g10 = P1[cA0], g11 = P1[cA1];
            const float wx0 = 1.0f - wA;
            const float h0 = g00 * wx0 + g01 * wA;
            const float h1 = g10 * wx0 + g11 * wA;
            t[ty * IWP + lane] = h0 * (1.0f - wy) + h1 * wy;
        }
        if (64 + lane < iw) {
            const float g00 = P0[cB0], g01 = P0[cB1], g10 = P1[cB0], g11 = P1[cB1];
            const float wx0 = 1.0f - wB;
            const float h0 = g00 * wx0 + g01 * wB;
            const float h1 = g10 * wx0 + g11 * wB;
            t[ty * IWP + 64 + lane] = h0 * (1.0f - wy) + h1 * wy;
        }
    }
}

// cvtColor(BGR2GRAY) of every frame, 4 pixels per thread (sift_impl.py:27-28).
// zp / zn: a word block to zero in passing (the keypoint stage's counters, sift_kp_counters)
__global__ void __launch_bounds__(256)
gray_frames(const uint8_t *__restrict__ bgr, uint8_t *__restrict__ gray, size_t npx,
            int32_t *__restrict__ zp = nullptr, int zn = 0) {
    if (zp && blockIdx.x == 0)
        for (int i = threadIdx.x; i < zn; i += 256) zp[i] = 0;
    const size_t i0 = ((size_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (i0 + 4 <= npx) {
        const uint32_t *p = (const uint32_t *)(bgr + i0 * 3);   // 12 bytes, 4-aligned
        const uint32_t w0 = p[0], w1 = p[1], w2 = p[2];
        uint8_t b[12];
        for (int k = 0; k < 4; ++k) {
            b[k] = (uint8_t)(w0 >> (8 * k));
            b[4 + k] = (uint8_t)(w1 >> (8 * k));
            b[8 + k] = (uint8_t)(w2 >> (8 * k));
        }
        uint32_t out = 0;
        for (int k = 0; k < 4; ++k) out |= (uint32_t)gray_u8(b + 3 * k) << (8 * k);
        *(uint32_t *)(gray + i0) = out;
    } else {
        for (size_t i = i0; i < npx; ++i) gray[i] = gray_u8(bgr + i * 3);
    }
}

// Register-blocked passes: SEG consecutive outputs of one row (or column) from SEG + NT - 1
// staged inputs, all index arithmetic compile-time after unrolling.
#ifndef PANO_TAIL_SYNC
#define PANO_TAIL_SYNC 0    // 1: full __syncthreads in blur_tail (A/B of lds_barrier)
#endif
#ifndef PANO_BLUR_ABL
#define PANO_BLUR_ABL 0     // timing ablations of blur_fast only: bit 2 no stores, 4 no loads
#endif
// Row pass, RowVec_32f: output j takes taps t = 0..NT-1 in order, the first as a product.
template <int NT, int SEG, typename PF = const float *>
__device__ __forceinline__ void row_seg(PF __restrict__ p, const float *__restrict__ k,
                                        float (&acc)[SEG]) {
#pragma unroll
    for (int i = 0; i < SEG + NT - 1; ++i) {
        const float v = p[i];
#pragma unroll
        for (int j = 0; j < SEG; ++j) {
            const int t = i - j;
            if (t == 0) acc[j] = v * k[0];
            else if (t > 0 && t < NT) acc[j] = __builtin_fmaf(v, k[t], acc[j]);
        }
    }
}

// Column pass, SymmColumnVec_32f: output j = centre product, then the pairs at distance
// d = 1..R outward, each pair summed in f32 before its fused multiply-add.
template <int NT, int SEG>
__device__ __forceinline__ void col_seg(const float *__restrict__ p, int stride, const float *__restrict__ k,
                                        float (&acc)[SEG]) {
    constexpr int R = (NT - 1) / 2;
    float v[SEG + NT - 1];
#pragma unroll
    for (int i = 0; i < SEG + NT - 1; ++i) v[i] = p[i * stride];
#pragma unroll
    for (int j = 0; j < SEG; ++j) acc[j] = v[j + R] * k[R];
#pragma unroll
    for (int d = 1; d <= R; ++d)
#pragma unroll
        for (int j = 0; j < SEG; ++j) acc[j] = __builtin_fmaf(v[j + R + d] + v[j + R - d], k[R + d], acc[j]);
}

// Runtime tap count fallback (sigma values other than the reference defaults).
template <typename PF = const float *, typename KF = const float *>
__device__ __forceinline__ float row_one(PF __restrict__ p, KF __restrict__ k, int n) {
    float acc = p[0] * k[0];
    for (int t = 1; t < n; ++t) acc = __builtin_fmaf(p[t], k[t], acc);
    return acc;
}
__device__ __forceinline__ float col_one(const float *__restrict__ p, int stride, const float *__restrict__ k,
                                         int n) {
    const int r = (n - 1) / 2;
    float acc = p[r * stride] * k[r];
    for (int d = 1; d <= r; ++d) acc = __builtin_fmaf(p[(r + d) * stride] + p[(r - d) * stride], k[r + d], acc);
    return acc;
}

constexpr int SEG = 16;

template <int MODE, int NT>
__global__ void __launch_bounds__(256)
blur_level(LoadArgs la, float *__restrict__ out, float *__restrict__ dog,
           float *__restrict__ in_copy, int H, int W, Taps taps) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int n = NT > 0 ? NT : taps.n;
    const int r = (n - 1) / 2;
    const unsigned tb = xcd_swizzle(linear_block_id(), gridDim.x * gridDim.y * gridDim.z);
    const int x0 = (int)(tb % gridDim.x) * TX, y0 = (int)((tb / gridDim.x) % gridDim.y) * TY;
    const int f = (int)(tb / (gridDim.x * gridDim.y));
    const int tw = min(TX, W - x0), th = min(TY, H - y0);   // valid outputs of this tile
    const int IW = TX + 2 * r, IH = TY + 2 * r;
    const int IWP = IW | 1;                                  // odd row pitch: no bank conflicts
    float *tin = smem;                 // [IH][IWP]
    float *trow = smem + IH * IWP;     // [IH][TXP]
    const int tid = threadIdx.x;
    const int ih = th + 2 * r, iw = tw + 2 * r;              // staged extent actually needed

    for (int yb = 0; yb < ih; yb += 64)       // generic tap count: rows in chunks of 64
        stage_tile<MODE, 4, 16>(la, f, H, W, x0, y0 + yb, r, min(64, ih - yb), iw, IWP, tin + yb * IWP);
    __syncthreads();
    if constexpr (NT > 0) {
        // row pass: lanes walk consecutive rows (odd pitch), each SEG outputs along x
        const int nseg = (tw + SEG - 1) / SEG;
        for (int it = tid; it < ih * nseg; it += 256) {
            const int row = it % ih, sg = it / ih;
            float acc[SEG];
            row_seg<NT, SEG>(tin + row * IWP + sg * SEG, taps.k, acc);
#pragma unroll
            for (int j = 0; j < SEG; ++j) trow[row * TXP + sg * SEG + j] = acc[j];
        }
        __syncthreads();
        // column pass: lanes walk consecutive columns, each SEG outputs down y
        const int nrs = (th + SEG - 1) / SEG;
        for (int it = tid; it < tw * nrs; it += 256) {
            const int x = it % tw, rs = it / tw;
            float acc[SEG];
            col_seg<NT, SEG>(trow + rs * SEG * TXP + x, TXP, taps.k, acc);
#pragma unroll
            for (int j = 0; j < SEG; ++j) {
                const int ty = rs * SEG + j;
                if (ty >= th) break;
                const float o = acc[j];
                const size_t gi = ((size_t)f * H + y0 + ty) * W + x0 + x;
                if (out) out[gi] = o;
                const float c = tin[(ty + r) * IWP + x + r];
                if (dog) dog[gi] = o - c;
                if (in_copy) in_copy[gi] = c;
            }
        }
    } else {
        for (int i = tid; i < ih * tw; i += 256) {
            const int ty = i / tw, tx = i - ty * tw;
            trow[ty * TXP + tx] = row_one(tin + ty * IWP + tx, taps.k, n);
        }
        __syncthreads();
        for (int i = tid; i < th * tw; i += 256) {
            const int ty = i / tw, tx = i - ty * tw;
            const float o = col_one(trow + ty * TXP + tx, TXP, taps.k, n);
            const size_t gi = ((size_t)f * H + y0 + ty) * W + x0 + tx;
            if (out) out[gi] = o;
            const float c = tin[(ty + r) * IWP + tx + r];
            if (dog) dog[gi] = o - c;
            if (in_copy) in_copy[gi] = c;
        }
    }
}

// The reference's kernel sizes (compile-time NT): 512-thread workgroups, ONE LDS tile.
// Stage the (64+2r)^2 input tile; the column-pass threads keep their DoG centres in
// registers; the row pass runs in place (each thread loads its SR + NT - 1 inputs, barrier,
// writes its SR outputs over them); the column pass (SC outputs per thread, all 512 threads
// busy) writes level, DoG and level-0 copy.  Half the LDS of a two-tile design, twice the
// waves per CU; per output the arithmetic is blur_level's (sequential fma in tap order).
// Tile height per tap count: the row pass has (TYT + 2R) x 4 items and the column pass
// 64 x TYT / SC, so TYT + 2R ~ 128 keeps all 8 waves busy in both passes (a 64-row tile
// leaves 2-3 waves idle in the row pass) and cuts the row-pass halo from 2R/64 to ~2R/100.
constexpr int tall_rows(int NT) { return ((128 - (NT - 1)) / 8) * 8; }

// Small planes (octaves 2-3 of a batch: a few hundred tiles) are latency-bound, not FMA-
// bound: blur_fast<..., 32, 256> uses 32 x 32 tiles of 256 threads with 8 row-pass and 4
// column-pass outputs per thread -- a quarter of the serial FMA chain per thread and 4x the
// workgroups of the 64 x 64 form.
#ifndef PANO_BASE_ROWS
#define PANO_BASE_ROWS 88   // output rows of the base level's tall tile (0: the levels' tall_rows(NT); measured: 88 fits tile + patch in 4 workgroups per CU, profiles/r06_base_rows_ab.txt)
#endif
#ifndef PANO_BASE_PATCH
#define PANO_BASE_PATCH 1   // 0: round-5 base staging (patch for interior tiles only) for A/B
#endif
constexpr bool base_patch = PANO_BASE_PATCH != 0;

// blur_fast's DoG planes go out as nontemporal (streaming) stores: nothing reads them until the
// extrema scan after the octave's last level, and the level planes the next launch reads at
// once keep the caches.  Measured (profiles/r06_blur_nt_ab.txt, two boxes): blur class -2 to
// -4 %, pooled parrington step -1 to -3 %; the level planes nontemporal too (bit 1) slows the
// next level's reads; nontemporal DoG loads in the scan (PANO_XNT=2) slow it at 1080p.
#ifndef PANO_BLUR_NT
#define PANO_BLUR_NT 1      // bit 0: DoG stores nontemporal; bit 1: level stores too (A/B)
#endif
template <int MODE, int NT, int TYT = TY, int TXT = TX, int NTHR = 512>
__global__ void __launch_bounds__(NTHR, 6)
blur_fast(LoadArgs la, float *__restrict__ out, float *__restrict__ dog,
          float *__restrict__ in_copy, int H, int W, Taps taps) {
    constexpr int R = (NT - 1) / 2;
    constexpr int IWP = (TXT + 2 * R) | 1;
    constexpr int SR = TXT == 64 ? 16 : 8, SC = TYT * TXT / NTHR;
    constexpr bool CENTER = MODE != MODE_BASE && MODE != MODE_BASEF;
    static_assert((TYT + 2 * R) * (TXT / SR) <= NTHR && TXT * (TYT / SC) <= NTHR && TYT % SC == 0,
                  "one item per thread");
    extern __shared__ __attribute__((aligned(16))) float tin[];   // [TYT + 2R][IWP]
    const unsigned tb = xcd_swizzle(linear_block_id(), gridDim.x * gridDim.y * gridDim.z);
    const int x0 = (int)(tb % gridDim.x) * TXT, y0 = (int)((tb / gridDim.x) % gridDim.y) * TYT;
    const int f = (int)(tb / (gridDim.x * gridDim.y));
    const int tw = min(TXT, W - x0), th = min(TYT, H - y0);
    const int tid = threadIdx.x;
    const int ih = th + 2 * R, iw = tw + 2 * R;
    if constexpr ((PANO_BLUR_ABL & 4) != 0) {
        for (int i = tid; i < (TYT + 2 * R) * IWP; i += NTHR) tin[i] = (float)(i & 255);
    } else if (MODE == MODE_LEVEL && (W & 3) == 0 && x0 >= R && y0 >= R && x0 + TXT + R <= W && y0 + TYT + R <= H)
        stage_interior<R, NTHR, TYT, TXT>(la.src + (size_t)f * H * W, W, x0, y0, IWP, tin);
    else if (TXT == TX && MODE == MODE_BASE && base_patch)
        stage_base_patch<R, NTHR, TYT>(la, f, H, W, x0, y0, ih, iw, IWP, tin, tin + (TYT + 2 * R) * IWP);
    else if (TXT == TX && MODE == MODE_BASE && x0 - R >= 2 && y0 - R >= 2 && x0 + TX + R <= W - 2 &&
             y0 + TYT + R <= H - 2)
        stage_base_interior<R, NTHR, TYT>(la, f, x0, y0, IWP, tin, tin + (TYT + 2 * R) * IWP);
    else
        stage_tile<MODE, NTHR / 64, (TYT + 2 * R + NTHR / 64 - 1) / (NTHR / 64)>(la, f, H, W, x0, y0, R, ih, iw,
                                                                             IWP, tin);
    __syncthreads();
    // column-pass item of this thread and its centres (before the row pass overwrites them)
    const int nrs = (th + SC - 1) / SC;
    const bool colw = tid < tw * nrs;
    const int cxp = colw ? tid % tw : 0, crs = colw ? tid / tw : 0;
    float cen[SC];
#pragma unroll
    for (int j = 0; j < SC; ++j)
        cen[j] = (CENTER && colw) ? tin[(crs * SC + j + R) * IWP + cxp + R] : 0.0f;
    // row pass, in place: each thread reads its SR + NT - 1 inputs and accumulates its SR
    // outputs before the barrier (inputs streamed, not held), then overwrites them
    const int nseg = (tw + SR - 1) / SR;
    const bool roww = tid < ih * nseg;
    const int row = roww ? tid % ih : 0, sg = roww ? tid / ih : 0;
    float ro[SR];
    if (roww) {
        float acc[SR];
        row_seg<NT, SR>(tin + row * IWP + sg * SR, taps.k, acc);
#pragma unroll
        for (int j = 0; j < SR; ++j) ro[j] = acc[j];
    }
    __syncthreads();
    if (roww) {
#pragma unroll
        for (int j = 0; j < SR; ++j) tin[row * IWP + sg * SR + j] = ro[j];
    }
    __syncthreads();
    if (!colw) return;
    // all SC outputs first (the sliding window interleaves their FMA chains), then predicated
    // stores: an early exit in the store loop let the compiler compute one output at a time,
    // a dependent chain of NT FMAs each
    float acc[SC];
    col_seg<NT, SC>(tin + crs * SC * IWP + cxp, IWP, taps.k, acc);
    float o[SC];
#pragma unroll
    for (int j = 0; j < SC; ++j) {
        o[j] = acc[j];
        asm volatile("" ::"v"(o[j]));                           // no sinking into the stores' branches
    }
    const int nvalid = th - crs * SC;                           // rows of this item inside the plane
    const size_t g0 = ((size_t)f * H + y0 + crs * SC) * W + x0 + cxp;
#pragma unroll
    for (int j = 0; j < SC; ++j) {
        const size_t gi = g0 + (size_t)j * W;
        if (j >= nvalid) continue;
        if constexpr ((PANO_BLUR_ABL & 2) != 0) {
            if (o[j] == -1.2345f) out[gi] = o[j] + cen[j];    // never true: keeps the work live
            continue;
        }
        if constexpr ((PANO_BLUR_NT & 2) != 0) {
            if (out) __builtin_nontemporal_store(o[j], out + gi);
        } else {
            if (out) out[gi] = o[j];
        }
        if constexpr (CENTER) {
            if constexpr ((PANO_BLUR_NT & 1) != 0) {
                if (dog) __builtin_nontemporal_store(o[j] - cen[j], dog + gi);
            } else {
                if (dog) dog[gi] = o[j] - cen[j];
            }
            if (in_copy) in_copy[gi] = cen[j];
        }
    }
}

// ------------------------------------------------------------------ fused level pairs
// Two cascaded levels in ONE launch for the latency-bound octaves (a few hundred to a few
// thousand workgroups per level, ~5-20 us of launch and wave-quantisation latency each):
// a TT x TT output tile stages G[l-1] with the halo of both levels (R1 + R2), computes G[l]
// on the tile plus the next level's halo (R2), replaces the part of that region outside the
// image by its BORDER_REFLECT_101 image (what the next level reads there, exactly), writes
// G[l] / DoG[l-1] of the tile, then computes G[l+1] on the tile from the region in LDS and
// writes G[l+1] / DoG[l].  Every output is blur_fast's arithmetic (sequential fma in tap
// order, one f32 rounding per pass), hence bit-identical; the price is level l's FMAs on the
// (TT + 2 R2)^2 region, the saving one launch and one HBM round trip of G[l] per pair.
constexpr int kPairSeg = 8;     // outputs per thread item in every pass

template <int NT1, int NT2, int TT>
struct PairShape {
    static constexpr int R1 = (NT1 - 1) / 2, R2 = (NT2 - 1) / 2, RS = R1 + R2;
    static constexpr int IH = TT + 2 * RS, IWP = (TT + 2 * RS) | 1;     // staged G[l-1]
    static constexpr int RP = (TT + 2 * R2 + kPairSeg) | 1;            // row-pass pitch
    static constexpr int SP = TT + 1;                                 // side tile pitch
    static constexpr int floats = IH * IWP + kPairSeg + (IH + kPairSeg) * RP + TT * SP;
};

template <int MODE, int NT1, int NT2, int TT, int NTHR>
__global__ void __launch_bounds__(NTHR)
blur_pair(LoadArgs la, float *__restrict__ out1, float *__restrict__ dog1, float *__restrict__ in_copy,
          float *__restrict__ out2, float *__restrict__ dog2, int H, int W, Taps t1, Taps t2) {
    using S = PairShape<NT1, NT2, TT>;
    constexpr int R2 = S::R2, RS = S::RS, IWP = S::IWP, RP = S::RP, SP = S::SP;
    constexpr int SG = kPairSeg, NW = NTHR / 64;
    extern __shared__ __attribute__((aligned(16))) float smp[];
    float *tin = smp;                                   // [IH][IWP] G[l-1], then the G[l] region
    float *rb = smp + S::IH * IWP + SG;                 // [IH + SG][RP] row-pass outputs
    float *side = rb + (S::IH + SG) * RP;               // [TT][SP] G[l-1], then G[l], of the tile
    const unsigned tb = xcd_swizzle(linear_block_id(), gridDim.x * gridDim.y * gridDim.z);
    const int x0 = (int)(tb % gridDim.x) * TT, y0 = (int)((tb / gridDim.x) % gridDim.y) * TT;
    const int f = (int)(tb / (gridDim.x * gridDim.y));
    const int tw = min(TT, W - x0), th = min(TT, H - y0);
    const int tid = threadIdx.x;
    const int ih = th + 2 * RS, iw = tw + 2 * RS;
    stage_tile<MODE, NW, (S::IH + NW - 1) / NW>(la, f, H, W, x0, y0, RS, ih, iw, IWP, tin);
    __syncthreads();
    for (int i = tid; i < th * tw; i += NTHR) {
        const int y = i / tw, x = i - y * tw;
        side[y * SP + x] = tin[(y + RS) * IWP + x + RS];
    }
    // ---- level l, row pass: every staged row, region columns c = 0 .. ow1 - 1
    const int ow1 = tw + 2 * R2, oh1 = th + 2 * R2;
    {
        const int nseg = (ow1 + SG - 1) / SG;
        for (int it = tid; it < ih * nseg; it += NTHR) {
            const int row = it % ih, sg = it / ih;
            float acc[SG];
            row_seg<NT1, SG>(tin + row * IWP + sg * SG, t1.k, acc);
#pragma unroll
            for (int j = 0; j < SG; ++j) rb[row * RP + sg * SG + j] = acc[j];
        }
    }
    __syncthreads();
    // ---- level l, column pass: region rows r = 0 .. oh1 - 1, into tin (pitch IWP)
    {
        const int nrs = (oh1 + SG - 1) / SG;
        for (int it = tid; it < ow1 * nrs; it += NTHR) {
            const int c = it % ow1, rs = it / ow1;
            float acc[SG];
            col_seg<NT1, SG>(rb + rs * SG * RP + c, RP, t1.k, acc);
#pragma unroll
            for (int j = 0; j < SG; ++j)
                if (rs * SG + j < oh1) tin[(rs * SG + j) * IWP + c] = acc[j];
        }
    }
    __syncthreads();
    // ---- region positions outside the image take their reflected image value (reads only
    // inside-image positions, writes only outside ones: one pass)
    const int ry0 = y0 - R2, rx0 = x0 - R2;
    if (ry0 < 0 || rx0 < 0 || y0 + th + R2 > H || x0 + tw + R2 > W) {
        for (int i = tid; i < oh1 * ow1; i += NTHR) {
            const int r = i / ow1, c = i - r * ow1;
            const int y = ry0 + r, x = rx0 + c;
            if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) continue;
            tin[r * IWP + c] = tin[(reflect101(y, H) - ry0) * IWP + reflect101(x, W) - rx0];
        }
        __syncthreads();
    }
    // ---- level l out: G[l], DoG[l-1] (and level 0 of the octave for MODE_DOWN)
    for (int i = tid; i < th * tw; i += NTHR) {
        const int y = i / tw, x = i - y * tw;
        const float g = tin[(y + R2) * IWP + x + R2], c = side[y * SP + x];
        const size_t gi = ((size_t)f * H + y0 + y) * W + x0 + x;
        if (out1) out1[gi] = g;
        dog1[gi] = g - c;
        if (MODE == MODE_DOWN && in_copy) in_copy[gi] = c;
        side[y * SP + x] = g;
    }
    // ---- level l + 1, row pass: region rows, tile columns
    {
        const int nseg = (tw + SG - 1) / SG;
        for (int it = tid; it < oh1 * nseg; it += NTHR) {
            const int row = it % oh1, sg = it / oh1;
            float acc[SG];
            row_seg<NT2, SG>(tin + row * IWP + sg * SG, t2.k, acc);
#pragma unroll
            for (int j = 0; j < SG; ++j) rb[row * RP + sg * SG + j] = acc[j];
        }
    }
    __syncthreads();
    // ---- level l + 1, column pass and out: G[l+1], DoG[l]
    {
        const int nrs = (th + SG - 1) / SG;
        for (int it = tid; it < tw * nrs; it += NTHR) {
            const int x = it % tw, rs = it / tw;
            float acc[SG];
            col_seg<NT2, SG>(rb + rs * SG * RP + x, RP, t2.k, acc);
#pragma unroll
            for (int j = 0; j < SG; ++j) {
                const int y = rs * SG + j;
                if (y >= th) break;
                const float g = acc[j];
                const size_t gi = ((size_t)f * H + y0 + y) * W + x0 + x;
                if (out2) out2[gi] = g;
                dog2[gi] = g - side[y * SP + x];
            }
        }
    }
}

// Block barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// global stores (__syncthreads' release fence drains every outstanding HBM write of the wave,
// a few microseconds per barrier; the tail writes each level's planes while it cascades and
// nothing in the kernel reads them back).
__device__ __forceinline__ void lds_barrier() {
#if PANO_TAIL_SYNC
    __syncthreads();
#else
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#endif
}

// ------------------------------------------------------------------ fused level chains
// Two or three consecutive levels of an octave in ONE launch (the "cascade": the octave's
// levels are written once and the intermediate level planes are never read back from HBM).
// A 64 x 64 output tile stages its input level over the tile plus the chain's cumulative
// halo HT (sum of the levels' radii), then, level by level in LDS, computes the level on the
// tile plus the halo the REMAINING levels still need, in place: a row pass (RowVec_32f order)
// and a column pass (SymmColumnVec_32f order), each reading all of a thread's inputs before a
// barrier and writing its outputs after it.  Positions of the computed region outside the
// image are then replaced by their BORDER_REFLECT_101 image inside the region (the next level
// must read reflected values; a blur of reflected inputs runs its taps in the opposite order
// and rounds differently).  The column pass writes the tile's outputs: the level (when a
// later stage reads it) and its DoG against the previous level's centre values, which the
// same thread read before the row pass.  Per output the arithmetic is blur_fast's, hence
// bit-identical.  HBM per octave pixel: the input plane (chain A: a quarter-size u8 gray or
// the previous octave's level read at half resolution; chain B: G2) and the written planes,
// ~36-44 B against ~64 B for the level-by-level form.
constexpr int kCT = 64;          // output tile side
constexpr int kChainThreads = 512;

struct ChainOut {
    float *g[3];                 // the chain's levels (nullptr: not written)
    float *d[3];                 // DoG of each level against the previous (nullptr: none)
    float *gin;                  // MODE_DOWN, full pyramid: the staged level 0 (G0) plane
};

__host__ __device__ constexpr int chain_r(int nt) { return nt > 0 ? (nt - 1) / 2 : 0; }
constexpr int kChainSR = 16;     // row-pass outputs per item
constexpr int kChainSC = 10;     // column-pass outputs per item
// LDS floats of a chain whose input halo is HT: the region, plus the rows / columns the last
// (partial) segments of every level read past it (their outputs are discarded)
__host__ __device__ constexpr int chain_rows(int ht, int nt0, int nt1, int nt2) {
    int rows = kCT + 2 * ht, hin = ht;
    const int nts[3] = {nt0, nt1, nt2};
    for (int k = 0; k < 3 && nts[k] > 0; ++k) {
        const int hout = hin - chain_r(nts[k]), nout = kCT + 2 * hout;
        const int need = ((nout + kChainSC - 1) / kChainSC) * kChainSC + nts[k] - 1;
        rows = rows > need ? rows : need;
        hin = hout;
    }
    return rows + 1;
}

// One level of a chain: the region of side kCT + 2 HIN in A (pitch P, origin (y0 - HIN,
// x0 - HIN) in image coordinates) -> the level on side kCT + 2 (HIN - R), stored top-left
// aligned (origin (y0 - HOUT, x0 - HOUT)).
template <int NT, int HIN, int P, bool DOG>
__device__ __forceinline__ void chain_step(float *A, const float *__restrict__ kg, int y0, int x0, int H,
                                           int W, int th, int tw, size_t fo, float *gout, float *dout,
                                           bool border) {
    constexpr int R = (NT - 1) / 2, HOUT = HIN - R;
    // this level's taps: uniform loads into scalar registers (three Taps structs as kernel
    // arguments spilled the scalar file into VGPR lanes)
    float k[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) k[t] = kg[t];
    constexpr int NIN = kCT + 2 * HIN, NOUT = kCT + 2 * HOUT;
    constexpr int SR = kChainSR, SC = kChainSC, NT_ = kChainThreads;
    constexpr int NSR = (NOUT + SR - 1) / SR, ITR = NIN * NSR, IR = (ITR + NT_ - 1) / NT_;
    constexpr int NSC = (NOUT + SC - 1) / SC, ITC = NOUT * NSC, IC = (ITC + NT_ - 1) / NT_;
    static_assert(IR <= 2 && IC <= 3, "chain items per thread");
    const int tid = threadIdx.x;
    // (1) DoG centres: the previous level at this thread's column-pass outputs inside the
    // tile, read before the row pass overwrites the region
    float cen[IC][SC];
    if constexpr (DOG) {
#pragma unroll
        for (int it = 0; it < IC; ++it) {
            const int item = tid + it * NT_;
            const int c = item % NOUT, q = item / NOUT;
#pragma unroll
            for (int j = 0; j < SC; ++j) {
                const int rr = q * SC + j;
                const bool in = item < ITC && rr >= HOUT && rr < HOUT + kCT && c >= HOUT && c < HOUT + kCT;
                cen[it][j] = in ? A[(rr + R) * P + c + R] : 0.0f;
            }
        }
    }
    // (2) row pass, in place (left-aligned): every item's inputs are read before the barrier
    float ro[IR][SR];
#pragma unroll
    for (int it = 0; it < IR; ++it) {
        const int item = tid + it * NT_;
        if (item < ITR) {
            const int r = item % NIN, sg = item / NIN;
            row_seg<NT, SR>(A + r * P + sg * SR, k, ro[it]);
        }
    }
    lds_barrier();
#pragma unroll
    for (int it = 0; it < IR; ++it) {
        const int item = tid + it * NT_;
        if (item < ITR) {
            const int r = item % NIN, sg = item / NIN;
#pragma unroll
            for (int j = 0; j < SR; ++j)
                if (sg * SR + j < NOUT) A[r * P + sg * SR + j] = ro[it][j];
        }
    }
    lds_barrier();
    // (3) column pass, in place (top-aligned), with the tile's outputs
    float co[IC][SC];
#pragma unroll
    for (int it = 0; it < IC; ++it) {
        const int item = tid + it * NT_;
        if (item < ITC) {
            const int c = item % NOUT, q = item / NOUT;
            col_seg<NT, SC>(A + q * SC * P + c, P, k, co[it]);
        }
    }
    lds_barrier();
#pragma unroll
    for (int it = 0; it < IC; ++it) {
        const int item = tid + it * NT_;
        if (item < ITC) {
            const int c = item % NOUT, q = item / NOUT;
            const int tx = c - HOUT;
#pragma unroll
            for (int j = 0; j < SC; ++j) {
                const int rr = q * SC + j;
                if (rr >= NOUT) break;
                A[rr * P + c] = co[it][j];
                const int ty = rr - HOUT;
                if (ty >= 0 && ty < th && tx >= 0 && tx < tw) {
                    const size_t gi = fo + (size_t)(y0 + ty) * W + x0 + tx;
                    if (gout) gout[gi] = co[it][j];
                    if constexpr (DOG) dout[gi] = co[it][j] - cen[it][j];
                }
            }
        }
    }
    lds_barrier();
    // (4) BORDER_REFLECT_101 of the region positions outside the image (reads inside
    // positions, writes outside ones: one pass).  Positions whose reflection falls outside the
    // region lie beyond what any later output reads, and are left as they are.
    if constexpr (HOUT > 0) {
        if (border) {
            const int oy = y0 - HOUT, ox = x0 - HOUT;
            for (int i = tid; i < NOUT * NOUT; i += NT_) {
                const int r = i / NOUT, c = i - r * NOUT;
                const int y = oy + r, x = ox + c;
                if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) continue;
                const int sr = reflect101(y, H) - oy, sc = reflect101(x, W) - ox;
                if ((unsigned)sr < (unsigned)NOUT && (unsigned)sc < (unsigned)NOUT) A[r * P + c] = A[sr * P + sc];
            }
            lds_barrier();
        }
    }
}

// MODE_BASE chains start at the base level (no DoG for it); the other modes' first level
// has a DoG against the staged level 0.
template <int MODE, int NT0, int NT1, int NT2>
__global__ void __launch_bounds__(kChainThreads, 4)
blur_chain(LoadArgs la, ChainOut co, int H, int W, const float *__restrict__ taps, int l0) {
    constexpr int HT = chain_r(NT0) + chain_r(NT1) + chain_r(NT2);
    constexpr int RS = kCT + 2 * HT, P = RS | 1;
    static_assert(RS <= 128, "stage_tile covers 128 columns");
    extern __shared__ __attribute__((aligned(16))) float A[];
    const unsigned tb = xcd_swizzle(linear_block_id(), gridDim.x * gridDim.y * gridDim.z);
    const int x0 = (int)(tb % gridDim.x) * kCT, y0 = (int)((tb / gridDim.x) % gridDim.y) * kCT;
    const int f = (int)(tb / (gridDim.x * gridDim.y));
    const int tw = min(kCT, W - x0), th = min(kCT, H - y0);
    const size_t fo = (size_t)f * H * W;
    constexpr int NW = kChainThreads / 64;
    // the whole region, reflected at the image borders (partial tiles included: every level
    // then computes finite values everywhere)
    stage_tile<MODE, NW, (RS + NW - 1) / NW>(la, f, H, W, x0, y0, HT, RS, RS, P, A);
    lds_barrier();
    if (MODE == MODE_DOWN && co.gin) {
        for (int i = threadIdx.x; i < kCT * kCT; i += kChainThreads) {
            const int ty = i / kCT, tx = i - ty * kCT;
            if (ty < th && tx < tw) co.gin[fo + (size_t)(y0 + ty) * W + x0 + tx] = A[(ty + HT) * P + tx + HT];
        }
    }
    const bool border = y0 - HT < 0 || x0 - HT < 0 || y0 + kCT + HT > H || x0 + kCT + HT > W;
    constexpr bool FIRST_DOG = MODE != MODE_BASE && MODE != MODE_BASEF;
    // taps rows: [level][PANO_MAX_TAPS], the chain's levels l0, l0 + 1, l0 + 2 (row 0 = the base)
    const float *k0 = taps + l0 * PANO_MAX_TAPS;
    chain_step<NT0, HT, P, FIRST_DOG>(A, k0, y0, x0, H, W, th, tw, fo, co.g[0], co.d[0], border);
    if constexpr (NT1 > 0)
        chain_step<NT1, HT - chain_r(NT0), P, true>(A, k0 + PANO_MAX_TAPS, y0, x0, H, W, th, tw, fo, co.g[1],
                                                    co.d[1], border);
    if constexpr (NT2 > 0)
        chain_step<NT2, HT - chain_r(NT0) - chain_r(NT1), P, true>(A, k0 + 2 * PANO_MAX_TAPS, y0, x0, H, W, th,
                                                                  tw, fo, co.g[2], co.d[2], border);
}

template <int MODE, int NT0, int NT1, int NT2>
int launch_chain(pano_ctx *ctx, const LoadArgs &la, const ChainOut &co, int n, int H, int W, int l0) {
    constexpr int HT = chain_r(NT0) + chain_r(NT1) + chain_r(NT2);
    constexpr int P = (kCT + 2 * HT) | 1;
    const size_t sm = (size_t)chain_rows(HT, NT0, NT1, NT2) * P * sizeof(float);
    static bool attr = false;
    if (!attr) {
        PANO_HIP(ctx, hipFuncSetAttribute((const void *)blur_chain<MODE, NT0, NT1, NT2>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm));
        attr = true;
    }
    dim3 grid((W + kCT - 1) / kCT, (H + kCT - 1) / kCT, n);
    {
        PanoProf prof_(ctx, PK_BLUR);
        blur_chain<MODE, NT0, NT1, NT2><<<grid, kChainThreads, sm, ctx->stream>>>(la, co, H, W, ctx->taps, l0);
    }
    PANO_LAUNCH_CHECK(ctx, "blur_chain");
    return PANO_OK;
}

// ------------------------------------------------------------------ streaming cascade
// Two or three consecutive levels of an octave in ONE launch WITHOUT the 2-D halo of the tile
// chains above: a workgroup owns a strip of kCasSW output columns of one band of rows and
// WALKS DOWN it, kCasK rows (one "chunk") per step.  Level j keeps its row-pass output (T_j)
// in an LDS ring of 2 d_j + 1 chunks, d_j = ceil(R_j / K): the column pass of chunk c needs T_j
// rows up to R_j beyond it, so level j runs d_j chunks behind its row pass, and level j+1's
// row pass consumes level j's chunk as soon as it is produced (from the staging buffer S).
// Vertically every intermediate row is computed once (only the band edges recompute the
// later levels' radii); horizontally level j is computed on the strip plus the halo the
// remaining levels need (sum of their radii).  The written planes are only those later
// stages read (the levels asked for and the DoGs); the intermediate levels never touch HBM.
//
// Wave roles.  Waves 0..3 compute and touch only LDS.  Wave 4 (the store wave) writes the
// outputs of the previous step to HBM from owned-column rings of every level (the DoG is its
// subtraction), and wave 5 (the loader) fetches the next chunk of the input level while the
// current one is computed.  On gfx9 a wait for a load also waits for every store issued
// before it (vmcnt is in order): a compute wave that stored its outputs would stall on HBM
// write latency at its next load; here no wave that waits on a load ever stores.
//
// Exactness: per output the arithmetic is blur_fast's -- RowVec_32f's sequential f32 FMA over
// the taps, SymmColumnVec_32f's symmetric column form -- with BORDER_REFLECT_101 taken on the
// LEVEL values: image rows outside the plane are read at their reflected row (the ring holds
// every row a chunk needs, reflected ones included), and the columns of S outside the plane
// are overwritten with their mirror before the next level reads them (a blur of reflected
// inputs would run its taps in the opposite order and round differently).  Hence the same
// bits as the level-by-level launches.  The taps are the reference's default ones compiled in
// (cas_taps.h, tools/gen_cas_taps.py); the launcher uses the cascade only when the run-time
// taps equal them bit for bit.
constexpr int kCasK = 8;                 // rows per step (one chunk)
constexpr int kCasSW = 64;               // owned output columns of a strip
constexpr int kCasCW = 4;                // compute waves
constexpr int kCasThreads = 64 * (kCasCW + 2);
constexpr int kCasStoreWave = kCasCW, kCasLoadWave = kCasCW + 1;
constexpr int kCasSR = 4;                // row-pass outputs per item
constexpr int kCasSC = kCasK / 2;        // column-pass outputs per item (two row halves)

struct CasOut {
    float *gin;                          // MODE_DOWN: the input (the octave's G0), or null
    float *g[3];                         // level j at its owned positions, or null
    float *d[3];                         // level j minus its predecessor (the input for j = 0), or null
};

template <int NL, int L0, bool HAS_IN>
struct Cas {
    static constexpr int nt(int j) { return kCasDefTaps[L0 + j]; }
    static constexpr int r(int j) { return (nt(j) - 1) / 2; }
    static constexpr int hx(int j) {     // rows / columns level j computes beyond the owned ones
        int s = 0;
        for (int i = j + 1; i < NL; ++i) s += r(i);
        return s;
    }
    static constexpr int hin() { return hx(0) + r(0); }
    static constexpr int w(int j) { return kCasSW + 2 * hx(j); }
    static constexpr int nsg(int j) { return (w(j) + kCasSR - 1) / kCasSR; }
    static constexpr int pt(int j) { return (nsg(j) * kCasSR) | 1; }             // T ring pitch (odd)
    static constexpr int d(int j) { return (r(j) + kCasK - 1) / kCasK; }         // chunk lookahead
    static constexpr int ns(int j) { return 2 * d(j) + 1; }                      // T ring chunks
    static constexpr int lag(int j) {
        int s = 0;
        for (int i = 0; i < j; ++i) s += d(i);
        return s;
    }
    static constexpr int win() { return w(0) + 2 * r(0); }
    static constexpr int pin() { return (nsg(0) * kCasSR + nt(0) - 1) | 1; }    // IN pitch (odd)
    static constexpr int ps() {                                                  // S pitch (odd)
        int m = 1;
        for (int j = 1; j < NL; ++j) {
            const int q = nsg(j) * kCasSR + nt(j) - 1;
            m = m > q ? m : q;
        }
        return m | 1;
    }
    // owned-column rings read by the store wave: level j's rows are kept until its successor's
    // DoG is stored (d_{j+1} steps later, plus the store's own step); the input's until DoG 0
    static constexpr int gs(int j) { return j + 1 < NL ? d(j + 1) + 2 : 2; }
    static constexpr int is() { return HAS_IN ? d(0) + 3 : 0; }
    static constexpr int off_s() { return kCasK * pin(); }
    static constexpr int off_t(int j) {
        int o = off_s() + kCasK * ps();
        for (int i = 0; i < j; ++i) o += ns(i) * kCasK * pt(i);
        return o;
    }
    static constexpr int off_g(int j) {
        int o = off_t(NL);
        for (int i = 0; i < j; ++i) o += gs(i) * kCasK * kCasSW;
        return o;
    }
    static constexpr int off_i() { return off_g(NL); }
    static constexpr int floats() { return off_i() + is() * kCasK * kCasSW; }
};

#ifndef PANO_CAS_TIMING
#define PANO_CAS_TIMING 0     // 1: per-phase clock stamps of one workgroup (diagnostics build)
#endif
#if PANO_CAS_TIMING
__device__ unsigned long long g_cas_clock[3][96][16];   // [compute / store / load wave][step][event]
#define PANO_CAS_STAMP(role, ev)                                                                      \
    do {                                                                                            \
        if (lane == 0 && blockIdx.x == PANO_CAS_TIMING - 1 && blockIdx.y == 0 && blockIdx.z == 0 && s < 96) \
            g_cas_clock[role][s][ev] = __builtin_amdgcn_s_memtime();                                 \
    } while (0)
#else
#define PANO_CAS_STAMP(role, ev) do {} while (0)
#endif

template <int MODE, int NL, int L0>
__global__ void __launch_bounds__(kCasThreads)
blur_cascade(LoadArgs la, CasOut co, int H, int W, int BH) {
    constexpr bool HAS_IN = MODE != MODE_BASE && MODE != MODE_BASEF;   // the input is a level
    using S = Cas<NL, L0, HAS_IN>;
    static_assert(S::win() <= 128 && S::w(0) <= 128, "two staged columns per lane, one column per col item");
    static_assert(kCasK * S::nsg(0) <= 64 * kCasCW, "one row-pass item per compute thread");
    static_assert(kCasK == 8 && kCasCW == 4, "two row halves over waves 0-1 / 2-3");
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const unsigned tb = xcd_swizzle(linear_block_id(), gridDim.x * gridDim.y * gridDim.z);
    const int sx = (int)(tb % gridDim.x), by = (int)((tb / gridDim.x) % gridDim.y);
    const int f = (int)(tb / (gridDim.x * gridDim.y));
    const int ox0 = sx * kCasSW, ox1 = min(W, ox0 + kCasSW);      // owned columns
    const int xs = min(ox0, W - kCasSW);                            // strip origin (W >= kCasSW)
    const int yb0 = by * BH, yb1 = min(H, yb0 + BH);               // owned rows
    const int ybase = max(0, yb0 - S::hin()), yend = min(H, yb1 + S::hin());
    int Y[NL], E[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) {
        Y[j] = max(0, yb0 - S::hx(j));
        E[j] = min(H, yb1 + S::hx(j));
    }
    const int nsteps = ((E[NL - 1] - 1 - ybase) >> 3) + S::lag(NL - 1) + S::d(NL - 1) + 1;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool border = xs - S::hx(0) < 0 || xs + kCasSW + S::hx(0) > W;
    const size_t fo = (size_t)f * H * W;
    float *IN = lds, *SB = lds + S::off_s();

    // ---- the loader: chunk c of the input level (reflected columns) into registers, then
    // into IN (and its owned columns into the input ring) once the current step is done with IN
    const Stager<MODE> sg(la, f, H, W);
    const bool has1 = 64 + lane < S::win();
    const ColMap m0 = sg.col(xs - S::hin() + lane);
    const ColMap m1 = sg.col(xs - S::hin() + (has1 ? 64 + lane : lane));
    float lv0[kCasK], lv1[kCasK];
    auto load_issue = [&](int c) {
        // branch-free: rows past the input's end load the last row again (never stored), lanes
        // without a second column load their first column twice, so all 16 loads are in flight
        // together (a predicated load made the compiler wait for each one before the next)
        const int r0 = ybase + c * kCasK;
#pragma unroll
        for (int q = 0; q < kCasK; ++q) {
            const int rr = min(r0 + q, yend - 1);
            lv0[q] = sg.get(rr, m0);
            lv1[q] = sg.get(rr, m1);
        }
    };
    auto load_commit = [&](int c) {
        const int r0 = ybase + c * kCasK;
#pragma unroll
        for (int q = 0; q < kCasK; ++q) {
            if (r0 + q < yend) {
                if (lane < S::win()) IN[q * S::pin() + lane] = lv0[q];
                if (has1) IN[q * S::pin() + 64 + lane] = lv1[q];
            }
        }
        if constexpr (HAS_IN) {
            // the wave's own LDS writes are in order: read the owned centres back
            float *ring = lds + S::off_i() + (c % S::is()) * kCasK * kCasSW;
#pragma unroll
            for (int q = 0; q < kCasK; ++q)
                if (r0 + q < yend) ring[q * kCasSW + lane] = IN[q * S::pin() + lane + S::hin()];
        }
    };
    // ---- the store wave: level j's outputs produced at step s, from the rings (all the
    // chunk's LDS reads first, then its stores)
    const int sgx = xs + lane;
    const bool own_c = sgx >= ox0 && sgx < ox1;
    // 16-byte output rows: plane rows and the strip 4-float aligned, owned range on 4-column groups
    const bool vec4 = (W & 3) == 0 && (xs & 3) == 0 && ((ox0 - xs) & 3) == 0 && ((ox1 - xs) & 3) == 0;
    auto store_level = [&](auto jc, int s) {
        constexpr int j = decltype(jc)::value;
        const int cg = s - S::lag(j) - S::d(j);
        if (cg < 0 || (!co.g[j] && !co.d[j])) return;
        const int g0 = ybase + cg * kCasK;
        const int lo = max(g0, yb0), hi = min(g0 + kCasK, yb1);
        if (lo >= hi) return;
        const float *gr = lds + S::off_g(j) + (cg % S::gs(j)) * kCasK * kCasSW + lane;
        const float *pr = nullptr;
        if constexpr (j > 0) pr = lds + S::off_g(j > 0 ? j - 1 : 0) + (cg % S::gs(j > 0 ? j - 1 : 0)) * kCasK * kCasSW + lane;
        else if constexpr (HAS_IN) pr = lds + S::off_i() + (cg % (S::is() > 0 ? S::is() : 1)) * kCasK * kCasSW + lane;
        if (vec4) {
            // 16-byte stores: lane = (row 0..3 of a half chunk, 4-column group); a wave keeps at
            // most 63 stores in flight, so fewer, wider ones keep the store wave off the barriers
            const int qh = lane >> 4, cgp = (lane & 15) * 4;
            const bool own4 = cgp >= ox0 - xs && cgp < ox1 - xs;
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                const int q = half * 4 + qh, y = g0 + q;
                const float4 gv = *(const float4 *)(gr - lane + q * kCasSW + cgp);
                float4 dv = gv;
                if (pr) {
                    const float4 pv = *(const float4 *)(pr - lane + q * kCasSW + cgp);
                    dv = make_float4(gv.x - pv.x, gv.y - pv.y, gv.z - pv.z, gv.w - pv.w);
                }
                if (!own4 || y < lo || y >= hi) continue;
                const size_t gi = fo + (size_t)y * W + xs + cgp;
                if (co.g[j]) *(float4 *)(co.g[j] + gi) = gv;
                if (co.d[j] && pr) *(float4 *)(co.d[j] + gi) = dv;
            }
            return;
        }
        float v[kCasK], dv[kCasK];
#pragma unroll
        for (int q = 0; q < kCasK; ++q) {
            v[q] = gr[q * kCasSW];
            dv[q] = pr ? v[q] - pr[q * kCasSW] : 0.0f;
        }
        if (!own_c) return;
#pragma unroll
        for (int q = 0; q < kCasK; ++q) {
            const int y = g0 + q;
            if (y < lo || y >= hi) continue;
            const size_t gi = fo + (size_t)y * W + sgx;
            if (co.g[j]) co.g[j][gi] = v[q];
            if (co.d[j] && pr) co.d[j][gi] = dv[q];
        }
    };
    auto store_input = [&](int s) {
        // the input chunk s (MODE_DOWN: the octave's G0 plane when a full pyramid is asked)
        if constexpr (HAS_IN) {
            if (!co.gin || !own_c) return;
            const int g0 = ybase + s * kCasK;
            const float *ir = lds + S::off_i() + (s % S::is()) * kCasK * kCasSW + lane;
            float v[kCasK];
#pragma unroll
            for (int q = 0; q < kCasK; ++q) v[q] = ir[q * kCasSW];
#pragma unroll
            for (int q = 0; q < kCasK; ++q) {
                const int y = g0 + q;
                if (y >= max(g0, yb0) && y < min(g0 + kCasK, yb1)) co.gin[fo + (size_t)y * W + sgx] = v[q];
            }
        }
    };

    if (wv == kCasLoadWave) {
        load_issue(0);
        load_commit(0);
    }
    lds_barrier();
    for (int s = 0; s < nsteps; ++s) {
        [[maybe_unused]] int ev = 0;
        if (wv == 0) PANO_CAS_STAMP(0, ev);
        if (wv == kCasLoadWave) { PANO_CAS_STAMP(2, 0); load_issue(s + 1); PANO_CAS_STAMP(2, 1); }
        else if (wv == kCasStoreWave && s > 0) store_input(s - 1);
        auto level = [&](auto jc) {
            constexpr int j = decltype(jc)::value;
            constexpr int NT = S::nt(j), R = S::r(j);
            constexpr const float *KT = kCasDefK[L0 + j];
            if (wv == kCasStoreWave && s > 0) {
                PANO_CAS_STAMP(1, 2 * j);
                store_level(jc, s - 1);   // beside the row pass
                PANO_CAS_STAMP(1, 2 * j + 1);
            }
            // ---- row pass of level j, chunk ct (the input's chunk for j = 0, else the chunk
            // of level j - 1 its column pass just left in S)
            const int ct = s - S::lag(j);
            const int t0 = ybase + ct * kCasK;
            const int tlo = max(t0, j == 0 ? ybase : Y[j > 0 ? j - 1 : 0]);
            const int thi = min(t0 + kCasK, j == 0 ? yend : E[j > 0 ? j - 1 : 0]);
            if (wv < kCasCW && ct >= 0 && tlo < thi) {
                const int q = tid / S::nsg(j), g = tid - q * S::nsg(j);
                const int y = t0 + q;
                if (q < kCasK && y >= tlo && y < thi) {
                    const float *src = (j == 0 ? IN + q * S::pin() : SB + q * S::ps()) + g * kCasSR;
                    float acc[kCasSR];
                    row_seg<NT, kCasSR>(src, KT, acc);
                    float *dst = lds + S::off_t(j) + ((ct % S::ns(j)) * kCasK + q) * S::pt(j) + g * kCasSR;
#pragma unroll
                    for (int k = 0; k < kCasSR; ++k) dst[k] = acc[k];
                }
            }
            lds_barrier();
            if (wv == 0) PANO_CAS_STAMP(0, ++ev);
            // ---- column pass of level j, chunk cg = ct - d_j: two row halves, one column per
            // lane; rows (and their ring slots) are wave-uniform
            const int cg = ct - S::d(j);
            const int g0 = ybase + cg * kCasK;
            const int glo = max(g0, Y[j]), ghi = min(g0 + kCasK, E[j]);
            const int h = wv >> 1, i = lane + 64 * (wv & 1);
            if (wv < kCasCW && cg >= 0 && glo < ghi && i < S::w(j)) {
                constexpr int NV = kCasSC + 2 * R, RS = S::ns(j) * kCasK;   // ring rows
                const float *T = lds + S::off_t(j) + i;
                const int yt = g0 + h * kCasSC - R;                          // first tap row
                float v[NV];
                if (yt >= 0 && yt + NV <= H) {
                    // no reflection: consecutive ring rows, wrapping once
                    int p = (yt - ybase) % RS;
#pragma unroll
                    for (int k = 0; k < NV; ++k) {
                        v[k] = T[p * S::pt(j)];
                        p = p + 1 == RS ? 0 : p + 1;
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < NV; ++k) {
                        int lr = reflect101(yt + k, H) - ybase;
                        lr = lr < 0 ? 0 : lr;                 // rows no valid output reads
                        v[k] = T[(lr % RS) * S::pt(j)];
                    }
                }
                float o[kCasSC];
#pragma unroll
                for (int qq = 0; qq < kCasSC; ++qq) o[qq] = v[qq + R] * KT[R];
#pragma unroll
                for (int dd = 1; dd <= R; ++dd)
#pragma unroll
                    for (int qq = 0; qq < kCasSC; ++qq)
                        o[qq] = __builtin_fmaf(v[qq + R + dd] + v[qq + R - dd], KT[R + dd], o[qq]);
#pragma unroll
                for (int qq = 0; qq < kCasSC; ++qq) asm volatile("" ::"v"(o[qq]));   // all outputs first
                const int hc = i - S::hx(j);                              // owned column index
                const bool own = hc >= 0 && hc < kCasSW;
                float *gr = lds + S::off_g(j) + (cg % S::gs(j)) * kCasK * kCasSW + hc;
#pragma unroll
                for (int qq = 0; qq < kCasSC; ++qq) {
                    const int qr = h * kCasSC + qq, y = g0 + qr;
                    if (y < glo || y >= ghi) continue;
                    if (j + 1 < NL) SB[qr * S::ps() + i] = o[qq];
                    if (own) gr[qr * kCasSW] = o[qq];
                }
            }
            lds_barrier();
            if (wv == 0) PANO_CAS_STAMP(0, ++ev);
            if (j + 1 < NL && border && cg >= 0 && glo < ghi) {
                // S's columns outside the plane <- their BORDER_REFLECT_101 mirror
                constexpr int WJ = S::w(j);
                if (wv < kCasCW) {
                    for (int e = tid; e < kCasK * WJ; e += 64 * kCasCW) {
                        const int q = e / WJ, ii = e - q * WJ;
                        const int gx = xs - S::hx(j) + ii;
                        if (gx >= 0 && gx < W) continue;
                        SB[q * S::ps() + ii] = SB[q * S::ps() + reflect101(gx, W) - (xs - S::hx(j))];
                    }
                }
                lds_barrier();
            }
        };
        level(std::integral_constant<int, 0>{});
        if constexpr (NL > 1) level(std::integral_constant<int, 1>{});
        if constexpr (NL > 2) level(std::integral_constant<int, 2>{});
        if (wv == kCasLoadWave) { PANO_CAS_STAMP(2, 2); load_commit(s + 1); PANO_CAS_STAMP(2, 3); }
        lds_barrier();
        if (wv == 0) PANO_CAS_STAMP(0, 15);
    }
    if (wv == kCasStoreWave) {
        store_input(nsteps - 1);
        store_level(std::integral_constant<int, 0>{}, nsteps - 1);
        if constexpr (NL > 1) store_level(std::integral_constant<int, 1>{}, nsteps - 1);
        if constexpr (NL > 2) store_level(std::integral_constant<int, 2>{}, nsteps - 1);
    }
}

template <int MODE, int NL, int L0>
int launch_cascade(pano_ctx *ctx, const LoadArgs &la, const CasOut &co, int n, int H, int W, int BH) {
    using S = Cas<NL, L0, MODE != MODE_BASE && MODE != MODE_BASEF>;
    const size_t sm = (size_t)S::floats() * sizeof(float);
    static bool attr = false;
    if (!attr) {
        PANO_HIP(ctx, hipFuncSetAttribute((const void *)blur_cascade<MODE, NL, L0>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm));
        attr = true;
    }
    dim3 grid((W + kCasSW - 1) / kCasSW, (H + BH - 1) / BH, n);
    {
        PanoProf prof_(ctx, PK_BLUR);
        blur_cascade<MODE, NL, L0><<<grid, kCasThreads, sm, ctx->stream>>>(la, co, H, W, BH);
    }
    PANO_LAUNCH_CHECK(ctx, "blur_cascade");
    return PANO_OK;
}

// ------------------------------------------------------------------ small-octave tail
// Octaves whose levels fit one 64 x 64 tile are latency-bound as separate launches (one
// tiny workgroup per frame, ~7 us each, 5 per octave).  blur_tail runs them all in ONE
// launch: a 512-thread workgroup per frame keeps the current level in LDS and cascades
// level by level, octave by octave (nearest 1/2 of level n_lvl-3 seeds the next octave),
// writing every Gaussian level and DoG to HBM.  No halo copy: the row pass computes only
// the H image rows (a reflected halo row IS the row pass of an image row), reading its
// reflected columns directly; the column pass reads reflected rows of the row-pass output.
// Two barriers per level.  Odd LDS pitch (65): lanes on consecutive rows / columns are
// bank-conflict free.  Per output it is blur_level's arithmetic (sequential fma in tap
// order, one f32 rounding per pass), hence bit-identical.
#ifndef PANO_TAIL_DIM
#define PANO_TAIL_DIM 64                      // octaves whose planes fit this square join the tail
#endif
#ifndef PANO_TAIL_THREADS
#define PANO_TAIL_THREADS 512
#endif
constexpr int kTailDim = PANO_TAIL_DIM;
constexpr int kTailOct = 8;
constexpr int kTP = kTailDim + 1;             // LDS pitch
constexpr int kTailThreads = PANO_TAIL_THREADS;

struct TailArgs {
    const float *prev;                          // G[o_tail-1][n_lvl-3], frame stride ph*pw
    int ph, pw;
    float *G[kTailOct][PANO_MAX_LEVELS];        // level planes (frame 0)
    float *D[kTailOct][PANO_MAX_LEVELS];        // DoG planes (frame 0)
    int H[kTailOct], W[kTailOct];
    int n_oct, n_lvl;
    int full;                                   // write level 0 and the top level too
    const float *taps;                          // [n_lvl][PANO_MAX_TAPS], level 0 unused
    int ntap[PANO_MAX_LEVELS];
};

__device__ __forceinline__ int tail_src(int d, double inv) {   // OpenCV INTER_NEAREST
    return (int)floor(d * inv);
}

// Tail LDS layout.  A level plane is stored with its BORDER_REFLECT_101 columns already in
// place: row y at y * kPP, image column x at kOff + x, and the mirrored columns the NEXT
// level's row pass reads (x in [-Rn, 0) and [W, W + Rn)) written by the thread that
// computes column x's value (tail_mirrors).  Likewise the row pass writes each row-pass
// output row also to the mirrored rows [-R, 0) and [H, H + R) of rowt (a reflected halo row
// IS the row pass of an image row).  So a level is two phases and two barriers: the row pass
// over the H image rows from the padded plane into rowt, and the column pass reading rowt
// rows through the octave's table of reflected row offsets (rowix: a wave-uniform LDS read
// per tap row), writing the next padded plane, its mirrors, the Gaussian level and the DoG.
constexpr int kRMax = (PANO_MAX_TAPS - 1) / 2;
constexpr int kOff = kRMax;                               // padded column of image column 0
constexpr int kPP = (kTailDim + 2 * kRMax) | 1;           // padded plane pitch (odd)
constexpr int kRowIx = kTailDim + 2 * kRMax + 8;          // reflected row table (+ SG overrun)

// call f(m) for every m of [-Rn, 0) u [n, n + Rn) whose BORDER_REFLECT_101 source is x (the
// reflection has period P = 2n - 2: sources x + kP and -x + kP)
template <typename F>
__device__ __forceinline__ void tail_mirrors(int x, int n, int Rn, F f) {
    if (Rn <= 0) return;
    if (n == 1) {
        for (int m = 1; m <= Rn; ++m) { f(-m); f(m); }
        return;
    }
    const int P = 2 * n - 2;
    for (int m = x - P; m >= -Rn; m -= P) f(m);
    for (int m = x + P; m < n + Rn; m += P) f(m);
    if (x != 0 && x != n - 1) {                          // x = 0 / n - 1: the same positions
        for (int m = -x; m >= -Rn; m -= P) f(m);
        for (int m = P - x; m < n + Rn; m += P) f(m);
    }
}

// One tail level: compile-time tap count NT with SG outputs per thread item (register-blocked
// sliding windows, taps in tap order: blur_level's arithmetic), or NT = 0: runtime count n,
// one output per item.  in / outp: padded planes (column 0 at kOff); rowt: [kTailDim][kTP];
// rowix[kRMax + r] = kTP * reflect101(r, H) for r in [-kRMax, H + kRMax).
// LDS / global address-space pointers: tail_level is a real call (inlining its ten
// instances into blur_tail ran out of scalar registers), so its pointer arguments carry
// their address space explicitly -- plain pointers would become flat accesses.
typedef __attribute__((address_space(3))) float lds_f32;
typedef __attribute__((address_space(3))) int lds_i32;
typedef __attribute__((address_space(1))) float gbl_f32;

template <int NT, int SG>
__device__ __noinline__ void tail_level(const lds_f32 *in, lds_f32 *outp, lds_f32 *rowt, const lds_i32 *rowix,
                                        int H, int W, int Rn, const lds_f32 *__restrict__ taps_g, int n_rt,
                                        gbl_f32 *g, gbl_f32 *d, int tid) {
    const int n = NT > 0 ? NT : n_rt;
    const int R = (n - 1) / 2;
    float k[NT > 0 ? NT : 1];
    if constexpr (NT > 0) {
#pragma unroll
        for (int t = 0; t < NT; ++t) k[t] = taps_g[t];
    }
    // row pass: item = (row y, segment of SG columns); lanes on consecutive rows
    const int nseg = (W + SG - 1) / SG;
    for (int it = tid; it < H * nseg; it += kTailThreads) {
        const int y = it % H, x0 = (it / H) * SG;
        const lds_f32 *p = in + y * kPP + kOff - R + x0;
        float acc[SG];
        if constexpr (NT > 0) {
            row_seg<NT, SG>(p, k, acc);
        } else {
#pragma unroll
            for (int j = 0; j < SG; ++j) acc[j] = row_one(p + j, taps_g, n);
        }
#pragma unroll
        for (int j = 0; j < SG; ++j)
            if (x0 + j < W) rowt[y * kTP + x0 + j] = acc[j];
    }
    lds_barrier();
    // column pass: item = (column x, segment of SG rows); lanes on consecutive columns
    const int nrs = (H + SG - 1) / SG;
    for (int it = tid; it < W * nrs; it += kTailThreads) {
        const int x = it % W, y0 = (it / W) * SG;
        // rows y0 - R ... through the octave's reflected row table (offsets into rowt)
        const lds_i32 *rix = rowix + kRMax + y0;
        float acc[SG];
        if constexpr (NT > 0) {
            constexpr int RR = (NT - 1) / 2;
            float v[SG + NT - 1];
#pragma unroll
            for (int i = 0; i < SG + NT - 1; ++i) v[i] = rowt[rix[i - RR] + x];
#pragma unroll
            for (int j = 0; j < SG; ++j) acc[j] = v[j + RR] * k[RR];
#pragma unroll
            for (int dd = 1; dd <= RR; ++dd)
#pragma unroll
                for (int j = 0; j < SG; ++j) acc[j] = __builtin_fmaf(v[j + RR + dd] + v[j + RR - dd], k[RR + dd], acc[j]);
        } else {
#pragma unroll
            for (int j = 0; j < SG; ++j) {
                float a = rowt[rix[j] + x] * taps_g[R];
                for (int dd = 1; dd <= R; ++dd)
                    a = __builtin_fmaf(rowt[rix[j + dd] + x] + rowt[rix[j - dd] + x], taps_g[R + dd], a);
                acc[j] = a;
            }
        }
#pragma unroll
        for (int j = 0; j < SG; ++j) {
            const int y = y0 + j;
            if (y >= H) break;
            const float o = acc[j];
            lds_f32 *orow = outp + y * kPP + kOff;
            orow[x] = o;
            tail_mirrors(x, W, Rn, [&](int m) { orow[m] = o; });
            if (g) g[y * W + x] = o;
            d[y * W + x] = o - in[y * kPP + kOff + x];
        }
    }
}

#ifndef PANO_TAIL_GENERIC
#define PANO_TAIL_GENERIC 0   // 1: every tail level through the runtime tap-count loops (small code)
#endif
#ifndef PANO_TAIL_TIMING
#define PANO_TAIL_TIMING 0    // 1: frame 0's workgroup records s_memtime after every level (diagnostics)
#endif
#if PANO_TAIL_TIMING
__device__ unsigned long long g_tail_clock[64];
#define PANO_TAIL_STAMP(i) \
    do { if (f == 0 && tid == 0 && (i) < 64) g_tail_clock[(i)] = (unsigned long long)__builtin_amdgcn_s_memtime(); } while (0)
#else
#define PANO_TAIL_STAMP(i) do {} while (0)
#endif

__global__ void __launch_bounds__(kTailThreads)
blur_tail(TailArgs ta) {
    __shared__ float taps_s[PANO_MAX_LEVELS * PANO_MAX_TAPS];   // every level's taps, loaded once
    __shared__ float lv[3][kTailDim * kPP];      // padded planes: current / next level, octave seed
    __shared__ float rowt[kTailDim * kTP];        // row-pass output
    __shared__ int rowix[kRowIx];                 // reflected row offsets into rowt
    // the tail is a latency chain of 18 workgroups running beside the extrema scan, which
    // fills every CU: raise its waves' issue priority so the chain is not starved
    __builtin_amdgcn_s_setprio(3);
    const int f = blockIdx.x, tid = threadIdx.x;
    PANO_TAIL_STAMP(0);
    // taps to LDS once: each level's loop then starts on LDS reads, not on a global load
    for (int i = tid; i < ta.n_lvl * PANO_MAX_TAPS; i += kTailThreads) taps_s[i] = ta.taps[i];
    int cur = 0, keep = -1;
    int stamp = 1;
    (void)stamp;
    for (int oi = 0; oi < ta.n_oct; ++oi) {
        const int H = ta.H[oi], W = ta.W[oi];
        // planes up to 32 x 32: 2 outputs per thread item (a short serial chain per thread);
        // larger: 8 (every item fits one pass of the 512 threads at 64 x 48)
        const bool small = H <= 32 && W <= 32;
        // ---- level 0: nearest 1/2 of the previous octave's level n_lvl-3
        {
            const int sh = oi == 0 ? ta.ph : ta.H[oi - 1];
            const int sw = oi == 0 ? ta.pw : ta.W[oi - 1];
            const double ifx = 1.0 / ((double)W / sw), ify = 1.0 / ((double)H / sh);
            const int R1 = (ta.ntap[1] - 1) / 2;
            int dst = 0;
            while (dst == keep) ++dst;
            float *o0 = lv[dst];
            float *g0 = ta.full ? ta.G[oi][0] + (size_t)f * H * W : nullptr;
            for (int i = tid; i < H * W; i += kTailThreads) {
                const int y = i / W, x = i - (i / W) * W;
                const int sy = min(tail_src(y, ify), sh - 1), sx = min(tail_src(x, ifx), sw - 1);
                const float v = oi == 0 ? ta.prev[(size_t)f * sh * sw + (size_t)sy * sw + sx]
                                        : lv[keep][sy * kPP + kOff + sx];
                float *orow = o0 + y * kPP + kOff;
                orow[x] = v;
                tail_mirrors(x, W, R1, [&](int m) { orow[m] = v; });
                if (g0) g0[i] = v;
            }
            for (int r = tid; r < kRowIx; r += kTailThreads)   // rows past H + kRMax: SG overrun
                rowix[r] = kTP * reflect101(min(r - kRMax, H + kRMax - 1), H);
            cur = dst;
            keep = -1;
            lds_barrier();
            PANO_TAIL_STAMP(stamp);
            ++stamp;
        }
        for (int l = 1; l < ta.n_lvl; ++l) {
            const int n = ta.ntap[l];
            const int Rn = l + 1 < ta.n_lvl ? (ta.ntap[l + 1] - 1) / 2 : 0;   // next level's halo
            int out = 0;
            while (out == cur || out == keep) ++out;
            float *g = (ta.full || l < ta.n_lvl - 1) ? ta.G[oi][l] + (size_t)f * H * W : nullptr;
            float *d = ta.D[oi][l - 1] + (size_t)f * H * W;
            const float *tg = taps_s + l * PANO_MAX_TAPS;
            const lds_f32 *Lin = (const lds_f32 *)lv[cur];
            lds_f32 *Lout = (lds_f32 *)lv[out], *Lrowt = (lds_f32 *)rowt;
            const lds_i32 *Lrix = (const lds_i32 *)rowix;
            const lds_f32 *Ltg = (const lds_f32 *)tg;
            gbl_f32 *Gg = (gbl_f32 *)g, *Gd = (gbl_f32 *)d;
#define PANO_TAIL_LEVEL(NT)                                                                        \
    (small ? tail_level<NT, 2>(Lin, Lout, Lrowt, Lrix, H, W, Rn, Ltg, n, Gg, Gd, tid)                  \
           : tail_level<NT, 8>(Lin, Lout, Lrowt, Lrix, H, W, Rn, Ltg, n, Gg, Gd, tid))
#if PANO_TAIL_GENERIC
            tail_level<0, 1>(Lin, Lout, Lrowt, Lrix, H, W, Rn, Ltg, n, Gg, Gd, tid);
#else
            switch (n) {   // the reference's kernel sizes; others take the runtime-count path
                case 11: PANO_TAIL_LEVEL(11); break;
                case 13: PANO_TAIL_LEVEL(13); break;
                case 17: PANO_TAIL_LEVEL(17); break;
                case 21: PANO_TAIL_LEVEL(21); break;
                case 27: PANO_TAIL_LEVEL(27); break;
                default: tail_level<0, 1>(Lin, Lout, Lrowt, Lrix, H, W, Rn, Ltg, n, Gg, Gd, tid); break;
            }
#endif
#undef PANO_TAIL_LEVEL
            lds_barrier();
            PANO_TAIL_STAMP(stamp);
            ++stamp;
            cur = out;
            if (l == ta.n_lvl - 3) keep = cur;
        }
    }
}

// getGaussianKernel(ksize, sigma, CV_32F) of OpenCV 4.x = getGaussianKernelBitExact cast to
// f32 (cv2_compat.getGaussianKernelBitExact): exp(x*x * (-0.125 / s^2)) for the integer
// x = 1-n, 3-n, ... (twice the offset), sum = 2 * sum(side taps) + 1, every tap times 1 / sum,
// the centre tap 1 / sum itself.  ksize = cvRound(8 s + 1) | 1 (float images).
Taps make_taps(double sigma) {
    Taps t;
    // non-finite or too wide sigmas are refused before the int conversion (nearbyint(inf) has
    // no int value): ksize = rint(8 s + 1) | 1 must fit PANO_MAX_TAPS
    if (!(sigma >= 0.0 && sigma * 8.0 + 1.0 < (double)PANO_MAX_TAPS)) {
        t.n = -1;
        return t;
    }
    int n = (int)nearbyint(sigma * 4 * 2 + 1) | 1;
    if (n > PANO_MAX_TAPS) n = -1;
    t.n = n;
    if (n < 0) return t;
    const double scale2x = -0.125 / (sigma * sigma);
    const int n2 = (n - 1) / 2;
    double vals[PANO_MAX_TAPS];
    double s = 0.0;
    for (int i = 0, x = 1 - n; i < n2; ++i, x += 2) {
        vals[i] = exp((double)(x * x) * scale2x);
        s += vals[i];
    }
    s *= 2.0;
    s += 1.0;
    const double mul1 = 1.0 / s;
    t.k[n2] = (float)mul1;
    for (int i = 0; i < n2; ++i) {
        const double v = vals[i] * mul1;
        t.k[i] = (float)v;
        t.k[n - 1 - i] = (float)v;
    }
    return t;
}

size_t smem_bytes(const Taps &t) {
    const int r = (t.n - 1) / 2;
    // trow rows are read up to SEG past the valid extent by the column pass: pad them
    return (size_t)((TY + 2 * r) * ((TX + 2 * r) | 1) + (TY + 2 * r + SEG) * TXP) * sizeof(float);
}

template <int MODE, int NT>
int launch_blur_nt(pano_ctx *ctx, const LoadArgs &la, float *out, float *dog, float *in_copy,
                   int n, int H, int W, const Taps &t) {
    dim3 grid((W + TX - 1) / TX, (H + TY - 1) / TY, n);
    static const bool tall = [] {
        const char *e = getenv("PANO_BLUR_TALL");   // 1 (default): tall tiles; 0: 64 x 64 tiles
        return e ? atoi(e) != 0 : true;
    }();
    static const int small_tiles = [] {
        const char *e = getenv("PANO_BLUR_SMALL");   // planes with fewer 64x64 tiles use 32x32 tiles
        return e ? atoi(e) : 300;                   // measured: octave 3 of parrington gains, 1-2 do not
    }();
    if constexpr (NT > 0) {
        constexpr int R = (NT - 1) / 2;
        if ((long)grid.x * grid.y * n < small_tiles) {
            const size_t sm = (size_t)(32 + 2 * R) * ((32 + 2 * R) | 1) * sizeof(float);
            dim3 g((W + 31) / 32, (H + 31) / 32, n);
            {
                PanoProf prof_(ctx, PK_BLUR);
                blur_fast<MODE, NT, 32, 32, 256><<<g, 256, sm, ctx->stream>>>(la, out, dog, in_copy, H, W, t);
            }
            PANO_LAUNCH_CHECK(ctx, "blur_fast");
            return PANO_OK;
        }
        // the base (MODE_BASE) also holds its gray patch in LDS: PANO_BASE_ROWS output rows per
        // tile (default: the levels' tall tile) -- 88 fits tile + patch in 40 KB, 4 workgroups per CU
        constexpr int TYT = MODE == MODE_BASE && PANO_BASE_ROWS > 0 ? PANO_BASE_ROWS : tall_rows(NT);
        // tall tiles only where they still leave >= 6 workgroups per CU (octave 0 of a batch):
        // on smaller planes the lost parallelism costs more than the halo saves
        static const long tall_min = [] {
            const char *e = getenv("PANO_BLUR_TALL_MIN");   // fewest tall-tile workgroups
            return e ? atol(e) : 1536L;
        }();
        const bool use_tall = tall && (long)grid.x * ((H + TYT - 1) / TYT) * n >= tall_min;
        const int ty = use_tall ? TYT : TY;
        // base: the patch rows its window needs ((ty + 2R) / 2 + 3), not the capacity
        const size_t sm = (size_t)((ty + 2 * R) * ((TX + 2 * R) | 1) +
                                   (MODE == MODE_BASE ? ((ty + 2 * R) / 2 + 3) * kPatchP : 0)) * sizeof(float);
        {
            PanoProf prof_(ctx, PK_BLUR);
            if (use_tall) {
                grid.y = (H + TYT - 1) / TYT;
                blur_fast<MODE, NT, TYT><<<grid, 512, sm, ctx->stream>>>(la, out, dog, in_copy, H, W, t);
            } else {
                blur_fast<MODE, NT, TY><<<grid, 512, sm, ctx->stream>>>(la, out, dog, in_copy, H, W, t);
            }
        }
        PANO_LAUNCH_CHECK(ctx, "blur_fast");
    } else {
        const size_t sm = smem_bytes(t);
        if (sm > 65536)
            PANO_HIP(ctx, hipFuncSetAttribute((const void *)blur_level<MODE, 0>,
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm));
        {
            PanoProf prof_(ctx, PK_BLUR);
            blur_level<MODE, 0><<<grid, 256, sm, ctx->stream>>>(la, out, dog, in_copy, H, W, t);
        }
        PANO_LAUNCH_CHECK(ctx, "blur_level");
    }
    return PANO_OK;
}

template <int MODE>
int launch_blur(pano_ctx *ctx, const LoadArgs &la, float *out, float *dog, float *in_copy, int n,
                int H, int W, const Taps &t) {
    switch (t.n) {   // the reference's kernel sizes: 11 (base), 11/13/17/21/27 (levels)
        case 11: return launch_blur_nt<MODE, 11>(ctx, la, out, dog, in_copy, n, H, W, t);
        case 13: return launch_blur_nt<MODE, 13>(ctx, la, out, dog, in_copy, n, H, W, t);
        case 17: return launch_blur_nt<MODE, 17>(ctx, la, out, dog, in_copy, n, H, W, t);
        case 21: return launch_blur_nt<MODE, 21>(ctx, la, out, dog, in_copy, n, H, W, t);
        case 27: return launch_blur_nt<MODE, 27>(ctx, la, out, dog, in_copy, n, H, W, t);
        default: return launch_blur_nt<MODE, 0>(ctx, la, out, dog, in_copy, n, H, W, t);
    }
}

// Fused pair (levels l, l + 1) of one octave; PANO_E_UNSUPPORTED for tap pairs without an
// instantiation (the caller then launches the levels one by one).
template <int MODE, int NT1, int NT2, int TT, int NTHR>
int launch_pair_tt(pano_ctx *ctx, const LoadArgs &la, float *out1, float *dog1, float *in_copy, float *out2,
                   float *dog2, int n, int H, int W, const Taps &t1, const Taps &t2) {
    const size_t sm = (size_t)PairShape<NT1, NT2, TT>::floats * sizeof(float);
    static bool attr = false;
    if (!attr) {
        PANO_HIP(ctx, hipFuncSetAttribute((const void *)blur_pair<MODE, NT1, NT2, TT, NTHR>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm));
        attr = true;
    }
    dim3 grid((W + TT - 1) / TT, (H + TT - 1) / TT, n);
    {
        PanoProf prof_(ctx, PK_BLUR);
        blur_pair<MODE, NT1, NT2, TT, NTHR><<<grid, NTHR, sm, ctx->stream>>>(la, out1, dog1, in_copy, out2, dog2,
                                                                           H, W, t1, t2);
    }
    PANO_LAUNCH_CHECK(ctx, "blur_pair");
    return PANO_OK;
}

// 32 x 32 tiles of 256 threads (default), or 64 x 64 of 512 (PANO_BLUR_PAIR_TT=64: less
// halo recompute, fewer workgroups)
template <int MODE, int NT1, int NT2>
int launch_pair_nt(pano_ctx *ctx, const LoadArgs &la, float *out1, float *dog1, float *in_copy, float *out2,
                   float *dog2, int n, int H, int W, const Taps &t1, const Taps &t2) {
    static const int tt = [] {
        const char *e = getenv("PANO_BLUR_PAIR_TT");
        return e && atoi(e) == 64 ? 64 : 32;
    }();
    if (tt == 64 && H >= 64 && W >= 64)
        return launch_pair_tt<MODE, NT1, NT2, 64, 512>(ctx, la, out1, dog1, in_copy, out2, dog2, n, H, W, t1, t2);
    return launch_pair_tt<MODE, NT1, NT2, 32, 256>(ctx, la, out1, dog1, in_copy, out2, dog2, n, H, W, t1, t2);
}

template <int MODE>
int launch_pair(pano_ctx *ctx, const LoadArgs &la, float *out1, float *dog1, float *in_copy, float *out2,
                float *dog2, int n, int H, int W, const Taps &t1, const Taps &t2) {
    if (t1.n == 11 && t2.n == 13)
        return launch_pair_nt<MODE, 11, 13>(ctx, la, out1, dog1, in_copy, out2, dog2, n, H, W, t1, t2);
    if constexpr (MODE == MODE_LEVEL) {
        if (t1.n == 21 && t2.n == 27)
            return launch_pair_nt<MODE, 21, 27>(ctx, la, out1, dog1, in_copy, out2, dog2, n, H, W, t1, t2);
        if (t1.n == 17 && t2.n == 21)
            return launch_pair_nt<MODE, 17, 21>(ctx, la, out1, dog1, in_copy, out2, dog2, n, H, W, t1, t2);
    }
    return PANO_E_UNSUPPORTED;
}

}  // namespace

// Scalars of S1/S2 exactly as the reference computes them (Python/numpy doubles; glibc
// pow/sqrt/exp are what both use).  Exposed for the CPU tests via pano_sift_plan.
int sift_plan(const pano_sift_params *p, int h, int w, int *n_oct, int *n_lvl, double *sig_base,
              double *sig_lvl) {
    const int ni = p->num_intervals;
    if (ni < 1 || ni + 3 > PANO_MAX_LEVELS) return PANO_E_UNSUPPORTED;
    const double d = p->sigma * p->sigma - (2 * p->assumed_blur) * (2 * p->assumed_blur);
    *sig_base = sqrt(d > 0.01 ? d : 0.01);
    const int bh = 2 * h, bw = 2 * w;
    const int mn = bh < bw ? bh : bw;
    int no = (int)nearbyint(log((double)mn) / log(2.0) - 1);
    if (no > PANO_MAX_OCTAVES) no = PANO_MAX_OCTAVES;
    if (no < 1) no = 1;
    *n_oct = no;
    *n_lvl = ni + 3;
    const double k = pow(2.0, 1.0 / ni);
    sig_lvl[0] = p->sigma;
    for (int i = 1; i < ni + 3; ++i) {
        const double prev = pow(k, (double)(i - 1)) * p->sigma;
        const double tot = k * prev;
        sig_lvl[i] = sqrt(tot * tot - prev * prev);
    }
    return PANO_OK;
}

extern "C" int pano_sift_taps(double sigma, double *out, int *n) {
    Taps t = make_taps(sigma);
    if (t.n < 0) return PANO_E_UNSUPPORTED;
    for (int i = 0; i < t.n; ++i) out[i] = t.k[i];
    *n = t.n;
    return PANO_OK;
}

// Lay out the pyramid of n frames whose octave 0 is H0 x W0 (the 2x base), at most max_oct
// octaves (fewer when a plane would shrink below 1 px), nl Gaussian levels per octave.
int sift_reserve_dims(pano_ctx *ctx, int n, int H0, int W0, int max_oct, int nl) {
    size_t goff = 0, doff = 0;
    int oh = H0, ow = W0, no = std::min(std::max(max_oct, 1), PANO_MAX_OCTAVES);
    for (int o = 0; o < no; ++o) {
        ctx->oct_h[o] = oh;
        ctx->oct_w[o] = ow;
        const size_t plane = (size_t)n * oh * ow;
        for (int l = 0; l < nl; ++l) {
            ctx->gauss_off[o][l] = goff;
            goff += (plane + 63) & ~size_t(63);
        }
        for (int l = 0; l < nl - 1; ++l) {
            ctx->dog_off[o][l] = doff;
            doff += (plane + 63) & ~size_t(63);
        }
        oh /= 2;
        ow /= 2;
        if (oh < 1 || ow < 1) { no = o + 1; break; }
    }
    ctx->n_oct = no;
    ctx->n_lvl = nl;
    const size_t need = (goff + doff) * sizeof(float);
    if (need > ctx->pyr_bytes) {
        const int rc = pano_grow(ctx, (void **)&ctx->pyr, &ctx->pyr_bytes, need);
        if (rc) return rc;
    }
    ctx->dog = ctx->pyr + goff;
    ctx->n = n;
    ctx->h = (H0 + 1) / 2;
    ctx->w = (W0 + 1) / 2;
    return PANO_OK;
}

int sift_reserve_pyramid(pano_ctx *ctx, int n, int h, int w, const pano_sift_params *p) {
    int no, nl;
    double sb, sl[PANO_MAX_LEVELS];
    int rc = sift_plan(p, h, w, &no, &nl, &sb, sl);
    if (rc) return pano_fail(ctx, rc, "unsupported SIFT parameters");
    return sift_reserve_dims(ctx, n, 2 * h, 2 * w, no, nl);
}

// The pyramid from one of three sources (PyrSource): BGR u8 frames (gray + x2 + base blur:
// compute_keypoints_and_descriptors), f32 gray frames (generate_base_image on a caller's
// image) or a caller's f32 base (generate_gaussian_images on any base: copied to level 0 of
// octave 0).  n frames; h x w is the gray size, H0 x W0 = 2h x 2w the base size (base source:
// the caller's base size, octave count capped at max_oct).
int launch_sift_pyramid_src(pano_ctx *ctx, const PyrSource &src, int n, int h, int w,
                            const pano_sift_params *p, bool defer_tail, bool full) {
    ctx->kp_zeroed = false;
    sift_join_tail(ctx);                  // a previous call's tail must finish first
    sift_join_x(ctx);
    ctx->early_oct = -1;
    int no, nl;
    double sb, sl[PANO_MAX_LEVELS];
    const int gh = src.base ? std::max(1, h / 2) : h, gw = src.base ? std::max(1, w / 2) : w;
    int rc = sift_plan(p, gh, gw, &no, &nl, &sb, sl);
    if (rc) return pano_fail(ctx, rc, "unsupported SIFT parameters");
    if (src.base && src.sig) {
        // generate_gaussian_images(base, n, kernels) with the caller's list (sift_impl.py:82-97:
        // level l = GaussianBlur(level l - 1, kernels[l]); the next octave from level -3)
        if (src.n_sig < 3 || src.n_sig > PANO_MAX_LEVELS)
            return pano_fail(ctx, PANO_E_UNSUPPORTED, "gaussian kernel list: 3 to PANO_MAX_LEVELS entries");
        nl = src.n_sig;
        for (int l = 0; l < nl; ++l) sl[l] = src.sig[l];
    }
    rc = src.base ? sift_reserve_dims(ctx, n, h, w, src.max_oct, nl) : sift_reserve_pyramid(ctx, n, h, w, p);
    if (rc) return rc;
    no = ctx->n_oct;
    Taps tb = make_taps(sb);
    Taps tl[PANO_MAX_LEVELS];
    for (int l = 1; l < nl; ++l) tl[l] = make_taps(sl[l]);
    if (tb.n < 0) return pano_fail(ctx, PANO_E_UNSUPPORTED, "Gaussian kernel too wide");
    for (int l = 1; l < nl; ++l)
        if (tl[l].n < 0) return pano_fail(ctx, PANO_E_UNSUPPORTED, "Gaussian kernel too wide");
    float *G = ctx->pyr, *D = ctx->dog;
    // fused level chains (blur_chain, PANO_BLUR_CHAIN=1) for the octaves whose planes hold the
    // (3, 4, 5) chain's halo, with the reference's tap counts.  Measured on MI355X:
    // bit-exact, ~40 % less HBM traffic, but 1.6x slower than the level-by-level launches at
    // octave 0 (the halo recompute and the two resident workgroups per CU leave the VALU ~30 %
    // busy), so off by default.  Read per call so tests can compare both forms.
    const char *chain_env = getenv("PANO_BLUR_CHAIN");
    const bool chain_on = chain_env && atoi(chain_env) != 0;
    const bool chain_taps = chain_on && nl == 6 && tl[1].n == 11 && tl[2].n == 13 && tl[3].n == 17 &&
                            tl[4].n == 21 && tl[5].n == 27;
    // PANO_BLUR_CHAIN=k (k >= 1): chains from octave k - 1 on (1: every octave)
    const int chain_min_oct = chain_on ? atoi(chain_env) - 1 : 0;
    auto chain_ok = [&](int o) {
        return chain_taps && o >= chain_min_oct && ctx->oct_h[o] >= 64 && ctx->oct_w[o] >= 64;
    };
    const bool chain_base = src.bgr && !src.base_only && chain_ok(0) && tb.n == 11;
    // A/B (PANO_BASE_PAIR=1, read per call): the base level and level 1 of octave 0 in one
    // blur_chain launch (G0 on the tile plus level 1's halo in LDS, never written unless the full
    // pyramid is asked): one launch and G0's HBM round trip fewer, the base's FMAs on the halo.
    // Measured (profiles/r06_base_pair_ab.txt): bit-exact, blur class +1 %, pooled step +2 %: off
    const char *bp_env = getenv("PANO_BASE_PAIR");
    const bool base_pair = bp_env && atoi(bp_env) != 0 && !chain_on && src.bgr && !src.base_only && nl >= 3 &&
                           tb.n == 11 && tl[1].n == 11 && ctx->oct_h[0] >= 64 && ctx->oct_w[0] >= 64;
    // streaming cascades (blur_cascade, PANO_BLUR_CASCADE=1): per octave walker A (octave 0 from
    // the gray frames: base, 1, 2; else levels 1, 2) and walker B (levels 3, 4, 5 from G2)
    const char *cas_env = getenv("PANO_BLUR_CASCADE");     // read per call: tests compare both forms
    const int cas_on = cas_env ? atoi(cas_env) : 0;
    static const int cas_bh = [] {
        const char *e = getenv("PANO_CAS_BH");   // band rows per workgroup
        return e ? std::max(8, atoi(e)) : 256;
    }();
    // the cascade compiles in the reference's default taps (cas_taps.h): only when they are the
    // run-time ones, bit for bit
    bool cas_taps = cas_on && !chain_on && nl == kCasDefLevels && tb.n == kCasDefTaps[0] &&
                    memcmp(tb.k, kCasDefK[0], sizeof(float) * tb.n) == 0;
    for (int l = 1; cas_taps && l < nl; ++l)
        cas_taps = tl[l].n == kCasDefTaps[l] && memcmp(tl[l].k, kCasDefK[l], sizeof(float) * tl[l].n) == 0;
    auto cas_ok = [&](int o) { return cas_taps && ctx->oct_h[o] >= 64 && ctx->oct_w[o] >= kCasSW; };
    const bool cas_base = src.bgr && !src.base_only && cas_ok(0);
    // pano_sift(_u8) runs the keypoint stage next: its counters are zeroed by gray_frames
    int32_t *zp = nullptr;
    size_t zn = 0;
    if (ctx->early_armed && src.bgr && !src.base_only) {
        rc = sift_kp_counters(ctx, &zp, &zn);
        if (rc) return rc;
    }
    if (src.base) {
        // generate_gaussian_images(base, ...): the caller's base is level 0 of octave 0
        PANO_HIP(ctx, hipMemcpyAsync(G + ctx->gauss_off[0][0], src.base,
                                     (size_t)n * ctx->oct_h[0] * ctx->oct_w[0] * sizeof(float),
                                     hipMemcpyDeviceToDevice, ctx->stream));
    } else if (src.grayf) {
        LoadArgs la{};
        la.grayf = src.grayf;
        la.sh = h;
        la.sw = w;
        rc = launch_blur<MODE_BASEF>(ctx, la, G + ctx->gauss_off[0][0], nullptr, nullptr, n,
                                     ctx->oct_h[0], ctx->oct_w[0], tb);
        if (rc) return rc;
    } else if (chain_base || cas_base || base_pair) {
        // gray frames only: the base level is the first level of octave 0's first chain
        const size_t npx = (size_t)n * h * w;
        rc = pano_grow(ctx, (void **)&ctx->gray, &ctx->gray_bytes, npx + 16);
        if (rc) return rc;
        const unsigned blocks = (unsigned)((npx + 1023) / 1024);
        {
            PanoProf prof_(ctx, PK_BLUR);
            gray_frames<<<blocks, 256, 0, ctx->stream>>>(src.bgr, ctx->gray, npx, zp, (int)zn);
        }
        PANO_LAUNCH_CHECK(ctx, "gray_frames");
        ctx->kp_zeroed = zp != nullptr;
    } else {
        // gray frames (u8) for the base image
        const size_t npx = (size_t)n * h * w;
        rc = pano_grow(ctx, (void **)&ctx->gray, &ctx->gray_bytes, npx + 16);
        if (rc) return rc;
        const unsigned blocks = (unsigned)((npx + 1023) / 1024);
        {
            PanoProf prof_(ctx, PK_BLUR);
            gray_frames<<<blocks, 256, 0, ctx->stream>>>(src.bgr, ctx->gray, npx, zp, (int)zn);
        }
        PANO_LAUNCH_CHECK(ctx, "gray_frames");
        ctx->kp_zeroed = zp != nullptr;
        LoadArgs la{};
        la.gray = ctx->gray;
        la.sh = h;
        la.sw = w;
        rc = launch_blur<MODE_BASE>(ctx, la, G + ctx->gauss_off[0][0], nullptr, nullptr, n,
                                    ctx->oct_h[0], ctx->oct_w[0], tb);
        if (rc) return rc;
    }
    if (src.base_only) {
        ctx->pyr_full = false;
        return PANO_OK;
    }
    // first octave of the fused small-octave tail (every level fits one 64 x 64 tile)
    int o_tail = no;
    for (int o = 1; o < no; ++o)
        if (ctx->oct_h[o] <= kTailDim && ctx->oct_w[o] <= kTailDim) { o_tail = o; break; }
    if (no - o_tail > kTailOct) o_tail = no - kTailOct;
    // The small octaves run on a high-priority side stream, beside the main stream's last
    // large-octave levels and extrema scan: the last o_tail - o_side blur_fast octaves (their
    // launches are one workgroup's latency each) and then the fused tail (octaves <= 64 x 64,
    // blur_tail).  The fork comes as soon as the side's first input exists (G[o_side-1][nl-3]);
    // keypoints split the extrema scan at o_side and join before the second part.
    static const int side_oct = [] {
        const char *e = getenv("PANO_SIDE_OCT");   // measured: 0 beats 1 and 2 (co-run contention)
        return e ? atoi(e) : 0;
    }();
    const int o_side = o_tail < no ? std::max(1, o_tail - std::max(0, side_oct)) : no;
    hipStream_t main_stream = ctx->stream;
    // PANO_TAIL_MAIN=1 (read per call): the tail on the main stream, no fork in the launch
    // sequence (a captured graph is then one chain)
    const char *tail_main_env = getenv("PANO_TAIL_MAIN");
    const bool tail_main = (tail_main_env && atoi(tail_main_env) != 0) || (ctx->flags_opt & PANO_CTX_TAIL_MAIN);
    auto fork = [&]() -> int {
        if (tail_main) return PANO_OK;
        if (!ctx->side) {
            int lo_prio = 0, hi_prio = 0;   // numerically lower = higher priority
            PANO_HIP(ctx, hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio));
            // Default priority.  Measured (tools/jpeg_run_check.py, same box): with the side
            // stream at high priority, graphs captured after the first one in a process replayed
            // at 1.42 ms per parrington stitch instead of 1.05 (every few main-chain kernels
            // waiting ~35 us); at default priority every capture replays at 1.05-1.06 ms.
            // PANO_SIDE_PRIO=1: high priority (A/B only).
            const char *pe = getenv("PANO_SIDE_PRIO");
            const bool hi = pe && atoi(pe) == 1;
            if (hi) PANO_HIP(ctx, hipStreamCreateWithPriority(&ctx->side, hipStreamNonBlocking, hi_prio));
            else PANO_HIP(ctx, hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking));
            PANO_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
            PANO_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming));
        }
        PANO_HIP(ctx, hipEventRecord(ctx->ev_fork, main_stream));
        PANO_HIP(ctx, hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
        return PANO_OK;
    };
    auto launch_tail = [&]() -> int {
        TailArgs ta{};
        for (int l = 1; l < nl; ++l) ta.ntap[l] = tl[l].n;
        ta.taps = ctx->taps;
        ta.prev = G + ctx->gauss_off[o_tail - 1][nl - 3];
        ta.ph = ctx->oct_h[o_tail - 1];
        ta.pw = ctx->oct_w[o_tail - 1];
        ta.n_oct = no - o_tail;
        ta.n_lvl = nl;
        ta.full = full ? 1 : 0;
        for (int oi = 0; oi < ta.n_oct; ++oi) {
            const int o = o_tail + oi;
            ta.H[oi] = ctx->oct_h[o];
            ta.W[oi] = ctx->oct_w[o];
            for (int l = 0; l < nl; ++l) ta.G[oi][l] = G + ctx->gauss_off[o][l];
            for (int l = 0; l + 1 < nl; ++l) ta.D[oi][l] = D + ctx->dog_off[o][l];
        }
        hipStream_t ts = tail_main ? main_stream : ctx->side;
        {
            PanoProf prof_(ctx, PK_BLUR, ts);
            blur_tail<<<n, kTailThreads, 0, ts>>>(ta);
        }
        PANO_LAUNCH_CHECK(ctx, "blur_tail");
        if (tail_main) return PANO_OK;
        PANO_HIP(ctx, hipEventRecord(ctx->ev_join, ctx->side));
        ctx->tail_pending = true;
        ctx->o_tail = o_side;
        return PANO_OK;
    };
    // device copy of the taps, [level][PANO_MAX_TAPS] with row 0 the base's (the tail and the
    // chains read them); uploaded only when they change, so never inside a graph capture after
    // the eager first call
    {
        float th[PANO_MAX_LEVELS * PANO_MAX_TAPS] = {};
        for (int t = 0; t < tb.n; ++t) th[t] = tb.k[t];
        for (int l = 1; l < nl; ++l)
            for (int t = 0; t < tl[l].n; ++t) th[l * PANO_MAX_TAPS + t] = tl[l].k[t];
        if (!ctx->taps) {
            PANO_HIP(ctx, hipMalloc((void **)&ctx->taps, sizeof(th)));
            ctx->taps_valid = false;
        }
        if (!ctx->taps_valid || memcmp(th, ctx->taps_host, sizeof(th)) != 0) {
            if (ctx->capturing) return pano_fail(ctx, PANO_E_UNSUPPORTED, "tap upload inside a graph capture");
            memcpy(ctx->taps_host, th, sizeof(th));
            PANO_HIP(ctx, hipMemcpy(ctx->taps, ctx->taps_host, sizeof(th), hipMemcpyHostToDevice));
            ctx->taps_valid = true;
        }
    }
    // fused level pairs (blur_pair, PANO_BLUR_PAIR) on the latency-bound octaves: (1, 2) and
    // (4, 5) of every octave o >= 1 whose plane has fewer than PANO_BLUR_PAIR_TILES 64 x 64
    // tiles per batch; level 3 alone keeps the next octave's (and the tail's) start after it
    static const long pair_tiles = [] {
        const char *e = getenv("PANO_BLUR_PAIR_TILES");
        return e ? atol(e) : 4000L;
    }();
    static const int pair_mask = [] {
        // bit 0: levels (1, 2); bit 1: (4, 5).  Measured on MI355X: (1, 2) within
        // noise of the level-by-level launches at parrington and 1080p, (4, 5) slower (level
        // 4's 21 taps over the 27-tap halo region: 3.3x its FMAs), so off by default
        const char *e = getenv("PANO_BLUR_PAIR");
        return e ? atoi(e) : 0;
    }();
    // Levels nl-2 and nl-1 of octave o (4 and 5 by default) on a second side stream, beside
    // octave o+1's first levels, which read only level nl-3 of octave o: the octaves' chains
    // of small latency-bound launches then overlap instead of running back to back.  From
    // octave PANO_OCT_FORK on (-1: off); joined into the main stream after the octave loop.
    // Measured on MI355X: bit-exact; at default stream priority within noise of
    // the unforked chain (1.067-1.075 against 1.05-1.07 ms per parrington stitch), so off.
    static const int oct_fork = [] {
        const char *e = getenv("PANO_OCT_FORK");
        return e ? atoi(e) : -1;
    }();
    bool lvl_forked = false;
    for (int o = 0; o < o_tail; ++o) {
        const int H = ctx->oct_h[o], W = ctx->oct_w[o];
        ctx->stream = o >= o_side && !tail_main ? ctx->side : main_stream;     // side-stream octaves
        const bool fork_lvl = oct_fork >= 0 && o >= oct_fork && o < o_side && nl >= 4 && !chain_ok(o) && !cas_ok(o);
        if (cas_ok(o)) {
            auto Gp = [&](int l) { return G + ctx->gauss_off[o][l]; };
            auto Dp = [&](int l) { return D + ctx->dog_off[o][l]; };
            const int bh = std::min(H, cas_bh);
            LoadArgs la{};
            CasOut ca{};
            if (o == 0 && cas_base) {
                la.gray = ctx->gray;
                la.sh = h;
                la.sw = w;
                ca.g[0] = full ? Gp(0) : nullptr;
                ca.g[1] = Gp(1); ca.d[1] = Dp(0);
                ca.g[2] = Gp(2); ca.d[2] = Dp(1);
                rc = launch_cascade<MODE_BASE, 3, 0>(ctx, la, ca, n, H, W, bh);
            } else {
                ca.g[0] = Gp(1); ca.d[0] = Dp(0);
                ca.g[1] = Gp(2); ca.d[1] = Dp(1);
                if (o == 0) {
                    la.src = Gp(0);
                    rc = launch_cascade<MODE_LEVEL, 2, 1>(ctx, la, ca, n, H, W, bh);
                } else {
                    la.src = G + ctx->gauss_off[o - 1][nl - 3];
                    la.sh = ctx->oct_h[o - 1];
                    la.sw = ctx->oct_w[o - 1];
                    la.ifx = 1.0 / ((double)W / la.sw);
                    la.ify = 1.0 / ((double)H / la.sh);
                    ca.gin = full ? Gp(0) : nullptr;
                    rc = launch_cascade<MODE_DOWN, 2, 1>(ctx, la, ca, n, H, W, bh);
                }
            }
            if (rc) { ctx->stream = main_stream; return rc; }
            LoadArgs lb{};
            lb.src = Gp(2);
            CasOut cb{};
            cb.g[0] = Gp(3); cb.d[0] = Dp(2);
            cb.g[1] = full ? Gp(4) : nullptr; cb.d[1] = Dp(3);
            cb.g[2] = full ? Gp(5) : nullptr; cb.d[2] = Dp(4);
            rc = launch_cascade<MODE_LEVEL, 3, 3>(ctx, lb, cb, n, H, W, bh);
            if (rc) { ctx->stream = main_stream; return rc; }
            if (o == o_side - 1 && o_tail < no) {
                rc = fork();
                if (rc) { ctx->stream = main_stream; return rc; }
            }
            continue;
        }
        if (chain_ok(o)) {
            // chain A: levels 1-2 (octave 0 from gray: base, 1, 2); chain B: levels 3-5 from G2.
            // Written: G1-G3 and DoG 0-4 (every level in a full pyramid)
            auto Gp = [&](int l) { return G + ctx->gauss_off[o][l]; };
            auto Dp = [&](int l) { return D + ctx->dog_off[o][l]; };
            LoadArgs la{};
            ChainOut ca{};
            if (o == 0 && chain_base) {
                la.gray = ctx->gray;
                la.sh = h;
                la.sw = w;
                ca.g[0] = full ? Gp(0) : nullptr;
                ca.g[1] = Gp(1); ca.d[1] = Dp(0);
                ca.g[2] = Gp(2); ca.d[2] = Dp(1);
                rc = launch_chain<MODE_BASE, 11, 11, 13>(ctx, la, ca, n, H, W, 0);
            } else if (o == 0) {
                la.src = Gp(0);
                ca.g[0] = Gp(1); ca.d[0] = Dp(0);
                ca.g[1] = Gp(2); ca.d[1] = Dp(1);
                rc = launch_chain<MODE_LEVEL, 11, 13, 0>(ctx, la, ca, n, H, W, 1);
            } else {
                la.src = G + ctx->gauss_off[o - 1][nl - 3];
                la.sh = ctx->oct_h[o - 1];
                la.sw = ctx->oct_w[o - 1];
                la.ifx = 1.0 / ((double)W / la.sw);
                la.ify = 1.0 / ((double)H / la.sh);
                ca.gin = full ? Gp(0) : nullptr;
                ca.g[0] = Gp(1); ca.d[0] = Dp(0);
                ca.g[1] = Gp(2); ca.d[1] = Dp(1);
                rc = launch_chain<MODE_DOWN, 11, 13, 0>(ctx, la, ca, n, H, W, 1);
            }
            if (rc) { ctx->stream = main_stream; return rc; }
            LoadArgs lb{};
            lb.src = Gp(2);
            ChainOut cb{};
            cb.g[0] = Gp(3); cb.d[0] = Dp(2);
            cb.g[1] = full ? Gp(4) : nullptr; cb.d[1] = Dp(3);
            cb.g[2] = full ? Gp(5) : nullptr; cb.d[2] = Dp(4);
            rc = launch_chain<MODE_LEVEL, 17, 21, 27>(ctx, lb, cb, n, H, W, 3);
            if (rc) { ctx->stream = main_stream; return rc; }
            if (o == o_side - 1 && o_tail < no) {
                rc = fork();
                if (rc) { ctx->stream = main_stream; return rc; }
            }
            continue;
        }
        static const bool pair_o0 = [] {      // A/B: fused pairs on octave 0 too
            const char *e = getenv("PANO_BLUR_PAIR_O0");
            return e && atoi(e) != 0;
        }();
        const bool pairs_here = (o >= 1 || pair_o0) && nl == 6 && H >= 32 && W >= 32 &&
                                (long)((W + 63) / 64) * ((H + 63) / 64) * n < pair_tiles;
        int l_first = 1;
        if (o == 0 && base_pair) {
            LoadArgs la{};
            la.gray = ctx->gray;
            la.sh = h;
            la.sw = w;
            ChainOut ca{};
            ca.g[0] = full ? G + ctx->gauss_off[0][0] : nullptr;
            ca.g[1] = (full || 1 < nl - 1) ? G + ctx->gauss_off[0][1] : nullptr;
            ca.d[1] = D + ctx->dog_off[0][0];
            rc = launch_chain<MODE_BASE, 11, 11, 0>(ctx, la, ca, n, H, W, 0);
            if (rc) { ctx->stream = main_stream; return rc; }
            l_first = 2;
        }
        for (int l = l_first; l < nl; ++l) {
            if (fork_lvl && l == nl - 2) {
                if (!ctx->lvl_side) {
                    int lo_prio = 0, hi_prio = 0;
                    PANO_HIP(ctx, hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio));
                    (void)lo_prio;
                    PANO_HIP(ctx, hipStreamCreateWithFlags(&ctx->lvl_side, hipStreamNonBlocking));
                    PANO_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_lvl_join, hipEventDisableTiming));
                }
                if (!ctx->ev_lvl[o]) PANO_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_lvl[o], hipEventDisableTiming));
                PANO_HIP(ctx, hipEventRecord(ctx->ev_lvl[o], main_stream));
                PANO_HIP(ctx, hipStreamWaitEvent(ctx->lvl_side, ctx->ev_lvl[o], 0));
                ctx->stream = ctx->lvl_side;
                lvl_forked = true;
            }
            float *out = G + ctx->gauss_off[o][l];
            float *dg = D + ctx->dog_off[o][l - 1];
            LoadArgs la{};
            const bool pair = pairs_here && ((l == 1 && (pair_mask & 1)) || (l == 4 && (pair_mask & 2)));
            if (pair) {
                float *out2 = G + ctx->gauss_off[o][l + 1];
                float *dg2 = D + ctx->dog_off[o][l];
                const bool keep1 = full || l + 1 < nl - 1 || l < nl - 2;   // G[l] read downstream
                const bool keep2 = full || l + 1 < nl - 1;
                if (l == 1 && o > 0) {
                    la.src = G + ctx->gauss_off[o - 1][nl - 3];
                    la.sh = ctx->oct_h[o - 1];
                    la.sw = ctx->oct_w[o - 1];
                    la.ifx = 1.0 / ((double)W / la.sw);
                    la.ify = 1.0 / ((double)H / la.sh);
                    rc = launch_pair<MODE_DOWN>(ctx, la, keep1 ? out : nullptr, dg,
                                                full ? G + ctx->gauss_off[o][0] : nullptr, keep2 ? out2 : nullptr,
                                                dg2, n, H, W, tl[l], tl[l + 1]);
                } else {
                    la.src = G + ctx->gauss_off[o][l - 1];
                    rc = launch_pair<MODE_LEVEL>(ctx, la, (full || l < nl - 2) ? out : nullptr, dg, nullptr,
                                                 keep2 ? out2 : nullptr, dg2, n, H, W, tl[l], tl[l + 1]);
                }
                if (rc == PANO_OK) {
                    ++l;                                   // level l + 1 done too
                    continue;
                }
                if (rc != PANO_E_UNSUPPORTED) { ctx->stream = main_stream; return rc; }
                la = LoadArgs{};                           // no fused form: level by level
            }
            if (l == 1 && o > 0) {
                // next-octave base = INTER_NEAREST (w//2, h//2) of level nl-3 of octave o-1,
                // materialised as G[o][0] by the same launch
                la.src = G + ctx->gauss_off[o - 1][nl - 3];
                la.sh = ctx->oct_h[o - 1];
                la.sw = ctx->oct_w[o - 1];
                la.ifx = 1.0 / ((double)W / la.sw);
                la.ify = 1.0 / ((double)H / la.sh);
                rc = launch_blur<MODE_DOWN>(ctx, la, (full || l < nl - 1) ? out : nullptr, dg,
                                            full ? G + ctx->gauss_off[o][0] : nullptr, n, H, W, tl[l]);
            } else {
                la.src = G + ctx->gauss_off[o][l - 1];
                rc = launch_blur<MODE_LEVEL>(ctx, la, (full || l < nl - 1) ? out : nullptr, dg, nullptr,
                                             n, H, W, tl[l]);
            }
            if (rc) { ctx->stream = main_stream; return rc; }
            if (o == o_side - 1 && l == nl - 3 && o_tail < no) {
                rc = fork();
                if (rc) { ctx->stream = main_stream; return rc; }
            }
        }
        // this octave's DoG levels are complete on the main stream: its extrema scan may start
        // beside the next octaves' (latency-bound) blur launches
        if (ctx->early_armed && !full && !fork_lvl && o < o_side) {
            rc = sift_early_extrema(ctx, p, o);
            if (rc) { ctx->stream = main_stream; return rc; }
        }
    }
    ctx->stream = main_stream;
    if (lvl_forked) {
        PANO_HIP(ctx, hipEventRecord(ctx->ev_lvl_join, ctx->lvl_side));
        PANO_HIP(ctx, hipStreamWaitEvent(main_stream, ctx->ev_lvl_join, 0));
    }
    if (o_tail < no) {
        rc = launch_tail();
        if (rc) return rc;
        static const bool tail_solo = getenv("PANO_TAIL_SOLO") != nullptr;   // diagnostics
        if (tail_solo) sift_join_tail(ctx);
    }
    if (o_tail < no && !defer_tail) sift_join_tail(ctx);
    ctx->pyr_full = full;
    return PANO_OK;
}

#if PANO_CAS_TIMING
// diagnostics build only (not in pano.h): the stamps of the last blur_cascade launch
extern "C" int pano_dbg_cas_clock(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_cas_clock), sizeof(g_cas_clock)) == hipSuccess ? 0 : -1;
}
#endif

#if PANO_TAIL_TIMING
// diagnostics build only (not in pano.h): the stamps of the last blur_tail, after a sync
extern "C" int pano_dbg_tail_clock(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tail_clock), sizeof(g_tail_clock)) == hipSuccess ? 0 : -1;
}
#endif

int launch_sift_pyramid(pano_ctx *ctx, const uint8_t *bgr, int n, int h, int w,
                        const pano_sift_params *p, bool defer_tail, bool full) {
    PyrSource src{};
    src.bgr = bgr;
    return launch_sift_pyramid_src(ctx, src, n, h, w, p, defer_tail, full);
}

// ------------------------------------------------------------------ stage access
// generate_DoG_images (sift_impl.py:100-111) over the resident Gaussian levels: DoG[o][l] =
// G[o][l+1] - G[o][l] in f32, every octave and level of the batch.
__global__ void __launch_bounds__(256)
dog_from_levels(const float *__restrict__ g0, const float *__restrict__ g1, float *__restrict__ d, size_t npx) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < npx; i += (size_t)gridDim.x * 256)
        d[i] = g1[i] - g0[i];
}

int launch_sift_dog(pano_ctx *ctx) {
    if (!ctx->pyr || ctx->n_oct <= 0) return pano_fail(ctx, PANO_E_ARG, "pano_sift_dog: no resident pyramid");
    for (int o = 0; o < ctx->n_oct; ++o) {
        const size_t npx = (size_t)ctx->n * ctx->oct_h[o] * ctx->oct_w[o];
        const unsigned blocks = (unsigned)std::min<size_t>((npx + 255) / 256, 4096);
        for (int l = 0; l + 1 < ctx->n_lvl; ++l) {
            dog_from_levels<<<blocks, 256, 0, ctx->stream>>>(ctx->pyr + ctx->gauss_off[o][l],
                                                             ctx->pyr + ctx->gauss_off[o][l + 1],
                                                             ctx->dog + ctx->dog_off[o][l], npx);
            PANO_LAUNCH_CHECK(ctx, "dog_from_levels");
        }
    }
    return PANO_OK;
}
