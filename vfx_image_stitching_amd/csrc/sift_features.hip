// sift_features.hip -- S5..S9 of sift_impl.py on the pyramid built by sift_pyramid.hip.
//
//   extrema_scan      find_scale_space_extrema :117-140 + is_pixel_an_extremum :143-163
//                     (LDS-tiled, every octave in one launch)
//   localize          localize_extremum_via_quadratic_fit :169-211 (thread per candidate)
//   orientation       compute_keypoints_with_orientations :246-293 (wave per candidate)
//   bucket_*          compare_keypoints :299-316 (rank = sorted slot: counting sort on x)
//   emit_keypoints    remove_duplicate_keypoints :319-327 + convert_keypoints_to_input_image_size
//                     :333-343 (workgroup per frame)
//   descriptor_wave   unpack_octave :349-358 + generate_descriptors :361-526
//                     (persistent waves, one keypoint per wave at a time)
//
// Parity notes (DESIGN.md "Parity"):
//  * extrema decisions are exact f32 comparisons; the cube / gradient / Hessian are the
//    reference's f32 expressions in its evaluation order (no contraction);
//  * lstsq (numpy: LAPACK dgelsd in double, result cast to f32) is an LU solve with partial
//    pivoting in double, falling back to a Jacobi pseudo-inverse with numpy's
//    rcond = 3 * DBL_EPSILON cut when the Hessian is near-singular;
//  * np.dot of two 3-vectors = f32 products summed in double (OpenBLAS tail loop);
//  * histograms accumulate in 64-bit fixed point (order independent => deterministic, and
//    more accurate than the reference's sequential sums);
//  * np.linalg.norm of the 128-vector reproduces OpenBLAS's SkylakeX sdot order exactly;
//  * numpy's SIMD expf/atan2f are not correctly rounded (1-3 ulp); the kernels use
//    (near) correctly rounded versions, so angles and descriptor bins agree to ulps and
//    integer descriptors to <= 1 LSB.
#include "pano_internal.h"

#include <algorithm>

namespace {

constexpr float kRad2DegF32 = 180.0f / 3.14159265358979323846f;   // numpy f32 rad2deg
constexpr double kHistScale = 1099511627776.0;                    // 2^40 fixed point
constexpr double kHistInv = 1.0 / 1099511627776.0;

// a / b correctly rounded from y = RN(1 / b) (Markstein): q = RN(a y) is within one ulp, the
// remainder a - b q is exact under fma, and RN(q + r y) is the correctly rounded quotient
// (no under/overflow here: |a| < 2^12, b > 2^-4).  Same value as the hardware divide.
__device__ __forceinline__ double div_rn(double a, double b, double y) {
    const double q = a * y;
    const double r = fma(-q, b, a);
    return fma(r, y, q);
}

// llrint for |x| < 2^51 in two instructions: adding 1.5 * 2^52 rounds to an integer (ties to
// even, as llrint in the default mode) and leaves it in the low mantissa bits.  Histogram
// contributions are < 2^9 * 2^40, far inside the range.
__device__ __forceinline__ unsigned long long rint_fix(double x) {
    const double magic = 6755399441055744.0;
    return (unsigned long long)(__double_as_longlong(x + magic) - __double_as_longlong(magic));
}
// Per-frame scratch capacities scale with the pyramid: raw DoG extrema <= sum(Po) / 32
// (32768 at 512 x 384, 345k at 1080p), localised candidates and oriented keypoints <= 1/4
// of that.  Every count is checked against its capacity (PANO_E_OVERFLOW), never clamped
// silently.
constexpr int kExtMin = 32768;
constexpr int kCandMin = 8192;

struct PyrArgs {   // all octaves, for the descriptor (level pointers are per frame batch)
    const float *gauss[PANO_MAX_OCTAVES][PANO_MAX_LEVELS];
    int H[PANO_MAX_OCTAVES], W[PANO_MAX_OCTAVES];
    int n_oct, n_lvl;
};

struct LocParams {
    double thresh;          // floor(0.5 * contrast / ni * 255)
    float contrast;         // f32(contrast_threshold)
    float edge_lhs;         // f32(eigen_ratio)
    float edge_rhs;         // f32((eigen_ratio + 1)^2)
    float sigma_f;          // f32(sigma)
    int ni, border, max_iter, octave;
};

// ------------------------------------------------------------------ 3x3 lstsq
// Symmetric Jacobi eigen-decomposition -> min-norm least-squares solution, cutting
// singular values <= rcond * s_max like LAPACK dgelsd with numpy's default rcond.
__device__ void lstsq3_sym(const double A[3][3], const double b[3], double x[3]) {
    double a[3][3], v[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            a[i][j] = A[i][j];
            v[i][j] = (i == j) ? 1.0 : 0.0;
        }
    // Cyclic Jacobi converges quadratically: stop once the off-diagonal mass is below
    // 1e-20 of the diagonal -- later rotations would move x by ~1e-20 relative, far under
    // the f32 rounding of the result (the solve only has to reproduce dgelsd -> float32).
    for (int sweep = 0; sweep < 16; ++sweep) {
        const double off = fabs(a[0][1]) + fabs(a[0][2]) + fabs(a[1][2]);
        if (off <= 1e-20 * (fabs(a[0][0]) + fabs(a[1][1]) + fabs(a[2][2]))) break;
        for (int pq = 0; pq < 3; ++pq) {
            const int p = pq == 2 ? 1 : 0;
            const int q = pq == 0 ? 1 : 2;
            const double apq = a[p][q];
            if (apq == 0.0) continue;
            const double theta = (a[q][q] - a[p][p]) / (2.0 * apq);
            const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
            const double c = 1.0 / sqrt(t * t + 1.0);
            const double s = t * c;
            for (int k = 0; k < 3; ++k) {   // A <- A J
                const double akp = a[k][p], akq = a[k][q];
                a[k][p] = c * akp - s * akq;
                a[k][q] = s * akp + c * akq;
            }
            for (int k = 0; k < 3; ++k) {   // A <- J^T A
                const double apk = a[p][k], aqk = a[q][k];
                a[p][k] = c * apk - s * aqk;
                a[q][k] = s * apk + c * aqk;
            }
            a[p][q] = a[q][p] = 0.0;
            for (int k = 0; k < 3; ++k) {
                const double vkp = v[k][p], vkq = v[k][q];
                v[k][p] = c * vkp - s * vkq;
                v[k][q] = s * vkp + c * vkq;
            }
        }
    }
    double smax = 0.0;
    for (int k = 0; k < 3; ++k) smax = fmax(smax, fabs(a[k][k]));
    const double cut = 3.0 * 2.220446049250313e-16 * smax;
    x[0] = x[1] = x[2] = 0.0;
    for (int k = 0; k < 3; ++k) {
        const double lam = a[k][k];
        if (!(fabs(lam) > cut)) continue;
        const double coef = (v[0][k] * b[0] + v[1][k] * b[1] + v[2][k] * b[2]) / lam;
        for (int i = 0; i < 3; ++i) x[i] += coef * v[i][k];
    }
}

// Well-conditioned fast path for the same solve: LU with partial pivoting in double.
// dgelsd and LU both land within ~cond * 1e-16 of the exact solution, far below the f32
// rounding the result goes through; near-singular Hessians (a pivot under 1e-6 of the
// largest entry, i.e. cond >~ 1e6) take the Jacobi pseudo-inverse, which reproduces
// dgelsd's rank cut.  Returns false when the fallback is needed.
__device__ __forceinline__ bool solve3_lu(const double A[3][3], const double b[3], double x[3]) {
    double a0[3] = {A[0][0], A[0][1], A[0][2]}, a1[3] = {A[1][0], A[1][1], A[1][2]},
           a2[3] = {A[2][0], A[2][1], A[2][2]};
    double r0 = b[0], r1 = b[1], r2 = b[2];
    double amax = 0.0;
    for (int j = 0; j < 3; ++j) amax = fmax(amax, fmax(fabs(a0[j]), fmax(fabs(a1[j]), fabs(a2[j]))));
    const double tol = 1e-6 * amax;
    auto swp = [](double (&u)[3], double (&v)[3], double &ru, double &rv) {
        for (int j = 0; j < 3; ++j) { const double t = u[j]; u[j] = v[j]; v[j] = t; }
        const double t = ru; ru = rv; rv = t;
    };
    if (fabs(a1[0]) > fabs(a0[0]) && fabs(a1[0]) >= fabs(a2[0])) swp(a0, a1, r0, r1);
    else if (fabs(a2[0]) > fabs(a0[0])) swp(a0, a2, r0, r2);
    if (!(fabs(a0[0]) > tol)) return false;
    const double l1 = a1[0] / a0[0], l2 = a2[0] / a0[0];
    a1[1] -= l1 * a0[1]; a1[2] -= l1 * a0[2]; r1 -= l1 * r0;
    a2[1] -= l2 * a0[1]; a2[2] -= l2 * a0[2]; r2 -= l2 * r0;
    if (fabs(a2[1]) > fabs(a1[1])) swp(a1, a2, r1, r2);
    if (!(fabs(a1[1]) > tol)) return false;
    const double l = a2[1] / a1[1];
    a2[2] -= l * a1[2]; r2 -= l * r1;
    if (!(fabs(a2[2]) > tol)) return false;
    x[2] = r2 / a2[2];
    x[1] = (r1 - a1[2] * x[2]) / a1[1];
    x[0] = (r0 - a0[1] * x[1] - a0[2] * x[2]) / a0[0];
    return true;
}

// ------------------------------------------------------------------ S5 + S6
// S5: one launch covers every octave: workgroup = one 64 x 8 tile of the interior of one
// octave of one frame; the ni+2 DoG levels of the tile (+1 halo) are staged in LDS and each
// pixel is checked against its 26 neighbours there (exact f32 comparisons).  Candidates are
// appended per frame with their scan-order key; S6 runs densely, thread per candidate.
constexpr int ETX = 62, ETY = 16;   // output columns / rows of a tile
constexpr int ELW = 64;             // staged columns (ETX + 2 halo): one per lane

struct DogArgs {
    const float *dog[PANO_MAX_OCTAVES][PANO_MAX_LEVELS];
    int H[PANO_MAX_OCTAVES], W[PANO_MAX_OCTAVES];
    int tiles_x[PANO_MAX_OCTAVES];
    int tile_start[PANO_MAX_OCTAVES + 1];
    int n_oct;
};

// The reference's scan order (octave, layer, row, column) as one integer: 16 bits per
// coordinate, so frames up to 4096 px per side (base 8192, the sort's bucket limit).
__device__ __forceinline__ uint64_t scan_key(int o, int layer0, int y, int x) {
    return ((uint64_t)(o * 8 + layer0) << 32) | ((uint64_t)y << 16) | (uint64_t)x;
}

template <int NL>
__global__ void __launch_bounds__(256)
extrema_scan(DogArgs a, int border, double thresh, uint64_t *__restrict__ raw,
             int32_t *__restrict__ raw_cnt, int raw_cap, int tile_base) {
    constexpr int ni = NL - 2;
    __shared__ float s[NL][ETY + 2][ELW];
    __shared__ int wtot[4], wbase;
    const unsigned tb = xcd_swizzle(linear_block_id(), gridDim.x * gridDim.y);
    const int f = (int)(tb / gridDim.x);
    int t = (int)(tb % gridDim.x) + tile_base, o = 0;
    while (o + 1 < a.n_oct && t >= a.tile_start[o + 1]) ++o;
    t -= a.tile_start[o];
    const int H = a.H[o], W = a.W[o];
    const int x0 = border + (t % a.tiles_x[o]) * ETX;
    const int y0 = border + (t / a.tiles_x[o]) * ETY;
    const int tid = threadIdx.x;
    // stage the NL DoG levels of the tile (+1 halo): wave w stages (level, row) w, w+4, ...
    // with lane = column (62 outputs + 2 halo columns per row).  Level and row are scalar
    // (readfirstlane), so each staged row is one scalar row pointer + one coalesced load;
    // all of a lane's loads are issued before its first LDS store.
    const int lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    constexpr int NROWS = NL * (ETY + 2);
    constexpr int RB = (NROWS + 3) / 4;
    const int gx = min(x0 - 1 + lane, W - 1);
    float va[RB];
#pragma unroll
    for (int u = 0; u < RB; ++u) {
        const int rr = wv + 4 * u;
        if (rr < NROWS) {
            const int l = rr / (ETY + 2), yy = rr - l * (ETY + 2);
            const int gy = min(y0 - 1 + yy, H - 1);
            va[u] = a.dog[o][l][((size_t)f * H + gy) * W + gx];
        }
    }
#pragma unroll
    for (int u = 0; u < RB; ++u) {
        const int rr = wv + 4 * u;
        if (rr < NROWS) {
            const int l = rr / (ETY + 2), yy = rr - l * (ETY + 2);
            s[l][yy][lane] = va[u];
        }
    }
    __syncthreads();
    // is_pixel_an_extremum: v >= all 26 neighbours  <=>  v == max of the 3x3x3 cube (v is
    // in it), likewise <= / min.  The cube max/min is separable: lane = column, 3-wide
    // horizontal then 3-tall vertical max/min per level in registers (4 output rows per
    // thread), then the 3-level max/min per layer.  Exact: only f32 max/min/compare.
    constexpr int RPT = ETY / 4;                  // output rows per thread
    static_assert(ETX + 2 == ELW && ETY % 4 == 0, "lane = column, 4 row groups");
    const int py0 = wv * RPT;
    float vmx[NL][RPT], vmn[NL][RPT];
#pragma unroll
    for (int l = 0; l < NL; ++l) {
        float hmx[RPT + 2], hmn[RPT + 2];
#pragma unroll
        for (int r = 0; r < RPT + 2; ++r) {
            const float *row = &s[l][py0 + r][0];
            const float a0 = row[lane], a1 = row[min(lane + 1, ELW - 1)], a2 = row[min(lane + 2, ELW - 1)];
            hmx[r] = fmaxf(fmaxf(a0, a1), a2);
            hmn[r] = fminf(fminf(a0, a1), a2);
        }
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
            vmx[l][i] = fmaxf(fmaxf(hmx[i], hmx[i + 1]), hmx[i + 2]);
            vmn[l][i] = fminf(fminf(hmn[i], hmn[i + 1]), hmn[i + 2]);
        }
    }
    const int x = x0 + lane;
    uint32_t hits = 0;                            // bit i * 8 + L: extremum at row i, layer L
    if (lane < ETX && x < W - border) {
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
            const int py = py0 + i, y = y0 + py;
            if (y >= H - border) break;
#pragma unroll
            for (int L = 1; L <= ni; ++L) {
                const float v = s[L][py + 1][lane + 1];
                if (!((double)fabsf(v) > thresh)) continue;
                const bool ext = v > 0
                    ? v >= fmaxf(fmaxf(vmx[L - 1][i], vmx[L][i]), vmx[L + 1][i])
                    : v <= fminf(fminf(vmn[L - 1][i], vmn[L][i]), vmn[L + 1][i]);
                if (ext) hits |= 1u << (i * 8 + L);
            }
        }
    }
    // one global atomic per workgroup: wave prefix sums of the per-lane hit counts, wave
    // totals through LDS, then each lane writes its keys (key order is restored downstream)
    const int mine = __popc(hits);
    int incl = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
    }
    if (lane == 63) wtot[wv] = incl;
    __syncthreads();
    if (tid == 0) {
        const int tot = wtot[0] + wtot[1] + wtot[2] + wtot[3];
        wbase = tot ? atomicAdd(&raw_cnt[f * kCntStride], tot) : 0;
    }
    __syncthreads();
    int slot = wbase + incl - mine;
    for (int w = 0; w < wv; ++w) slot += wtot[w];
    while (hits) {
        const int b = __ffs(hits) - 1;
        hits &= hits - 1;
        if (slot < raw_cap)
            raw[(size_t)f * raw_cap + slot] = scan_key(o, b & 7, y0 + py0 + (b >> 3), x);
        ++slot;
    }
}

// Streaming form of the same test: one WAVE per item = a 62-column strip of SR output rows (extrema_xsr)
// of one octave of one frame.  Lane = column (lanes 0 and 63 are the 1-px halo); the wave
// walks down the rows with the NL DoG values of PD rows prefetched in registers, forms the
// horizontal 3-max/min of each level with two lane shifts, keeps the last three rows of those
// in registers for the vertical 3-max/min, and tests the row behind.  No LDS tile, no block
// barrier: each wave streams its rows as a chain of coalesced 256-byte loads.  Hits (rare)
// are gathered in a per-wave LDS buffer and appended with one atomic per flush.
constexpr int XSW = 62;          // output columns per strip
#ifndef PANO_XNT
#define PANO_XNT 0               // A/B: cache-policy bits of the streaming scan's DoG loads (2: nt)
#endif
#ifndef PANO_XPD
#define PANO_XPD 3
#endif
constexpr int XPD = PANO_XPD;    // rows prefetched ahead
#ifndef PANO_XSTREAM_BLOCKS
#define PANO_XSTREAM_BLOCKS 1    // waves per SIMD the register budget is sized for (6: 80 VGPRs, within noise; 8: spills, 2.5x slower)
#endif

struct XArgs {
    const float *dog[PANO_MAX_OCTAVES][PANO_MAX_LEVELS];
    int H[PANO_MAX_OCTAVES], W[PANO_MAX_OCTAVES];
    int strips_x[PANO_MAX_OCTAVES];
    int item_start[PANO_MAX_OCTAVES + 1];
    int n_oct;
    int sr;                      // output rows per item (extrema_xsr)
};

// Whole-wave lane shifts by one through DPP (wave_shr:1 / wave_shl:1, GFX9 DPP controls):
// one VALU op instead of a ds_bpermute round trip.  The end lanes get 0 (only halo lanes use
// them).  PANO_XDPP=0 keeps __shfl_up / __shfl_down.
#ifndef PANO_XDPP
#define PANO_XDPP 1
#endif
__device__ __forceinline__ float lane_from_below(float v) {     // lane i <- lane i - 1
#if PANO_XDPP
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, false));
#else
    return __shfl_up(v, 1);
#endif
}
__device__ __forceinline__ float lane_from_above(float v) {     // lane i <- lane i + 1
#if PANO_XDPP
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xf, 0xf, false));
#else
    return __shfl_down(v, 1);
#endif
}

__device__ __forceinline__ float max3f(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }
__device__ __forceinline__ float min3f(float a, float b, float c) { return fminf(fminf(a, b), c); }

template <int NL, int SR>
__global__ void __launch_bounds__(256, PANO_XSTREAM_BLOCKS)
extrema_stream(XArgs a, int border, double thresh, uint64_t *__restrict__ raw,
               int32_t *__restrict__ raw_cnt, int raw_cap, int item_base, int item_end) {
    constexpr int ni = NL - 2;
    constexpr int BUF = 64;
    __shared__ uint64_t kbuf[4][BUF];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int f = blockIdx.y;
    int t = item_base + (int)blockIdx.x * 4 + wv;
    if (t >= item_end) return;                                     // whole wave
    int o = 0;
    while (o + 1 < a.n_oct && t >= a.item_start[o + 1]) ++o;
    t -= a.item_start[o];
    const int H = a.H[o], W = a.W[o];
    const int x0 = border + (t % a.strips_x[o]) * XSW;
    const int y0 = border + (t / a.strips_x[o]) * SR;
    const int yend = min(y0 + SR, H - border);                     // last input row (inclusive)
    const int x = x0 - 1 + lane;
    const int gx = min(x, W - 1);
    const bool out_lane = lane >= 1 && lane <= XSW && x < W - border;
    // the NL planes of this frame as buffer resources (scalar registers) read at ONE per-lane
    // byte offset per row: five 64-bit per-lane pointers cost ten VGPRs
    __amdgpu_buffer_rsrc_t rs[NL];
#pragma unroll
    for (int l = 0; l < NL; ++l)
        rs[l] = __builtin_amdgcn_make_buffer_rsrc((void *)(a.dog[o][l] + (size_t)f * H * W), 0, H * W * 4, 0x00020000);
    auto ld = [&](int l, int r) {
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs[l], (r * W + gx) * 4, 0, PANO_XNT));
    };
    int nbuf = 0;                                                   // wave-uniform
    auto flush = [&]() {
        if (nbuf == 0) return;
        __builtin_amdgcn_wave_barrier();
        int base = 0;
        if (lane == 0) base = atomicAdd(&raw_cnt[f * kCntStride], nbuf);
        base = __shfl(base, 0);
        for (int i = lane; i < nbuf; i += 64)
            if (base + i < raw_cap) raw[(size_t)f * raw_cap + base + i] = kbuf[wv][i];
        __builtin_amdgcn_wave_barrier();
        nbuf = 0;
    };
    float nx[XPD][NL];                                              // prefetched rows
#pragma unroll
    for (int k = 0; k < XPD; ++k) {
        const int r = y0 - 1 + k;
        if (r <= yend) {
#pragma unroll
            for (int l = 0; l < NL; ++l) nx[k][l] = ld(l, r);
        }
    }
    float hxA[NL], hnA[NL], hxB[NL], hnB[NL], cB[NL];               // rows r-2 (A), r-1 (B)
    for (int r0 = y0 - 1; r0 <= yend; r0 += XPD) {
#pragma unroll
        for (int k = 0; k < XPD; ++k) {
            const int r = r0 + k;
            if (r > yend) break;
            float c[NL];
#pragma unroll
            for (int l = 0; l < NL; ++l) c[l] = nx[k][l];
            if (r + XPD <= yend) {
#pragma unroll
                for (int l = 0; l < NL; ++l) nx[k][l] = ld(l, r + XPD);
            }
            float hxC[NL], hnC[NL];
#pragma unroll
            for (int l = 0; l < NL; ++l) {
                const float lf = lane_from_below(c[l]), rt = lane_from_above(c[l]);
                hxC[l] = max3f(lf, c[l], rt);
                hnC[l] = min3f(lf, c[l], rt);
            }
            if (r >= y0 + 1) {                                      // test output row r - 1
                float vx[NL], vn[NL];
#pragma unroll
                for (int l = 0; l < NL; ++l) {
                    vx[l] = max3f(hxA[l], hxB[l], hxC[l]);
                    vn[l] = min3f(hnA[l], hnB[l], hnC[l]);
                }
#pragma unroll
                for (int L = 1; L <= ni; ++L) {
                    const float v = cB[L];
                    bool ext = false;
                    if (out_lane && (double)fabsf(v) > thresh)
                        ext = v > 0 ? v >= max3f(vx[L - 1], vx[L], vx[L + 1])
                                    : v <= min3f(vn[L - 1], vn[L], vn[L + 1]);
                    const unsigned long long m = __ballot(ext);
                    if (m) {                                        // wave-uniform
                        const int k2 = __popcll(m);
                        if (nbuf + k2 > BUF) flush();
                        if (ext) {
                            const int pos = nbuf + __popcll(m & ((1ull << lane) - 1));
                            kbuf[wv][pos] = scan_key(o, L, r - 1, x);
                        }
                        nbuf += k2;
                    }
                }
            }
#pragma unroll
            for (int l = 0; l < NL; ++l) {
                hxA[l] = hxB[l]; hnA[l] = hnB[l];
                hxB[l] = hxC[l]; hnB[l] = hnC[l];
                cB[l] = c[l];
            }
        }
    }
    flush();
}

__device__ __forceinline__ float dog_at(const DogArgs &a, int o, int lvl, int f, int y, int x) {
    return a.dog[o][lvl][((size_t)f * a.H[o] + y) * a.W[o] + x];
}

// One extremum through the quadratic fit and the contrast / edge tests.
// v / 255 by the reciprocal and one exact-residual correction: equal to the IEEE quotient for
// every f32 |v| <= 256, subnormals included (exhaustive: tools/probes/div360_check.c with
// the divisor 255); DoG values are within +-255
__device__ __forceinline__ float div255(float v) {
    constexpr float y = 1.0f / 255.0f;
    const float q = v * y;
    return fmaf(fmaf(-q, 255.0f, v), y, q);
}

__device__ bool localize_one(const DogArgs &a, const LocParams &lp, uint64_t key, int f, Cand &k) {
    const int o = (int)(key >> 32) / 8, layer0 = (int)(key >> 32) % 8;
    const int y = (int)((key >> 16) & 65535), x = (int)(key & 65535);
    const int ni = lp.ni, border = lp.border;
    const int H = a.H[o], W = a.W[o];
    // ---- quadratic fit (sift_impl.py:169-211), keeping the max_iter quirk
    int xi = x, yi = y, li = layer0;
    float c[3][3][3];
    float g[3], Hs[3][3], u[3];
    for (int it = 0; it < lp.max_iter; ++it) {
        for (int dz = 0; dz < 3; ++dz)
            for (int dy = 0; dy < 3; ++dy)
                for (int dx = 0; dx < 3; ++dx)
                    c[dz][dy][dx] = div255(dog_at(a, o, li - 1 + dz, f, yi - 1 + dy, xi - 1 + dx));
        const float cv = c[1][1][1];
        g[0] = 0.5f * (c[1][1][2] - c[1][1][0]);
        g[1] = 0.5f * (c[1][2][1] - c[1][0][1]);
        g[2] = 0.5f * (c[2][1][1] - c[0][1][1]);
        const float v2 = 2.0f * cv;
        const float dxx = (c[1][1][2] - v2) + c[1][1][0];
        const float dyy = (c[1][2][1] - v2) + c[1][0][1];
        const float dss = (c[2][1][1] - v2) + c[0][1][1];
        const float dxy = 0.25f * (((c[1][2][2] - c[1][2][0]) - c[1][0][2]) + c[1][0][0]);
        const float dxs = 0.25f * (((c[2][1][2] - c[2][1][0]) - c[0][1][2]) + c[0][1][0]);
        const float dys = 0.25f * (((c[2][2][1] - c[2][0][1]) - c[0][2][1]) + c[0][0][1]);
        Hs[0][0] = dxx; Hs[0][1] = dxy; Hs[0][2] = dxs;
        Hs[1][0] = dxy; Hs[1][1] = dyy; Hs[1][2] = dys;
        Hs[2][0] = dxs; Hs[2][1] = dys; Hs[2][2] = dss;
        double A[3][3], b[3], sol[3];
        for (int i = 0; i < 3; ++i) {
            b[i] = g[i];
            for (int j = 0; j < 3; ++j) A[i][j] = Hs[i][j];
        }
        if (!solve3_lu(A, b, sol)) lstsq3_sym(A, b, sol);
        for (int i = 0; i < 3; ++i) u[i] = -(float)sol[i];
        if (fabsf(u[0]) < 0.5f && fabsf(u[1]) < 0.5f && fabsf(u[2]) < 0.5f) break;
        xi += (int)rintf(u[0]);
        yi += (int)rintf(u[1]);
        li += (int)rintf(u[2]);
        if (yi < border || yi >= H - border || xi < border || xi >= W - border || li < 1 ||
            li > ni)
            return false;
    }
    double dacc = 0.0;
    for (int i = 0; i < 3; ++i) dacc += (double)(g[i] * u[i]);
    const float val = c[1][1][1] + 0.5f * (float)dacc;
    if (fabsf(val) * (float)ni < lp.contrast) return false;
    const float tr = Hs[0][0] + Hs[1][1];
    const float det = (float)((double)Hs[0][0] * (double)Hs[1][1] -
                              (double)Hs[0][1] * (double)Hs[1][0]);
    if (det <= 0.0f || lp.edge_lhs * (tr * tr) >= lp.edge_rhs * det) return false;
    const float so = (float)(1 << o);
    k.x = ((float)xi + u[0]) * so;
    k.y = ((float)yi + u[1]) * so;
    k.octave_field = o + li * 256 + (int)rintf((u[2] + 0.5f) * 255.0f) * 65536;
    const float e = ((float)li + u[2]) / (float)ni;
    const float p2 = (float)exp2((double)e);            // 2 ** np.float32 (libm powf)
    k.size = (lp.sigma_f * p2) * (float)(1 << (o + 1));
    k.response = fabsf(val);
    k.octave = (int16_t)o;
    k.layer = (int16_t)li;
    k.frame = f;
    k.order = key;
    return true;
}

__global__ void __launch_bounds__(256)
localize(DogArgs a, LocParams lp, const uint64_t *__restrict__ raw,
         const int32_t *__restrict__ raw_cnt, int raw_cap, Cand *__restrict__ cands,
         int32_t *__restrict__ cand_cnt, int cand_cap) {
    // grid (frame, block): the dispatcher walks x fastest, so every frame's live blocks (the
    // low block indices; the grid is sized by the capacity) go out before the empty ones
    const int f = blockIdx.x;
    const int ci = blockIdx.y * 256 + threadIdx.x;
    int cnt = raw_cnt[f * kCntStride];
    cnt = cnt < raw_cap ? cnt : raw_cap;
    if ((int)blockIdx.y * 256 >= cnt) return;   // uniform
    bool keep = false;
    Cand k;
    if (ci < cnt) keep = localize_one(a, lp, raw[(size_t)f * raw_cap + ci], f, k);
    const unsigned long long m = __ballot(keep);
    const int lane = threadIdx.x & 63;
    int base = 0;
    if (lane == 0 && m) base = atomicAdd(&cand_cnt[f * kCntStride], __popcll(m));
    base = __shfl(base, 0);
    const int slot = base + __popcll(m & ((1ull << lane) - 1));
    if (keep && slot < cand_cap) cands[(size_t)f * cand_cap + slot] = k;
}


// ------------------------------------------------------------------ S7
#ifndef PANO_ORI_ABL
#define PANO_ORI_ABL 0         // timing ablations of orientation only (bit 1: no atan2f, 2: no expf,
                               // 4: no patch loads, 8: no emit atomic -- slots from the work index)
#endif
#ifndef PANO_ORI_COPIES
#define PANO_ORI_COPIES 1      // histogram copies per wave (measured: 4 and 8 no faster)
#endif
constexpr int kOriCopies = PANO_ORI_COPIES;
#ifndef PANO_ORI_CLAIM
#define PANO_ORI_CLAIM 1       // candidates claimed per atomic (per-XCD work counter)
#endif
constexpr int kOriClaim = PANO_ORI_CLAIM;
constexpr float kInv360 = 1.0f / 360.0f;   // RN(1 / 360)
#ifndef PANO_ORI_PATCH
#define PANO_ORI_PATCH 37
#endif
constexpr int kOriPatch = PANO_ORI_PATCH;   // staged patch side: radius <= 17 (default params: <= 16)
#ifndef PANO_ORI_STAGE
#define PANO_ORI_STAGE 8
#endif
constexpr int kOriStage = PANO_ORI_STAGE;
#ifndef PANO_ORI_BLOCKS
#define PANO_ORI_BLOCKS 6        // waves per SIMD the register budget is sized for (80 VGPRs; measured 1-3 % faster than 88)
#endif   // patch loads per lane in flight (37^2 / 64 <= 22: two rounds)

// atan2(y, x) in units of pi/4 ("octants", (-4, 4]): octant reduction to a = min/max in
// [0, 1] and an odd minimax polynomial of degree 15 (f32 Horner, |error| < 2.1e-7 octant).
// The descriptor only uses the angle through the continuous trilinear weights, so a few
// ulps here move each contribution by ~1e-7 relative -- the size of the reference's own f32
// np.add.at rounding (sift_impl.py:499-500); atan2(0, 0) = 0 as numpy's.
__device__ __forceinline__ float atan2_oct(float y, float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    // v_rcp_f32 flushes a subnormal argument (0 * inf = NaN): gradients that small (flat
    // black borders of the cylindrical frames after the cascaded blurs) have magnitude 0 in
    // f32 anyway, so their angle is taken as 0, numpy's atan2(0, 0)
    const float a = mx >= 1.17549435e-38f ? mn * __builtin_amdgcn_rcpf(mx) : 0.0f;
    const float t = a * a;
    float p = -0.005166319198906422f;
    p = fmaf(p, t, 0.027850419282913208f);
    p = fmaf(p, t, -0.07120880484580994f);
    p = fmaf(p, t, 0.1227816641330719f);
    p = fmaf(p, t, -0.1770951747894287f);
    p = fmaf(p, t, 0.2539685070514679f);
    p = fmaf(p, t, -0.42436903715133667f);
    p = fmaf(p, t, 1.2732386589050293f);
    float r = p * a;                               // atan(a) / (pi / 4), in [0, 1]
    r = ay > ax ? 2.0f - r : r;
    r = x < 0.0f ? 4.0f - r : r;
    return y < 0.0f ? -r : r;
}

struct OriParams {
    double scale_factor, radius_factor, peak_ratio;
    int fast_bin;           // orientation bins from atan2_oct away from bin edges (PANO_ORI_FAST_BIN)
};

// The orientation bin of a gradient (sift_impl.py:268-275): np.rad2deg(np.arctan2(dy, dx)) in
// f32, np.remainder(., 360), round(angle * 36 / 360) mod 36 -- the exact f32 sequence.
__device__ __forceinline__ int ori_bin_exact(float gx, float gy) {
    const float a = atan2f(gy, gx) * kRad2DegF32;
    // np.remainder(a, 360) for |a| <= 180 (atan2f in [-pi, pi] times the f32 rad2deg)
    const float ang = a < 0.0f ? a + 360.0f : (a == 0.0f ? 0.0f : a);
    // (ang * 36) / 360 by the reciprocal and one exact-residual correction: the same bin as the
    // IEEE division for every f32 (exhaustive: tools/probes/div360_check.c)
    const float a36 = ang * 36.0f;
    const float q0 = a36 * kInv360;
    const int bin = (int)rintf(fmaf(fmaf(-q0, 360.0f, a36), kInv360, q0));
    return bin >= PANO_ORI_BINS ? bin - PANO_ORI_BINS : bin;
}

// The same bin from atan2_oct (|error| < 2.1e-7 octant = 1e-5 deg) wherever the angle is more
// than kOriBinGuard bins (2e-3 deg, 100x the error of either path) from a bin edge
// (10k + 5 deg); within the guard, ori_bin_exact.  Identical bins for every gradient of
// non-zero magnitude (a zero magnitude adds 0 to any bin): test_orientation_fast_bin_identical.
constexpr float kOriBinGuard = 2e-4f;
__device__ __forceinline__ int ori_bin(float gx, float gy, bool fast) {
    if (fast && PANO_ORI_BINS == 36) {
        float u = atan2_oct(gy, gx) * 4.5f;        // octants -> bins of 10 deg, (-18, 18]
        u = u < 0.0f ? u + 36.0f : u;
        const float fu = u - floorf(u);
        if (fabsf(fu - 0.5f) > kOriBinGuard) {
            const int bin = (int)floorf(u + 0.5f);
            return bin >= 36 ? bin - 36 : bin;
        }
    }
    return ori_bin_exact(gx, gy);
}

// Dense candidate index gk (frames back to back, counts strided kCntStride and clamped to
// [0, cap]) -> (frame, index); false past the last candidate.
__device__ __forceinline__ bool locate_strided(const int32_t *__restrict__ counts, int n_frames, int cap,
                                               int gk, int &f, int &k) {
    const int lane = threadIdx.x & 63;
    int base = 0;
    for (int f0 = 0; f0 < n_frames; f0 += 64) {
        int c = f0 + lane < n_frames ? counts[(f0 + lane) * kCntStride] : 0;
        c = c < 0 ? 0 : (c < cap ? c : cap);
        int incl = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int t = __shfl_up(incl, d);
            if (lane >= d) incl += t;
        }
        const int tot = __shfl(incl, 63);
        if (gk < base + tot) {
            const int j = __popcll(__ballot(base + incl <= gk));
            f = f0 + j;
            k = gk - base - (__shfl(incl, j) - __shfl(c, j));
            return true;
        }
        base += tot;
    }
    return false;
}

// Persistent waves claim their next work item one item ahead (kClaimAhead), so the queue
// atomic's latency overlaps the current item, or when they finish one.  Measured: ahead is
// slower at parrington (a wave holding a claimed item behind a long one delays the drain).
#ifndef PANO_CLAIM_AHEAD
#define PANO_CLAIM_AHEAD 0
#endif
constexpr bool kClaimAhead = PANO_CLAIM_AHEAD != 0;
#ifndef PANO_CLAIM_STATIC
#define PANO_CLAIM_STATIC 1    // orientation / descriptor: each wave's first item dealt, not claimed
#endif
constexpr bool kClaimStatic = PANO_CLAIM_STATIC != 0 && !kClaimAhead;
// Prefetched claims (orientation / descriptor): while a wave's item is more than PANO_CLAIM_FAR
// items per XCD wave from its range's end, the wave issues the atomic for its next item before
// working on this one, so the atomic's round trip overlaps the item's loads; the last items are
// claimed on demand, so no wave holds a claimed item behind a long one while others drain
// (what made kClaimAhead slower).  0 = off.  Measured slower too (profiles/r06_claim_far_ab.txt:
// orientation 0.089 -> 0.101 ms, descriptor 0.215 -> 0.226 ms at parrington with 2): the returning
// atomic joins the in-order vmcnt queue ahead of the item's own loads, so its contended latency
// lands on the first load wait instead of overlapping.
#ifndef PANO_CLAIM_FAR
#define PANO_CLAIM_FAR 0
#endif
constexpr int kClaimFar = kClaimAhead ? 0 : PANO_CLAIM_FAR;

// The dense work index of a persistent wave -> (frame, index).  For <= 64 frames the clamped
// counts and their inclusive prefix live in registers (lane = frame), loaded once per wave, so
// each dequeue is one ballot and two lane reads instead of a scan over HBM-resident counts.
struct FrameIndex {
    int c = 0, incl = 0;
    bool regs = false;
    __device__ void init(const int32_t *__restrict__ counts, int stride, int n_frames, int cap) {
        const int lane = threadIdx.x & 63;
        regs = n_frames <= 64;
        if (!regs) return;
        c = lane < n_frames ? counts[lane * stride] : 0;
        c = c < 0 ? 0 : (c < cap ? c : cap);
        incl = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int t = __shfl_up(incl, d);
            if (lane >= d) incl += t;
        }
    }
    // gk < total (the caller's bound): frames wholly before gk, then the offset inside
    __device__ __forceinline__ void locate(int gk, int &f, int &k) const {
        const int j = __popcll(__ballot(incl <= gk));
        f = j;
        k = gk - (__shfl(incl, j) - __shfl(c, j));
    }
};

// One candidate's orientations (sift_impl.py:246-293) by one wave: the (side+2)^2 neighbourhood
// of the keypoint staged in LDS (pt), each lane its run of column-major samples into 2^40
// fixed-point u64 LDS atomics (hs: kOriCopies copies), smoothing and peak interpolation in f64
// (the reference's).  Returns per lane p < 36 whether bin p is an emitted peak, and its angle.
// img: the octave's Gaussian level (H x W) the reference passes as gauss_img; kx, ky: the
// keypoint in base-image coordinates.  Shared by the batched kernel (orientation) and the
// per-keypoint entry (orient_list, pano_sift_orient).
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#ifndef PANO_ORI_FAST_WALK
#define PANO_ORI_FAST_WALK 1   // interior candidates walk without per-sample bounds tests (identical bins)
#endif
constexpr bool kOriFastWalk = PANO_ORI_FAST_WALK != 0;
#ifndef PANO_ORI_TIMING
#define PANO_ORI_TIMING 0      // 1: diagnostics build, per-wave phase clocks of orientation (tools/ori_clock.py)
#endif
#if PANO_ORI_TIMING
constexpr int kOriClkWaves = 16384;
__device__ unsigned long long g_ori_clk[kOriClkWaves][8];
#define PANO_ORI_NOW() ((unsigned long long)__builtin_amdgcn_s_memrealtime())
extern "C" int pano_dbg_ori_clock(unsigned long long *out, int reset) {
    if (reset) {
        void *p = nullptr;
        if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_ori_clk)) != hipSuccess) return -1;
        return hipMemset(p, 0, sizeof(g_ori_clk)) == hipSuccess ? 0 : -1;
    }
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ori_clk), sizeof(g_ori_clk)) == hipSuccess ? 0 : -1;
}
#endif

__device__ __forceinline__ bool orient_one(const float *__restrict__ img, int H, int W, int o, float kx, float ky,
                                           float ksize, const OriParams &op,
                                           unsigned long long (*hs)[PANO_ORI_BINS], double *hd, double *sm,
                                           float *pt, int lane, double &angle,
                                           unsigned long long *ts = nullptr) {
    for (int i = lane; i < kOriCopies * PANO_ORI_BINS; i += 64) (&hs[0][0])[i] = 0ull;
    {
        const float scale = (float)(op.scale_factor * (double)ksize) / (float)(1 << (o + 1));
        const int radius = (int)rintf((float)op.radius_factor * scale);
        const float wfac = -0.5f / (scale * scale);
        const int cy = (int)rintf(ky / (float)(1 << o));
        const int cx = (int)rintf(kx / (float)(1 << o));
        const int side = 2 * radius + 1;
        const int S = side * side;
        // stage the (side+2)^2 neighbourhood (clamped; out-of-image samples are skipped
        // below) so each sample's four gradient taps are LDS reads
        const int P = side + 2;
        const bool staged = P <= kOriPatch;
        if (staged) {
            // kOriStage loads per lane in flight before their LDS stores (a plain loop waited
            // for each load in turn: one memory latency per 64 elements, up to 22 per candidate)
            const int by = cy - radius - 1, bx = cx - radius - 1;
            for (int e0 = 0; e0 < P * P; e0 += 64 * kOriStage) {
                float v[kOriStage];
#pragma unroll
                for (int u = 0; u < kOriStage; ++u) {
                    const int e = e0 + 64 * u + lane;
                    const int r = e / P, c = e - (e / P) * P;
                    const int yy = min(max(by + r, 0), H - 1), xx = min(max(bx + c, 0), W - 1);
#if PANO_ORI_ABL & 4                                  // timing ablation: no patch loads
                    v[u] = (float)(yy ^ xx);
#else
                    v[u] = e < P * P ? img[(size_t)yy * W + xx] : 0.0f;
#endif
                }
#pragma unroll
                for (int u = 0; u < kOriStage; ++u) {
                    const int e = e0 + 64 * u + lane;
                    const int r = e / P, c = e - (e / P) * P;
                    if (e < P * P) pt[r * kOriPatch + c] = v[u];
                }
            }
        }
        wave_sync_lds();
#if PANO_ORI_TIMING
        if (ts) ts[0] = PANO_ORI_NOW();
#endif
        // lane l walks its own run of Q consecutive column-major samples (neighbouring
        // lanes are Q samples apart: different bins, fewer same-address LDS atomics)
        const int Q = (S + 63) / 64;
        const int j0 = lane * Q;
        const int jend = min(j0 + Q, S);
        // INTERIOR: every sample of the square and its four taps inside the image and staged,
        // so no per-sample bounds test and LDS taps only (kOriFastWalk)
        auto walk = [&](auto interior) {
            constexpr bool INTERIOR = decltype(interior)::value;
            int xi = j0 / side, yi = j0 - (j0 / side) * side;
            for (int j = j0; j < jend; ++j, (++yi == side) ? (yi = 0, ++xi) : 0) {
                const int dx = xi - radius, dy = yi - radius;
                float gx, gy;
                if constexpr (INTERIOR) {
                    const float *q = pt + (yi + 1) * kOriPatch + xi + 1;
                    gx = q[1] - q[-1];
                    gy = q[-kOriPatch] - q[kOriPatch];
                } else {
                    const int yy = cy + dy, xx = cx + dx;
                    if (xx <= 0 || xx >= W - 1 || yy <= 0 || yy >= H - 1) continue;
                    if (staged) {
                        const float *q = pt + (yi + 1) * kOriPatch + xi + 1;
                        gx = q[1] - q[-1];
                        gy = q[-kOriPatch] - q[kOriPatch];
                    } else {
                        gx = img[(size_t)yy * W + xx + 1] - img[(size_t)yy * W + xx - 1];
                        gy = img[(size_t)(yy - 1) * W + xx] - img[(size_t)(yy + 1) * W + xx];
                    }
                }
                const float mag = sqrtf(gx * gx + gy * gy);
                // dx^2 + dy^2 as the exact f32 sum of exact f32 squares (|d| <= 2^7): the same
                // value as the integer expression converted, without the integer multiplies
                const float fdx = (float)dx, fdy = (float)dy;
                const float d2 = kOriFastWalk ? fdx * fdx + fdy * fdy : (float)(dx * dx + dy * dy);
#if PANO_ORI_ABL & 2                                  // timing ablation: no expf
                const float w = wfac * d2 + 1.0f;
#else
                const float w = expf(wfac * d2);
#endif
#if PANO_ORI_ABL & 1                                  // timing ablation: no atan2f
                const int bin = (int)(fabsf(gy + gx) * 0.1f) % PANO_ORI_BINS;
#else
                const int bin = ori_bin(gx, gy, op.fast_bin != 0);
#endif
                const double val = (double)(w * mag);
                atomicAdd(&hs[lane % kOriCopies][bin], rint_fix(val * kHistScale));
            }
        };
        const bool interior = staged && cx - radius > 0 && cx + radius < W - 1 && cy - radius > 0 && cy + radius < H - 1;
        if (kOriFastWalk && interior) walk(std::true_type{});
        else walk(std::false_type{});
    }
    wave_sync_lds();
#if PANO_ORI_TIMING
    if (ts) ts[1] = PANO_ORI_NOW();
#endif
    if (lane < PANO_ORI_BINS) {
        unsigned long long t = 0;
#pragma unroll
        for (int c = 0; c < kOriCopies; ++c) t += hs[c][lane];
        hd[lane] = (double)(long long)t * kHistInv;
    }
    wave_sync_lds();
    const int nb = PANO_ORI_BINS;
    double svl = -1.0;                 // this lane's smoothed bin (histogram values are >= 0)
    if (lane < nb) {
        const int b = lane;
        svl = ((6 * hd[b] + 4 * (hd[(b + nb - 1) % nb] + hd[(b + 1) % nb])) + hd[(b + nb - 2) % nb]) +
              hd[(b + 2) % nb];
        svl = svl / 16.0;
        sm[b] = svl;
    }
    double mx = svl;                   // the maximum: exact in any order
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) mx = fmax(mx, __shfl_xor(mx, d));
    wave_sync_lds();
    // peaks: lane p < 36 is bin p
    const int p = lane;
    bool emit = false;
    angle = 0.0;
    if (lane < nb) {
        const double l = sm[(p + nb - 1) % nb], r = sm[(p + 1) % nb];
        if (svl > l && svl > r && svl >= op.peak_ratio * mx) {
            const double interp = np_remainder((double)p + 0.5 * (l - r) / ((l - 2 * svl) + r), (double)nb);
            angle = 360.0 - interp * 360.0 / nb;
            if (fabs(angle - 360.0) < 1e-7) angle = 0.0;
            emit = true;
        }
    }
    return emit;
}

// One WAVE per candidate, persistent: the grid is the resident workgroups (a grid sized by the
// candidate capacity dispatched ~37k mostly-empty workgroups at parrington, 410k at 1080p),
// each XCD takes a contiguous eighth of the candidates and its waves pull them from the XCD's
// own counter (as descriptor_wave).  Per candidate: the (side+2)^2 neighbourhood staged in
// LDS, each lane its run of column-major samples into 2^40 fixed-point u64 LDS atomics,
// smoothing and peak interpolation in f64 (the reference's), one aggregated append.
__global__ void __launch_bounds__(256, PANO_ORI_BLOCKS)
orientation(PyrArgs pa, OriParams op, const Cand *__restrict__ cands,
            const int32_t *__restrict__ cand_cnt, int cand_cap, int n_frames, int32_t *__restrict__ work,
            RawKp *__restrict__ raw, int32_t *__restrict__ raw_cnt, int raw_cap) {
    // kOriCopies interleaved copies of each wave's histogram (copy = lane % kOriCopies): lanes
    // on similar gradient directions hit the same bin; spreading them over copies cuts the
    // same-address LDS atomic serialisation, and integer sums merge exactly
    __shared__ unsigned long long hist[4][kOriCopies][PANO_ORI_BINS];
    __shared__ double hd[4][PANO_ORI_BINS];
    __shared__ double sm[4][PANO_ORI_BINS];
    __shared__ float patch[4][kOriPatch * kOriPatch];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int total = 0;
    for (int f0 = 0; f0 < n_frames; f0 += 64) {
        int c = f0 + lane < n_frames ? cand_cnt[(f0 + lane) * kCntStride] : 0;
        c = c < 0 ? 0 : (c < cand_cap ? c : cand_cap);
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d);
        total += c;
    }
    const int xcd = blockIdx.x & 7;                                   // gridDim.x % 8 == 0
    const int lo_k = (int)((long long)total * xcd / 8), hi_k = (int)((long long)total * (xcd + 1) / 8);
    int32_t *wq = work + xcd * kCntStride;
    FrameIndex fi;
    fi.init(cand_cnt, kCntStride, n_frames, cand_cap);
    int claim = 0;
    int cl_next = 0, cl_end = 0;                 // wave-uniform: claimed candidates [cl_next, cl_end)
    bool pre = false;                            // wave-uniform: a claim is in flight in lane 0's claim
    // every wave's first chunk without an atomic (wave i of the XCD takes chunk i; the counter
    // hands out the rest after them): claiming at launch serialised ~770 atomics on each XCD's
    // counter before its last wave could start
    const int wx = (int)(gridDim.x >> 3) * 4, nw_x = kClaimStatic ? wx : 0;   // waves per XCD
    if (kClaimStatic) {
        cl_next = ((int)(blockIdx.x >> 3) * 4 + wv) * kOriClaim;
        cl_end = cl_next + kOriClaim;
    }
#if PANO_ORI_TIMING
    unsigned long long t_entry = PANO_ORI_NOW(), acc[4] = {0, 0, 0, 0}, ts[2] = {0, 0}, tq = 0, t1 = 0;
    int ncand = 0;
#endif
    if (kClaimAhead && lane == 0) claim = atomicAdd(wq, 1);
    for (;;) {
#if PANO_ORI_TIMING
        tq = PANO_ORI_NOW();
#endif
        int gk;
        if constexpr (kClaimAhead) {
            gk = lo_k + __shfl(claim, 0);
            if (gk >= hi_k) break;
            if (lane == 0) claim = atomicAdd(wq, 1);
        } else {
            if (cl_next >= cl_end) {              // kOriClaim candidates per atomic (as the descriptor)
                if (!pre && lane == 0) claim = atomicAdd(wq, kOriClaim);
                cl_next = nw_x * kOriClaim + __shfl(claim, 0);
                cl_end = cl_next + kOriClaim;
                pre = false;
            }
            gk = lo_k + cl_next++;
            if (gk >= hi_k) break;
            if (kClaimFar && cl_next >= cl_end && gk + kClaimFar * wx * kOriClaim < hi_k) {
                if (lane == 0) claim = atomicAdd(wq, kOriClaim);    // next claim in flight
                pre = true;
            }
        }
        int f = 0, ci = 0;
        if (fi.regs) fi.locate(gk, f, ci);
        else if (!locate_strided(cand_cnt, n_frames, cand_cap, gk, f, ci)) break;
        f = __builtin_amdgcn_readfirstlane(f);
        ci = __builtin_amdgcn_readfirstlane(ci);
        const Cand k = cands[(size_t)f * cand_cap + ci];
        double angle;
        const int p = lane;
#if PANO_ORI_TIMING
        __builtin_amdgcn_s_waitcnt(0);                // the candidate record has arrived
        t1 = PANO_ORI_NOW();
        unsigned long long *tsp = ts;
#else
        unsigned long long *tsp = nullptr;
#endif
        const bool emit = orient_one(pa.gauss[k.octave][k.layer] + (size_t)f * pa.H[k.octave] * pa.W[k.octave],
                                     pa.H[k.octave], pa.W[k.octave], k.octave, k.x, k.y, k.size, op, hist[wv],
                                     hd[wv], sm[wv], patch[wv], lane, angle, tsp);
        const unsigned long long m = __ballot(emit);
        if (m) {
            int base = 0;
#if PANO_ORI_ABL & 8
            base = (gk * 2) % (raw_cap - 64);
#else
            if (lane == __ffsll((long long)m) - 1) base = atomicAdd(&raw_cnt[f * kCntStride], __popcll(m));
#endif
            base = __shfl(base, __ffsll((long long)m) - 1);
            if (emit) {
                RawKp q;
                q.x = k.x;
                q.y = k.y;
                q.size = k.size;
                q.angle = (float)angle;
                q.response = k.response;
                q.octave = k.octave_field;
                q.frame = f;
                q.order = ((uint64_t)k.order << 6) | (uint64_t)p;
                const int slot = base + __popcll(m & ((1ull << lane) - 1));
                if (slot < raw_cap) raw[(size_t)f * raw_cap + slot] = q;
            }
        }
        wave_sync_lds();                   // hist / hd / sm / patch reused by the next candidate
#if PANO_ORI_TIMING
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long t_end = PANO_ORI_NOW();
        acc[0] += t1 - tq;                 // claim, locate, candidate load
        acc[1] += ts[0] - t1;              // patch staging
        acc[2] += ts[1] - ts[0];           // sample walk
        acc[3] += t_end - ts[1];           // histogram, smoothing, peaks, emit
        ++ncand;
#endif
    }
#if PANO_ORI_TIMING
    const int gw = (int)blockIdx.x * 4 + wv;
    if (lane == 0 && gw < kOriClkWaves) {
        unsigned long long *o = g_ori_clk[gw];
        o[0] = t_entry;
        o[1] = PANO_ORI_NOW();
        o[2] = (unsigned long long)ncand;
        o[3] = acc[0];
        o[4] = acc[1];
        o[5] = acc[2];
        o[6] = acc[3];
        o[7] = (unsigned long long)(xcd + 1);
    }
#endif
}

// ------------------------------------------------------------------ S6 / S7 per caller candidate
// The reference's per-candidate helpers (localize_extremum_via_quadratic_fit :169-211,
// compute_keypoints_with_orientations :246-293) on caller-given candidates of ONE octave, through
// the batched kernels' own device functions (localize_one, orient_one): pano_sift_localize /
// pano_sift_orient.
//
// localize_list, thread per candidate (x, y, layer) of octave a.octave's DoG levels: out[i] is the
// keypoint (angle -1, cv2.KeyPoint's default) and layer_out[i] its final layer, or -1 when the
// fit rejects it; a candidate whose 3x3x3 cube leaves the levels is refused (-2) before any read.
__global__ void __launch_bounds__(256)
localize_list(DogArgs a, LocParams lp, int o, const int32_t *__restrict__ cand, int n,
              pano_kp *__restrict__ out, int32_t *__restrict__ layer_out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int x = cand[3 * i], y = cand[3 * i + 1], layer = cand[3 * i + 2];
    if (x < 1 || y < 1 || x > a.W[o] - 2 || y > a.H[o] - 2 || layer < 1 || layer > lp.ni) {
        layer_out[i] = -2;
        return;
    }
    Cand k;
    const bool keep = localize_one(a, lp, scan_key(o, layer, y, x), 0, k);
    layer_out[i] = keep ? (int32_t)k.layer : -1;
    pano_kp q;
    q.x = keep ? k.x : 0.0f;
    q.y = keep ? k.y : 0.0f;
    q.size = keep ? k.size : 0.0f;
    q.angle = -1.0f;
    q.response = keep ? k.response : 0.0f;
    q.octave = keep ? k.octave_field : 0;
    out[i] = q;
}

// orient_list, wave per caller keypoint (base-image coordinates, the octave's Gaussian level
// img): out[i][0 .. counts[i]) are the oriented copies in peak order, as the reference appends
// them (at most PANO_ORI_MAX_PEAKS: a peak exceeds both neighbours); counts[i] = -1 refuses a
// keypoint with a non-finite position or a window radius above 1024 px.
__global__ void __launch_bounds__(256)
orient_list(const float *__restrict__ img, int H, int W, int o, OriParams op, const pano_kp *__restrict__ kps,
            int n, pano_kp *__restrict__ out, int32_t *__restrict__ counts) {
    __shared__ unsigned long long hist[4][kOriCopies][PANO_ORI_BINS];
    __shared__ double hd[4][PANO_ORI_BINS];
    __shared__ double sm[4][PANO_ORI_BINS];
    __shared__ float patch[4][kOriPatch * kOriPatch];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int i = blockIdx.x * 4 + wv; i < n; i += gridDim.x * 4) {      // wave-uniform
        const pano_kp k = kps[i];
        // a caller keypoint whose window would be absurd (radius > 1024 px, non-finite fields)
        // is refused (count -1) instead of walking it
        const float rr = (float)op.radius_factor * ((float)(op.scale_factor * (double)k.size) / (float)(1 << (o + 1)));
        if (!(rr >= 0.0f && rr <= 1024.0f) || !isfinite(k.x) || !isfinite(k.y)) {
            if (lane == 0) counts[i] = -1;
            continue;
        }
        double angle;
        const bool emit = orient_one(img, H, W, o, k.x, k.y, k.size, op, hist[wv], hd[wv], sm[wv], patch[wv],
                                     lane, angle);
        const unsigned long long m = __ballot(emit);
        if (emit) {
            pano_kp q = k;
            q.angle = (float)angle;
            out[(size_t)i * PANO_ORI_MAX_PEAKS + __popcll(m & ((1ull << lane) - 1))] = q;
        }
        if (lane == 0) counts[i] = __popcll(m);
        wave_sync_lds();
    }
}

// ------------------------------------------------------------------ S8
__device__ __forceinline__ uint32_t sortable(float v) {
    const uint32_t b = __float_as_uint(v);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// strict "a before b" of compare_keypoints (x, y asc; size desc; angle asc; response desc),
// ties by scan order (the reference's stable sort keeps scan order)
__device__ __forceinline__ bool rec_before(const RawKp &a, const RawKp &b) {
    if (a.x != b.x) return a.x < b.x;
    if (a.y != b.y) return a.y < b.y;
    if (a.size != b.size) return a.size > b.size;
    if (a.angle != b.angle) return a.angle < b.angle;
    if (a.response != b.response) return a.response > b.response;
    return a.order < b.order;
}

// The reference's sort (compare_keypoints, stable) is a strict total order once scan order
// breaks ties, so each keypoint's sorted position is its RANK.  Ranks come from a counting
// sort on floor(x) (monotone in the primary key): bucket_count histograms the integer x of
// every raw keypoint (the atomic's return value is its slot), bucket_scan turns the counts
// into bucket starts, bucket_scatter lists each bucket's members, and bucket_rank adds to
// the bucket start the number of members that sort before the keypoint (64-bit (x, y) key,
// the full comparator on an equal key).  O(count x bucket size) instead of count^2 per
// frame: a handful of compares per keypoint (1080p: ~30k raw keypoints over 3840 buckets).
// emit_keypoints then de-duplicates neighbours and converts (one workgroup per frame).
__device__ __forceinline__ int x_bucket(float x, int nb) {
    const int b = (int)floorf(x);
    return b < 0 ? 0 : (b >= nb ? nb - 1 : b);
}

__device__ __forceinline__ unsigned long long xy_key(const RawKp &r) {
    return ((unsigned long long)sortable(r.x) << 32) | sortable(r.y);
}

// bucket_build, one workgroup per frame: floor(x) histogram in LDS (the atomic's return
// value is the keypoint's slot in its bucket), exclusive scan to bucket starts, and the
// bucket member lists -- the three passes of the counting sort with block barriers between
// them instead of kernel boundaries.
constexpr int kSortThreads = 1024;
constexpr int kSortMaxBuckets = 8192 + 1;     // base width + 1 (frames <= 4096 px)

__global__ void __launch_bounds__(kSortThreads)
bucket_build(const RawKp *__restrict__ raw, const int32_t *__restrict__ raw_cnt, int raw_cap, int nb,
             int32_t *__restrict__ bstart, int32_t *__restrict__ bslot, uint32_t *__restrict__ mem) {
    __shared__ int32_t bc[kSortMaxBuckets];
    __shared__ int32_t wsum[kSortThreads / 64];
    const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int cnt = raw_cnt[f * kCntStride];
    if (cnt > raw_cap || nb > kSortMaxBuckets) return;   // emit_keypoints reports the overflow
    const RawKp *rec = raw + (size_t)f * raw_cap;
    int32_t *slot = bslot + (size_t)f * raw_cap;
    for (int b = tid; b < nb; b += kSortThreads) bc[b] = 0;
    __syncthreads();
    for (int i = tid; i < cnt; i += kSortThreads) slot[i] = atomicAdd(&bc[x_bucket(rec[i].x, nb)], 1);
    __syncthreads();
    // exclusive scan of bc: each thread a contiguous run, wave scans of the run totals
    const int per = (nb + kSortThreads - 1) / kSortThreads, b0 = tid * per;
    int run = 0;
    for (int k = 0; k < per; ++k)
        if (b0 + k < nb) run += bc[b0 + k];
    int incl = run;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int base = incl - run;
    for (int w = 0; w < wv; ++w) base += wsum[w];
    for (int k = 0; k < per; ++k) {
        const int b = b0 + k;
        if (b >= nb) break;
        const int c = bc[b];
        bc[b] = base;
        bstart[(size_t)f * nb + b] = base;
        base += c;
    }
    __syncthreads();
    uint32_t *mb = mem + (size_t)f * raw_cap;
    for (int i = tid; i < cnt; i += kSortThreads) mb[bc[x_bucket(rec[i].x, nb)] + slot[i]] = (uint32_t)i;
}

// Rank of each keypoint = bucket start + members that sort before it.  The same loop flags a
// duplicate (remove_duplicate_keypoints :319-327 keeps the first of each run of equal (pt,
// size, angle); those four are the comparator's leading keys, so such runs are contiguous
// and a keypoint is dropped iff an equal one sorts before it): sorted[rank] = index | dup << 31.
constexpr uint32_t kDupBit = 0x80000000u;

__global__ void __launch_bounds__(256)
bucket_rank(const RawKp *__restrict__ raw, const int32_t *__restrict__ raw_cnt, int raw_cap, int nb,
            const int32_t *__restrict__ bstart, const uint32_t *__restrict__ mem,
            uint32_t *__restrict__ sorted) {
    const int f = blockIdx.x, i = blockIdx.y * 256 + threadIdx.x;   // (frame, block): see localize
    const int cnt = raw_cnt[f * kCntStride];
    if (cnt > raw_cap || i >= cnt) return;
    const RawKp *rec = raw + (size_t)f * raw_cap;
    const uint32_t *mb = mem + (size_t)f * raw_cap;
    const RawKp ri = rec[i];
    const unsigned long long ki = xy_key(ri);
    const int b = x_bucket(ri.x, nb);
    const int s = bstart[(size_t)f * nb + b];
    const int e = b + 1 < nb ? bstart[(size_t)f * nb + b + 1] : cnt;
    int r = s;
    bool dup = false;
    for (int m = s; m < e; ++m) {
        const uint32_t j = mb[m];
        if (j == (uint32_t)i) continue;
        const RawKp &rj = rec[j];
        const unsigned long long kj = xy_key(rj);
        const bool before = kj < ki || (kj == ki && rec_before(rj, ri));
        r += before;
        dup |= before && rj.x == ri.x && rj.y == ri.y && rj.size == ri.size && rj.angle == ri.angle;
    }
    if (r < cnt) sorted[(size_t)f * raw_cap + r] = (uint32_t)i | (dup ? kDupBit : 0u);
    else atomicExch(&sorted[(size_t)f * raw_cap], 0xFFFFFFFFu);   // order broken: flag
}

// De-duplicated keypoints in sorted order, converted (convert_keypoints_to_input_image_size
// :330-346), one workgroup per frame: a block scan of the keep flags over contiguous rank
// runs, then every thread writes its run's kept keypoints (index loads batched so the
// record loads of a run are in flight together).
__global__ void __launch_bounds__(kSortThreads)
emit_keypoints(const RawKp *__restrict__ raw, const int32_t *__restrict__ raw_cnt, int raw_cap,
               const uint32_t *__restrict__ sorted, pano_kp *__restrict__ out, int cap,
               int32_t *__restrict__ counts, int32_t *__restrict__ err,
               const int32_t *__restrict__ ext_cnt, int ext_cap,
               const int32_t *__restrict__ cand_cnt, int cand_cap,
               const uint8_t *__restrict__ desc_raw = nullptr, const int32_t *__restrict__ norm_raw = nullptr,
               uint8_t *__restrict__ desc_out = nullptr, int32_t *__restrict__ norm_out = nullptr,
               int32_t *__restrict__ map = nullptr) {
    __shared__ int32_t wsum[kSortThreads / 64];
    __shared__ int32_t total;
    const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const RawKp *rec = raw + (size_t)f * raw_cap;
    const uint32_t *idx = sorted + (size_t)f * raw_cap;
    const int cnt = raw_cnt[f * kCntStride];
    if (cnt > raw_cap || ext_cnt[f * kCntStride] > ext_cap || cand_cnt[f * kCntStride] > cand_cap) {
        if (tid == 0) { err[0] = PANO_E_OVERFLOW; counts[f] = -1; }
        return;
    }
    const int per = (cnt + kSortThreads - 1) / kSortThreads;
    const int beg = tid * per, end = min(beg + per, cnt);
    // every slot must hold a live index (the ranks are a permutation of 0..cnt-1)
    int bad = 0, mine = 0;
    for (int i = beg; i < end; ++i) {
        const uint32_t v = idx[i];
        bad |= (v & ~kDupBit) >= (uint32_t)cnt;
        mine += (v & kDupBit) == 0;
    }
    if (__syncthreads_or(bad)) {
        if (tid == 0) { err[0] = PANO_E_OVERFLOW; err[1] = 0x5017; counts[f] = -1; }
        return;
    }
    int incl = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int pos = incl - mine;
    for (int w = 0; w < wv; ++w) pos += wsum[w];
    if (tid == kSortThreads - 1) total = pos + mine;
    constexpr int B = 8;
    for (int i0 = beg; i0 < end; i0 += B) {
        uint32_t v[B];
        RawKp r[B];
#pragma unroll
        for (int k = 0; k < B; ++k) v[k] = i0 + k < end ? idx[i0 + k] : kDupBit;
#pragma unroll
        for (int k = 0; k < B; ++k)
            if (!(v[k] & kDupBit)) r[k] = rec[v[k]];
#pragma unroll
        for (int k = 0; k < B; ++k) {
            if (v[k] & kDupBit) continue;
            if (pos < cap) {
                pano_kp q;
                q.x = r[k].x * 0.5f;
                q.y = r[k].y * 0.5f;
                q.size = r[k].size * 0.5f;
                q.angle = r[k].angle;
                q.response = r[k].response;
                q.octave = (r[k].octave & ~255) | ((r[k].octave - 1) & 255);
                out[(size_t)f * cap + pos] = q;
                if (desc_raw) map[(size_t)f * raw_cap + pos] = (int32_t)v[k];
            }
            ++pos;
        }
    }
    __syncthreads();
    if (tid == 0) {
        counts[f] = total;                       // the true count, even above cap
        if (total > cap) err[0] = PANO_E_OVERFLOW;   // keypoints past cap were dropped
    }
    if (desc_raw) {
        // descriptors computed in raw order (descriptor_wave<.., RAW>): rows to sorted order,
        // 8 lanes x 16 bytes per row
        const int m = min(total, cap);
        const int32_t *mp = map + (size_t)f * raw_cap;
        for (int e = tid; e < m * 8; e += kSortThreads) {
            const int kq = e >> 3, part = e & 7;
            const int src = mp[kq];
            const uint4 v = *(const uint4 *)(desc_raw + ((size_t)f * raw_cap + src) * PANO_DESC_DIM + 16 * part);
            *(uint4 *)(desc_out + ((size_t)f * cap + kq) * PANO_DESC_DIM + 16 * part) = v;
            if (part == 0) norm_out[(size_t)f * cap + kq] = norm_raw[(size_t)f * raw_cap + src];
        }
    }
}

// ------------------------------------------------------------------ S9
// OpenBLAS 0.3.29 SkylakeX sdot order (oracle/numerics.py::sdot_skx), one thread.
__device__ float sdot_skx(const float *x, int n) {
    const int n64 = n & ~63, n32 = n & ~31;
    float a16[4][16];
    for (int k = 0; k < 4; ++k)
        for (int j = 0; j < 16; ++j) a16[k][j] = 0.0f;
    for (int i = 0; i < n64; i += 64)
        for (int k = 0; k < 4; ++k)
            for (int j = 0; j < 16; ++j) {
                const float t = x[i + 16 * k + j];
                a16[k][j] = fmaf(t, t, a16[k][j]);
            }
    float a8[4][8];
    for (int k = 0; k < 4; ++k)
        for (int j = 0; j < 8; ++j) a8[k][j] = a16[k][j] + a16[k][j + 8];
    for (int i = n64; i < n32; i += 32)
        for (int k = 0; k < 4; ++k)
            for (int j = 0; j < 8; ++j) {
                const float t = x[i + 8 * k + j];
                a8[k][j] = fmaf(t, t, a8[k][j]);
            }
    float v[8];
    for (int j = 0; j < 8; ++j) v[j] = ((a8[0][j] + a8[1][j]) + a8[2][j]) + a8[3][j];
    float h[4];
    for (int j = 0; j < 4; ++j) h[j] = v[j] + v[j + 4];
    const float kern = (h[0] + h[1]) + (h[2] + h[3]);
    double tail = 0.0;
    for (int j = n32; j < n; ++j) tail += (double)(x[j] * x[j]);
    return (float)((double)kern + tail);
}

struct DescParams {
    float hw_mult;     // f32(scale_multiplier * 0.5)
    float max_value;   // f32(descriptor_max_value)
};

// Wave-level restatement of sdot_skx(x, 128) (OpenBLAS SkylakeX order): lane L holds
// x[L] and x[64 + L]; returns the same float on every lane.
__device__ __forceinline__ float sdot_skx_wave128(float lo, float hi) {
    const int lane = threadIdx.x & 63;
    const float a16 = fmaf(hi, hi, fmaf(lo, lo, 0.0f));              // a16[k][j], L = 16k + j
    const float a8 = a16 + __shfl(a16, (lane & ~15) | ((lane + 8) & 15));   // valid for j < 8
    // v[j] = ((a8[0][j] + a8[1][j]) + a8[2][j]) + a8[3][j], j < 8 (a8[k][j] at lane 16k + j)
    const int j = lane & 7;
    const float v = ((__shfl(a8, j) + __shfl(a8, 16 + j)) + __shfl(a8, 32 + j)) + __shfl(a8, 48 + j);
    const float h = v + __shfl(v, (j + 4) & 7);                      // h[j] = v[j] + v[j + 4], j < 4
    const float kern = (__shfl(h, 0) + __shfl(h, 1)) + (__shfl(h, 2) + __shfl(h, 3));
    return (float)((double)kern + 0.0);
}

// Descriptors, one WAVE per keypoint, persistent: waves stride over the keypoints of the
// whole batch (no workgroups for empty capacity slots).  Per keypoint the wave derives, per
// patch column, the row interval inside the rotated square and the image (conservative; the
// exact bin test is per sample), merges them over SUPER-STRIPS of kDescGrp x kDescSW
// adjacent columns (union interval), scans their lengths into a dense (super-strip, row)
// index, and each group of kDescGrp adjacent lanes walks its own run of that index, lane
// `sub` of the group taking strip `sub` (kDescSW columns) of each super-strip row.  The
// gradient taps come from a sliding window of three image rows x (kDescSW + 2) columns: ONE
// wide load per step serves the strip's kDescSW samples, the next step's load in flight while
// the current samples are binned, and a group's loads of one step fall in ~one cache line.
// 4 samples per load instead of 1 cut it 0.35 -> 0.25 ms at parrington; since then the
// per-sample binning, not the loads, bounds it (L1-resident taps: -8 %, no LDS: -2 %).  Groups are Q steps apart: different cells /
// orientations, few same-address LDS atomics.  Each sample is
// spread trilinearly into the wave's 6 x 6 x 8 histogram (padding bins included: no bounds
// branches) as 2^22 fixed-point u64 LDS atomics, into one of kDescCopies interleaved copies
// (copy = lane % kDescCopies >= kDescGrp, so a group's lanes never share an address; summed at
// the end) -- integer sums, deterministic and order
// independent (LDS f32 atomics measured 5x slower on gfx950).  The normalisation is the
// reference's, np.linalg.norm in OpenBLAS's sdot order across the lanes.
//
// Arithmetic (generate_descriptors :361-526): every per-sample quantity is f32.  Everything
// the reference computes in float64 (rotation, bins, weights) enters only through continuous
// trilinear weights: a sample moving across a bin edge hands its weight over continuously, so
// f32 rounding moves each contribution by ~1e-7 relative -- the size of the reference's own
// float32 np.add.at accumulation (measured on the parrington goldens: 6e-6 of the integer
// elements 1 LSB off, vs 2e-6 for an exact-sum form; the bar is 1e-3).
//
// OUT_U8: the Stitcher's form -- integer descriptors as bytes [n][cap][128] plus their
// squared norms (exact integers) [n][cap], what the distance GEMM consumes; otherwise the
// drop-in form, f32 [n][cap][128].
constexpr int kDescWaves = 4;         // waves (keypoints in flight) per workgroup
constexpr int kDescCols = 128;        // patch sides up to this use the dense index (default
                                      // parameters: side <= 73)
#ifndef PANO_DESC_CELL
#define PANO_DESC_CELL 8              // u64 slots per spatial cell (8 orientation bins [+ padding])
#endif
// cell stride: with 8 slots a cell's bin b sits in LDS bank pair (16 cell + 2 b) mod 32, so only
// the cell's parity separates two lanes' cells; a stride of 9 shifts every cell by 18 banks
constexpr int kCell = PANO_DESC_CELL, kRowC = 6 * kCell;
constexpr int kHist = 6 * kRowC;      // padded histogram (reference: tensor of (ww+2, ww+2, nb))
#ifndef PANO_DESC_SKEW
#define PANO_DESC_SKEW 2              // u64 slots between histogram copies beyond kHist
#endif
// copy stride: kHist u64 is 576 dwords, a multiple of the 32 banks an LDS atomic's lane group
// spreads over, so without the skew the copies alias bank for bank and the two lanes of a
// pair (same row, adjacent strips: often the same bin) collide on a bank at different addresses
constexpr int kHistStride = kHist + PANO_DESC_SKEW;
constexpr float kFix = 4194304.0f;    // 2^22: contributions <= 255 sqrt(2) fit a u32
#ifndef PANO_DESC_SW
#define PANO_DESC_SW 4                // patch columns per strip: one (SW + 2)-float load per step
#endif
constexpr int kDescSW = PANO_DESC_SW;
#ifndef PANO_DESC_NS_PREFETCH
#define PANO_DESC_NS_PREFETCH 0       // 1: a strip change's rows loaded a step ahead (12 more VGPRs)
#endif
#ifndef PANO_DESC_COPIES
#define PANO_DESC_COPIES 2            // histogram copies per wave (copy = lane % copies)
#endif
#ifndef PANO_DESC_GRP
#define PANO_DESC_GRP 2               // lanes walking one row of kDescGrp adjacent strips together
#endif
constexpr int kDescGrp = PANO_DESC_GRP;
constexpr int kDescSS = kDescSW * kDescGrp;   // columns of a group's super-strip
// copy = lane % copies: the two lanes of a pair (default) bin into different copies, so they
// issue no same-address atomics (wider groups share copies: measured, the LDS is hidden)
constexpr int kDescCopies = PANO_DESC_COPIES;
static_assert(kDescSS <= 64 && (kDescGrp & (kDescGrp - 1)) == 0, "super-strip divides 64");

static_assert(kDescSW == 1 || kDescSW == 2 || kDescSW == 4 || kDescSW == 8, "strip width divides 64");
#ifndef PANO_DESC_RPI
#define PANO_DESC_RPI 1               // fixed-point scale folded into the sample weight (fewer VALU)
#endif
#ifndef PANO_DESC_UNROLL
#define PANO_DESC_UNROLL 0            // 1: the walk step unrolled 4x over rotating row buffers
#endif
#ifndef PANO_DESC_RING
#define PANO_DESC_RING 0              // > 0: tap rows prefetched this many steps ahead via LDS-DMA
#endif
#if PANO_DESC_RING
constexpr int kRing = PANO_DESC_RING;
#endif
#ifndef PANO_DESC_ROWS
#define PANO_DESC_ROWS 0              // 1: row-major walk over (row, strip) items (measured slower)
#endif
#ifndef PANO_DESC_PK
#define PANO_DESC_PK 0                // 1: the trilinear products as packed f32 pairs (measured slower)
#endif
#ifndef PANO_DESC_COMPACT
#define PANO_DESC_COMPACT 0           // 1: samples binned from a compaction queue, 64 at a time (measured slower)
#endif
#if PANO_DESC_COMPACT
constexpr int kDescQ = 128;           // queue entries per wave: <= 63 waiting + 64 appended
#endif
#ifndef PANO_DESC_RLANES
#define PANO_DESC_RLANES 8            // row walk: consecutive lanes on consecutive items
#endif
#if PANO_DESC_ROWS
constexpr int kRowLanes = PANO_DESC_RLANES;
constexpr int kRowTbl = 1920;         // row walk items per keypoint (u16 each; more: the square)
#endif
#ifndef PANO_DESC_ABL
#define PANO_DESC_ABL 0               // timing ablations only (1: plain LDS stores, 2: no LDS,
                                      // 3: every sample's taps from one cached location)
#endif

#ifndef PANO_DESC_ABL_TRIG
#define PANO_DESC_ABL_TRIG 0
#endif
#ifndef PANO_DESC_CLAIM
#define PANO_DESC_CLAIM 1             // keypoints claimed per atomic (per-XCD work counter)
#endif
constexpr int kDescClaim = PANO_DESC_CLAIM;
#ifndef PANO_DESC_ABL_NOCOL
#define PANO_DESC_ABL_NOCOL 0         // timing ablation: no per-column row intervals
#endif
#ifndef PANO_DESC_ABL_NOEPI
#define PANO_DESC_ABL_NOEPI 0         // timing ablation: no clamp / norm epilogue
#endif
#ifndef PANO_DESC_ABL_NOWALK
#define PANO_DESC_ABL_NOWALK 0        // timing ablation: no sample walk (setup, intervals, epilogue only)
#endif
#ifndef PANO_DESC_COUNT
#define PANO_DESC_COUNT 0             // 1: diagnostics build, lane-occupancy counters of the walk
#endif
#if PANO_DESC_COUNT
// [0] candidate lane-samples, [1] passing, [2] sample blocks executed (any lane passing),
// [3] walk steps (wave-level), [4] active lanes summed over steps, [5] keypoints
__device__ unsigned long long g_desc_cnt[8];
extern "C" int pano_dbg_desc_count(unsigned long long *out, int reset) {
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        return hipMemcpyToSymbol(HIP_SYMBOL(g_desc_cnt), z, sizeof(z)) == hipSuccess ? 0 : -1;
    }
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_desc_cnt), sizeof(g_desc_cnt)) == hipSuccess ? 0 : -1;
}
#endif

// Frame of dense keypoint index gk (frames' keypoints back to back, counts clamped to
// [0, cap]): chunked wave scan of the counts; false when gk is past the last keypoint.
__device__ __forceinline__ bool locate_keypoint(const int32_t *__restrict__ counts, int n_frames,
                                                int cap, int gk, int &f, int &k) {
    const int lane = threadIdx.x & 63;
    int base = 0;
    for (int f0 = 0; f0 < n_frames; f0 += 64) {
        int c = f0 + lane < n_frames ? counts[f0 + lane] : 0;
        c = c < 0 ? 0 : (c < cap ? c : cap);
        int incl = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int t = __shfl_up(incl, d);
            if (lane >= d) incl += t;
        }
        const int tot = __shfl(incl, 63);
        if (gk < base + tot) {
            const int j = __popcll(__ballot(base + incl <= gk));   // frames wholly before gk
            f = f0 + j;
            k = gk - base - (__shfl(incl, j) - __shfl(c, j));
            return true;
        }
        base += tot;
    }
    return false;
}

#ifndef PANO_DESC_TIMING
#define PANO_DESC_TIMING 0     // 1: diagnostics build, per-wave clocks of descriptor_wave (tools/desc_clock.py)
#endif
#if PANO_DESC_TIMING
constexpr int kDescClkWaves = 16384;
__device__ unsigned long long g_desc_clk[kDescClkWaves][4];
extern "C" int pano_dbg_desc_clock(unsigned long long *out, int reset) {
    if (reset) {
        void *p = nullptr;
        if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_desc_clk)) != hipSuccess) return -1;
        return hipMemset(p, 0, sizeof(g_desc_clk)) == hipSuccess ? 0 : -1;
    }
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_desc_clk), sizeof(g_desc_clk)) == hipSuccess ? 0 : -1;
}
#endif

// OCC: waves per SIMD the register budget is sized for.  With a strip change's rows loaded
// when reached (PANO_DESC_NS_PREFETCH=0, 12 VGPRs fewer) the 4-wave budget spills 5 registers
// instead of 13, and measures best at both sizes (same box, feature-stage timing): parrington
// 0.222 ms at 4 against 0.238 at 3 and 0.241 at 5; 1080p 2.86 ms against 3.10 and 2.99.  The
// 3-wave build stays for the A/B (PANO_DESC_OCC=3, read per call).
static int desc_occ(long long) {
    const char *e = getenv("PANO_DESC_OCC");
    if (e && e[0] == '3' && !e[1]) return 3;
    return 4;
}

// RAW: the keypoints are orientation's raw records (RawKp [n][cap], counts strided by
// kCntStride), converted on load exactly as emit_keypoints converts them; the descriptors go
// to raw order and emit_keypoints permutes them (the sort runs beside this kernel).
template <bool OUT_U8, int OCC, bool RAW = false>
__global__ void __launch_bounds__(64 * kDescWaves, OCC)
descriptor_wave(PyrArgs pa, DescParams dp, const pano_kp *__restrict__ kps,
                const int32_t *__restrict__ counts, int n_frames, int cap, int32_t *__restrict__ work,
                float *__restrict__ desc, uint8_t *__restrict__ desc_u8, int32_t *__restrict__ norms,
                const int32_t *__restrict__ order, const RawKp *__restrict__ rawk = nullptr) {
    constexpr int cstride = RAW ? kCntStride : 1;
    __shared__ unsigned long long hist[kDescWaves][kDescCopies * kHistStride];
    __shared__ int col_lo[kDescWaves][kDescCols / kDescSS], col_pre[kDescWaves][kDescCols / kDescSS + 1];   // per super-strip
    // column constants, 4 padding entries each side (rejecting values) for the row walk's
    // memory-aligned strips, which can start up to 3 columns before the patch or end after it
    __shared__ float col_br[kDescWaves][kDescCols + 8], col_bc[kDescWaves][kDescCols + 8];
#if PANO_DESC_ROWS
    __shared__ uint16_t row_tbl[kDescWaves][kRowTbl];   // row walk: (patch row, strip) per item
#endif
#if PANO_DESC_COMPACT
    // per-wave ring of candidate samples that passed the bin test (compaction queue)
    __shared__ float2 cq_g[kDescWaves][kDescQ], cq_b[kDescWaves][kDescQ];
    __shared__ float cq_w[kDescWaves][kDescQ];
#endif
#if PANO_DESC_RING
    __shared__ __attribute__((aligned(16))) float ring[kDescWaves][PANO_DESC_RING][2][64 * 4];   // LDS-DMA tap rows, per wave
#endif
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    unsigned long long *h0 = hist[wv];
    unsigned long long *h = h0 + (lane & (kDescCopies - 1)) * kHistStride;   // this lane's copy
    int *clo = col_lo[wv], *cpre = col_pre[wv];
    float *cbr = col_br[wv] + 4, *cbc = col_bc[wv] + 4;
    if (lane < 8) {                      // the padding: never written below, rejects every sample
        const int c = lane < 4 ? lane - 4 : kDescCols + lane - 4;
        cbr[c] = 1e30f;
        cbc[c] = 1e30f;
    }
    // XCD-aware split (workgroup b runs on XCD b % 8): each XCD takes one contiguous eighth of
    // the keypoints (x-sorted per frame: neighbouring windows), its waves striding over it, so
    // a window's pyramid rows are fetched into one XCD's L2, not eight
    int total = 0;
    for (int f0 = 0; f0 < n_frames; f0 += 64) {
        int c = f0 + lane < n_frames ? counts[(f0 + lane) * cstride] : 0;
        c = c < 0 ? 0 : (c < cap ? c : cap);
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d);
        total += c;
    }
    const int xcd = blockIdx.x & 7, nx = gridDim.x >> 3;           // gridDim.x % 8 == 0
    const int lo_k = (int)((long long)total * xcd / 8), hi_k = (int)((long long)total * (xcd + 1) / 8);
    // dynamic: a wave takes the XCD's next keypoint from the XCD's own counter (window sizes
    // vary ~3x; static striding left waves idle); one 128-byte line per counter
    int32_t *wq = work + xcd * kCntStride;
    unsigned long long abl_sink = 0;
    (void)nx;
    int f = 0, k = 0;
    FrameIndex fi;
    fi.init(counts, cstride, n_frames, cap);
    int claim = 0;
    int cl_next = 0, cl_end = 0;                 // wave-uniform: claimed keypoints [cl_next, cl_end)
    bool pre = false;                            // wave-uniform: a claim is in flight in lane 0's claim
    // every wave's first chunk without an atomic (as orientation)
    const int wx = (int)(gridDim.x >> 3) * kDescWaves, nw_x = kClaimStatic ? wx : 0;
    if (kClaimStatic) {
        cl_next = ((int)(blockIdx.x >> 3) * kDescWaves + wv) * kDescClaim;
        cl_end = cl_next + kDescClaim;
    }
#if PANO_DESC_TIMING
    const unsigned long long t_entry = (unsigned long long)__builtin_amdgcn_s_memrealtime();
    int nkp = 0;
#endif
    if (kClaimAhead && lane == 0) claim = atomicAdd(wq, 1);
    for (;;) {
        int gk;
        if constexpr (kClaimAhead) {
            gk = lo_k + __shfl(claim, 0);
            if (gk >= hi_k) break;
            if (lane == 0) claim = atomicAdd(wq, 1);
        } else {
            // kDescClaim keypoints per atomic: the XCD's counter serialises its waves' claims
            // (the per-keypoint phase alone, no sample walk, took 76 us at parrington whatever
            // its arithmetic -- the claims, not the work)
            if (cl_next >= cl_end) {
                if (!pre && lane == 0) claim = atomicAdd(wq, kDescClaim);
                cl_next = nw_x * kDescClaim + __shfl(claim, 0);
                cl_end = cl_next + kDescClaim;
                pre = false;
            }
            gk = lo_k + cl_next++;
            if (gk >= hi_k) break;
            if (kClaimFar && cl_next >= cl_end && gk + kClaimFar * wx * kDescClaim < hi_k) {
                if (lane == 0) claim = atomicAdd(wq, kDescClaim);   // next claim in flight
                pre = true;
            }
        }
        if (fi.regs) fi.locate(gk, f, k);
        else if (RAW ? !locate_strided(counts, n_frames, cap, gk, f, k) : !locate_keypoint(counts, n_frames, cap, gk, f, k))
            break;
        if (order) k = order[(size_t)f * cap + k];     // locality order (desc_order)
#if PANO_DESC_COUNT
        if (lane == 0) atomicAdd(&g_desc_cnt[5], 1ull);
#endif
        for (int i = lane; i < kDescCopies * kHistStride; i += 64) h0[i] = 0ull;
        pano_kp kp;
        if constexpr (RAW) {                           // emit_keypoints' conversion, exactly
            const RawKp r = rawk[(size_t)f * cap + k];
            kp.x = r.x * 0.5f;
            kp.y = r.y * 0.5f;
            kp.size = r.size * 0.5f;
            kp.angle = r.angle;
            kp.response = r.response;
            kp.octave = (r.octave & ~255) | ((r.octave - 1) & 255);
        } else {
            kp = kps[(size_t)f * cap + k];
        }
        int oct = kp.octave & 255;
        if (oct >= 128) oct |= -128;
        const int lyr = (kp.octave >> 8) & 255;
        const float scl = oct >= 0 ? 1.0f / (float)(1 << oct) : (float)(1 << -oct);
        const int O = oct + 1;
        const size_t row = (size_t)f * cap + k;
        if (O < 0 || O >= pa.n_oct || lyr >= pa.n_lvl) {
            // a caller keypoint (pano_sift_describe) whose octave / layer is outside the pyramid:
            // zero descriptor (the Python boundary rejects these before the call)
            if constexpr (OUT_U8) {
                desc_u8[row * PANO_DESC_DIM + lane] = 0;
                desc_u8[row * PANO_DESC_DIM + 64 + lane] = 0;
                if (lane == 0) norms[row] = 0;
            } else {
                desc[row * PANO_DESC_DIM + lane] = 0.0f;
                desc[row * PANO_DESC_DIM + 64 + lane] = 0.0f;
            }
            continue;
        }
        const int rows = pa.H[O], cols = pa.W[O];
        const float *img = pa.gauss[O][lyr] + (size_t)f * rows * cols;
        const int px = (int)rint((double)scl * (double)kp.x);
        const int py = (int)rint((double)scl * (double)kp.y);
        const double angle = 360.0 - (double)kp.angle;
        const double rad = angle * (3.141592653589793 / 180.0);
#if PANO_DESC_ABL_TRIG                         // timing ablation: f32 hardware sin / cos
        const double cos_a = (double)__cosf((float)rad), sin_a = (double)__sinf((float)rad);
#else
        const double cos_a = cos(rad), sin_a = sin(rad);
#endif
        const float hw = (dp.hw_mult * scl) * kp.size;
        const double hwd = (double)hw, inv_hw = 1.0 / hwd;
        int half = (int)rint(hwd * 1.4142135623730951 * 5.0 * 0.5);
        const int diag = (int)sqrt((double)(rows * rows + cols * cols));
        half = half < diag ? half : diag;
        const int side = 2 * half + 1;
        // ob = remainder((ori - angle) * 8 / 360, 8): one bin is one octant (45 deg), so with
        // the gradient angle in octants ob = ori8 - angle * 8 / 360 (mod 8)
        const float a8 = (float)(angle * (8.0 / 360.0));
        // rbin = ys (cos / hw) + (xs sin / hw + 1.5), cbin = ys (-sin / hw) + (xs cos / hw + 1.5)
        const double sr = sin_a * inv_hw, cr = cos_a * inv_hw;
        const float ar = (float)cr, ac = (float)-sr;
        auto sample_in = [&](float gx, float gy, float rbin, float cbin, float w) {
            const float mag = __builtin_amdgcn_sqrtf(gx * gx + gy * gy);
            float ob = atan2_oct(gy, gx) - a8;               // (-12, 4]
            ob = ob < 0.0f ? ob + 8.0f : ob;
            ob = ob < 0.0f ? ob + 8.0f : ob;
#if PANO_DESC_RPI
            // scaled to the 2^22 fixed point up front (a power of two: every product below is
            // exactly 2^22 times its unscaled value), so each contribution is one multiply and
            // one round-half-up conversion, v_cvt_rpi_i32_f32 = floor(x + 0.5).  Against the
            // unscaled form's u32(fma(v, 2^22, 0.5)) the exhaustive device probe over every f32
            // x in [0, 2^31) (tools/probes/rpi_check.hip, profiles/r05_rpi_check.txt) finds
            // 4,194,305 inputs that differ, all by one unit of 2^-22: the odd integers of
            // [2^23, 2^24), where the fma's RN(x + 0.5) ties to even and rounds up, and x = 0.5,
            // which the instruction takes to 0.  Either is a 1e-7-relative restatement of the
            // reference's float32 np.add.at; the descriptor bytes of every fixture are unchanged
            const float wm = (w * mag) * kFix;
#else
            const float wm = w * mag;
#endif
            const float fr = floorf(rbin), fc = floorf(cbin), fo = floorf(ob);
            const float rf = rbin - fr, cf = cbin - fc;
            // (the reference's o0 = floor(ob) % 8, of = ob - o0 gives of = 8 when np.mod rounds a
            // tiny negative offset to 8.0; numpy's SIMD f32 arctan2 / rad2deg decide that case at
            // the ulp level, which no other arithmetic reproduces: here of = ob - floor(ob), the
            // continuous form -- DESIGN.md 4, "descriptor outliers")
            const int o0 = (int)fo & 7, o1 = (o0 + 1) & 7;
#if PANO_DESC_RPI
            // (r0 + 1, c0 + 1) bin from the integer-valued floors (exact in f32): one conversion
            const int base = (int)fmaf(fr, (float)kRowC, fmaf(fc, (float)kCell, (float)(kRowC + kCell)));
#else
            const int base = ((int)fr + 1) * kRowC + ((int)fc + 1) * kCell;   // (r0 + 1, c0 + 1) bin
#endif
            const float c1 = wm * rf, c0w = wm - c1;
#if PANO_DESC_PK
            typedef float f2v __attribute__((ext_vector_type(2)));
            const f2v cfv = {1.0f - cf, cf};
            const f2v vt = (f2v){c0w, c0w} * cfv, vb = (f2v){c1, c1} * cfv;
            const float v00 = vt.x, v01 = vt.y, v10 = vb.x, v11 = vb.y;
#else
            const float v00 = c0w * (1.0f - cf), v01 = c0w * cf, v10 = c1 * (1.0f - cf), v11 = c1 * cf;
#endif
            const float of = ob - fo;
            const float nof = 1.0f - of;
#if PANO_DESC_RPI
            auto fix = [](float v) {
                int r;
                asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(v));
                return (unsigned long long)(uint32_t)r;
            };
#else
            auto fix = [](float v) { return (unsigned long long)(uint32_t)fmaf(v, kFix, 0.5f); };
#endif
            unsigned long long *hA = h + base + o0, *hB = h + base + o1;
#if PANO_DESC_ABL == 0 && PANO_DESC_PK
            // the same eight f32 products as below, as v_pk_mul_f32 pairs (identical roundings)
            typedef float f2 __attribute__((ext_vector_type(2)));
            const f2 ov = {nof, of};
            const f2 p00 = (f2){v00, v00} * ov, p01 = (f2){v01, v01} * ov;
            const f2 p10 = (f2){v10, v10} * ov, p11 = (f2){v11, v11} * ov;
            atomicAdd(hA, fix(p00.x));      atomicAdd(hB, fix(p00.y));
            atomicAdd(hA + kCell, fix(p01.x));  atomicAdd(hB + kCell, fix(p01.y));
            atomicAdd(hA + kRowC, fix(p10.x)); atomicAdd(hB + kRowC, fix(p10.y));
            atomicAdd(hA + kRowC + kCell, fix(p11.x)); atomicAdd(hB + kRowC + kCell, fix(p11.y));
#elif PANO_DESC_ABL == 0
            atomicAdd(hA, fix(v00 * nof));      atomicAdd(hB, fix(v00 * of));
            atomicAdd(hA + kCell, fix(v01 * nof));  atomicAdd(hB + kCell, fix(v01 * of));
            atomicAdd(hA + kRowC, fix(v10 * nof)); atomicAdd(hB + kRowC, fix(v10 * of));
            atomicAdd(hA + kRowC + kCell, fix(v11 * nof)); atomicAdd(hB + kRowC + kCell, fix(v11 * of));
#elif PANO_DESC_ABL == 1
            hA[0] = fix(v00 * nof);  hB[0] = fix(v00 * of);
            hA[kCell] = fix(v01 * nof);  hB[kCell] = fix(v01 * of);
            hA[kRowC] = fix(v10 * nof); hB[kRowC] = fix(v10 * of);
            hA[kRowC + kCell] = fix(v11 * nof); hB[kRowC + kCell] = fix(v11 * of);
#else
            abl_sink += fix(v00 * nof) + fix(v00 * of) + fix(v01 * nof) + fix(v01 * of) + fix(v10 * nof) +
                        fix(v10 * of) + fix(v11 * nof) + fix(v11 * of) + (unsigned long long)(base + o0 + o1);
#endif
        };
        auto sample = [&](float gx, float gy, float rbin, float cbin, float w) {
            if (!(rbin > -1.0f && rbin < 4.0f && cbin > -1.0f && cbin < 4.0f)) return;
            sample_in(gx, gy, rbin, cbin, w);
        };
        // very large patches (non-default parameters), or more row-walk items than its table:
        // every sample of the square
        auto square_walk = [&]() {
            const int S = side * side;
            for (int j = lane; j < S; j += 64) {
                const int xi = j / side, yi = j - (j / side) * side;
                const int xs = xi - half, ys = yi - half;
                const int rr = py + ys, cc = px + xs;
                if (!(rr > 0 && rr < rows - 1 && cc > 0 && cc < cols - 1)) continue;
                const double rq = ((double)xs * sin_a + (double)ys * cos_a) * inv_hw;
                const double cq = ((double)xs * cos_a - (double)ys * sin_a) * inv_hw;
                if (!(fabs(rq) < 2.5 + 1e-6 && fabs(cq) < 2.5 + 1e-6)) continue;
                const float *q = img + (size_t)rr * cols + cc;
                sample(q[1] - q[-1], q[-cols] - q[cols], (float)rq + 1.5f, (float)cq + 1.5f,
                       (float)exp(-0.125 * (rq * rq + cq * cq)));
            }
        };
        if (side <= kDescCols) {
            const double lim = 2.5 * hwd * (1.0 + 1e-9) + 1e-9;   // |rot| / hw < 2.5 with slack
            // |a ys + b| < lim -> ys in an interval (rrot: a = cos, b = xs sin; crot: a = -sin,
            // b = xs cos); conservative: widened by 1e-6, so approximate quotients are fine
            const double ia_r = fabs(cos_a) < 1e-12 ? 0.0 : 1.0 / cos_a;
            const double ia_c = fabs(sin_a) < 1e-12 ? 0.0 : -1.0 / sin_a;
            const float kq = (float)(-0.125 * 1.4426950408889634 * inv_hw * inv_hw);
            constexpr int kEmpty = 1 << 20;
            int run = 0;                                   // wave-wide running total
            for (int c4 = 0; c4 < (PANO_DESC_ABL_NOCOL ? 0 : side); c4 += 64) {
                const int c = c4 + lane;
                int lo = kEmpty, hi = -kEmpty;
                // a column outside the patch or the image gets a bin base no sample passes
                // (rbin >= 4): its strip-mates' rows are walked, its own samples rejected
                float brc = 1e30f, bcc = 1e30f;
                if (c < side) {
                    const int xs = c - half, cc = px + xs;
                    if (cc > 0 && cc < cols - 1) {
                        brc = (float)((double)xs * sr) + 1.5f;
                        bcc = (float)((double)xs * cr) + 1.5f;
                        lo = max(-half, 1 - py);
                        hi = min(half, rows - 2 - py);
                        const double bvs[2] = {xs * sin_a, xs * cos_a};
                        const double ias[2] = {ia_r, ia_c};
#pragma unroll
                        for (int qd = 0; qd < 2; ++qd) {
                            const double bv = bvs[qd], ia = ias[qd];
                            if (ia == 0.0) {
                                if (!(fabs(bv) < lim)) hi = lo - 1;
                                continue;
                            }
                            const double t1 = (-lim - bv) * ia, t2 = (lim - bv) * ia;
                            const double l = fmax(fmin(t1, t2) - 1e-6, -half - 1.0);
                            const double u = fmin(fmax(t1, t2) + 1e-6, half + 1.0);
                            lo = max(lo, (int)ceil(l));
                            hi = min(hi, (int)floor(u));
                        }
                        if (hi < lo) { lo = kEmpty; hi = -kEmpty; }
                    }
                }
                cbr[c] = brc;
                cbc[c] = bcc;
                // super-strip = kDescSS adjacent columns: the union of their row intervals
                // (the exact bin test per sample rejects the extra rows)
#pragma unroll
                for (int d = 1; d < kDescSS; d <<= 1) {
                    lo = min(lo, __shfl_xor(lo, d));
                    hi = max(hi, __shfl_xor(hi, d));
                }
                const bool lead = (lane & (kDescSS - 1)) == 0;
                const int n_s = lead && hi >= lo ? hi - lo + 1 : 0;
                int incl = n_s;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const int t = __shfl_up(incl, d);
                    if (lane >= d) incl += t;
                }
                if (lead && c < side) {
                    clo[c / kDescSS] = lo;
                    cpre[c / kDescSS] = run + incl - n_s;
                }
                run += __shfl(incl, 63);
            }
            const int nstrip = (side + kDescSS - 1) / kDescSS;
            if (lane == 0) cpre[nstrip] = run;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#if PANO_DESC_ROWS
            // Row walk.  The column walk below hands each lane group a run of one strip's rows:
            // the 64 lanes of a load touch 64 rows, and the four strips that share a 128-byte
            // line reach it at different times, each fetch an L1 miss (timing ablations: with
            // the same rows but the wave's lanes in one 64-column span of each, 0.085 against
            // 0.220 ms at parrington).  Here the window's (row, strip) items are numbered row
            // by row -- per row the exact column interval of the rotated square, strips of 4
            // columns aligned to the image's 4-column grid -- and lane l takes items l, l + 64,
            // ...: one load instruction covers ~5 consecutive rows, each row's strips side by
            // side, and the rows above / below were fetched by the neighbouring lanes.  Same
            // samples and arithmetic as the column walk (integer histogram: bit-identical).
            bool rows_done = false;
            {
                const int ylo = max(-half, 1 - py), yhi = min(half, rows - 2 - py);
                const int xlo = max(-half, 1 - px), xhi = min(half, cols - 2 - px);
                // per row ys: rrot = xs sin + ys cos, crot = xs cos - ys sin
                const double ib_r = fabs(sin_a) < 1e-12 ? 0.0 : 1.0 / sin_a;
                const double ib_c = fabs(cos_a) < 1e-12 ? 0.0 : 1.0 / cos_a;
                uint16_t *tb = row_tbl[wv];
                if (lane < 4) {                    // a strip may end up to 3 columns past the patch
                    cbr[side + lane] = 1e30f;
                    cbc[side + lane] = 1e30f;
                }
                int rrun = 0;
                for (int r4 = 0; r4 < side; r4 += 64) {
                    const int r = r4 + lane, ys = r - half;
                    int klo = 0, n = 0;
                    if (r < side && ys >= ylo && ys <= yhi && xlo <= xhi) {
                        int lo = xlo, hi = xhi;
                        const double bvs[2] = {ys * cos_a, -ys * sin_a};
                        const double ias[2] = {ib_r, ib_c};
#pragma unroll
                        for (int qd = 0; qd < 2; ++qd) {
                            const double bv = bvs[qd], ia = ias[qd];
                            if (ia == 0.0) {
                                if (!(fabs(bv) < lim)) hi = lo - 1;
                                continue;
                            }
                            const double t1 = (-lim - bv) * ia, t2 = (lim - bv) * ia;
                            const double l = fmax(fmin(t1, t2) - 1e-6, -half - 1.0);
                            const double u = fmin(fmax(t1, t2) + 1e-6, half + 1.0);
                            lo = max(lo, (int)ceil(l));
                            hi = min(hi, (int)floor(u));
                        }
                        if (hi >= lo) {                    // image columns px + lo .. px + hi
                            klo = (px + lo) >> 2;
                            n = ((px + hi) >> 2) - klo + 1;
                        }
                    }
                    int incl = n;
#pragma unroll
                    for (int d = 1; d < 64; d <<= 1) {
                        const int tt = __shfl_up(incl, d);
                        if (lane >= d) incl += tt;
                    }
                    const int b0 = rrun + incl - n;
                    if (b0 + n <= kRowTbl)
                        for (int k2 = 0; k2 < n; ++k2) tb[b0 + k2] = (uint16_t)((r << 8) | (klo + k2 - ((px - half) >> 2) + 1));
                    rrun += __shfl(incl, 63);
                }
                if (rrun <= kRowTbl) {
                    rows_done = true;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    // strip k (stored relative to the patch's first strip, + 1 so it stays >= 0)
                    // covers image columns 4k .. 4k + 3: taps 4k - 1 .. 4k + 4 of the row, 4k .. 4k + 3
                    // of the rows above and below; 16-byte loads when rows start 16-byte aligned
                    const int kb = ((px - half) >> 2) - 1;
                    const bool al = ((cols & 3) == 0) && (((uintptr_t)img & 15) == 0);
                    struct Taps { float m[4], c[6], p[4]; };
                    auto fetch = [&](int t, Taps &T, int &ys, int &k) {
                        const unsigned e = tb[t];
                        ys = (int)(e >> 8) - half;
                        k = kb + (int)(e & 255);
                        const float *q = img + (size_t)(py + ys) * cols + 4 * k;
                        if (al) {
                            const float4 a = *(const float4 *)(q - cols), b = *(const float4 *)q,
                                         c = *(const float4 *)(q + cols);
                            T.m[0] = a.x; T.m[1] = a.y; T.m[2] = a.z; T.m[3] = a.w;
                            T.c[1] = b.x; T.c[2] = b.y; T.c[3] = b.z; T.c[4] = b.w;
                            T.p[0] = c.x; T.p[1] = c.y; T.p[2] = c.z; T.p[3] = c.w;
                        } else {
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                T.m[i] = q[i - cols];
                                T.c[i + 1] = q[i];
                                T.p[i] = q[i + cols];
                            }
                        }
                        T.c[0] = q[-1];
                        T.c[5] = q[4];
                    };
                    // kRowLanes consecutive lanes take consecutive items (one row span per load);
                    // the 64 / kRowLanes lane sets walk their own contiguous part of the items,
                    // in other rows -- other spatial cells, so the histogram atomics of a wave
                    // spread over addresses (fully interleaved, adjacent pixels of one cell with
                    // similar gradients serialise on the same LDS words)
                    constexpr int NSET = 64 / kRowLanes;
                    const int per = ((rrun + NSET - 1) / NSET + kRowLanes - 1) / kRowLanes * kRowLanes;
                    const int t0 = (lane / kRowLanes) * per + (lane % kRowLanes);
                    const int tend = min(t0 - (lane % kRowLanes) + per, rrun);
                    Taps A, B;
                    int ysA = 0, kA = 0;
                    if (t0 < tend) fetch(t0, A, ysA, kA);
                    for (int t = t0; t < tend; t += kRowLanes) {
                        int ysB = 0, kB = 0;
                        if (t + kRowLanes < tend) fetch(t + kRowLanes, B, ysB, kB);
                        const float ysf = (float)ysA, ys2 = ysf * ysf;
                        const int c0 = 4 * kA - px + half;       // patch column of the strip's first
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int xs = c0 + i - half;
                            sample(A.c[i + 2] - A.c[i], A.m[i] - A.p[i], fmaf(ysf, ar, cbr[c0 + i]),
                                   fmaf(ysf, ac, cbc[c0 + i]), __builtin_amdgcn_exp2f(kq * (ys2 + (float)(xs * xs))));
                        }
                        A = B;
                        ysA = ysB;
                        kA = kB;
                    }
                }
            }
            if (!rows_done) square_walk();
#else
            {
            // lane group g (kDescGrp adjacent lanes) walks its run of (super-strip, row) steps;
            // lane `sub` of the group takes strip `sub` of each super-strip, so one load
            // instruction covers a group's kDescSS-column row span in ~1 cache line
#if PANO_DESC_ABL_NOWALK
            const int nsamp = 0;                           // timing ablation: per-keypoint work only
#else
            const int nsamp = run;                         // (super-strip, row) steps
#endif
            constexpr int NG = 64 / kDescGrp;
            const int Q = (nsamp + NG - 1) / NG;
            const int sub = lane & (kDescGrp - 1);
            int t = (lane / kDescGrp) * Q;
            const int tend = min(t + Q, nsamp);
#if PANO_DESC_COMPACT
            // Compaction.  About half the lane slots of the direct walk carry a rejected
            // sample (the super-strip's union interval, the rotated square's corners, ragged
            // run ends): measured at parrington, 175 VALU lane-slots per binned sample against
            // ~87 instructions of binning.  Here the walk only forms each candidate's inputs
            // (taps, bin coordinates, weight exponent) and appends the ones that pass the bin
            // test to the wave's LDS ring (ballot + mbcnt); every time 64 are waiting, each lane
            // bins one -- the same samples with the same arithmetic, so the integer histogram
            // is bit-identical.  The walk runs Q wave-uniform steps, `live` per lane.
            {
                float2 *qg = cq_g[wv], *qb = cq_b[wv];
                float *qw = cq_w[wv];
                int qh = 0, qn = 0;                      // wave-uniform ring head / count
                auto drain = [&](int n) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    if (lane < n) {
                        const int e = (qh + lane) & (kDescQ - 1);
                        const float2 g = qg[e], b = qb[e];
                        sample_in(g.x, g.y, b.x, b.y, __builtin_amdgcn_exp2f(qw[e]));
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();     // read before the slots are refilled
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    qh = (qh + n) & (kDescQ - 1);
                    qn -= n;
                };
                auto put = [&](bool live, float gx, float gy, float rbin, float cbin, float warg) {
                    const bool ok = live && rbin > -1.0f && rbin < 4.0f && cbin > -1.0f && cbin < 4.0f;
                    const unsigned long long m = __ballot(ok);
                    if (ok) {
                        const int r = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                        const int e = (qh + qn + r) & (kDescQ - 1);
                        qg[e] = make_float2(gx, gy);
                        qb[e] = make_float2(rbin, cbin);
                        qw[e] = warg;
                    }
                    qn += __popcll(m);
                    if (qn >= 64) drain(64);
                };
                constexpr int WN = kDescSW + 2;
                int sx = 0, ys = 0, yend = 0;
                auto win = [&](int sxx, int y, float (&T)[WN]) {
                    const float *q = img + (size_t)(py + y) * cols + (px + sxx * kDescSS + sub * kDescSW - half) - 1;
#pragma unroll
                    for (int i = 0; i < WN; ++i) T[i] = q[i];
                };
                float br[kDescSW], bc[kDescSW], xs2[kDescSW];
                auto strip_consts = [&](int sxx) {
#pragma unroll
                    for (int i = 0; i < kDescSW; ++i) {
                        const int c = sxx * kDescSS + sub * kDescSW + i;
                        br[i] = cbr[c];
                        bc[i] = cbc[c];
                        xs2[i] = (float)((c - half) * (c - half));
                    }
                };
                float Tm[WN], T0[WN], Tp[WN];
                if (t < tend) {
                    int shi = nstrip - 1;                // largest strip with cpre[sx] <= t
                    while (sx < shi) {
                        const int mid = (sx + shi + 1) >> 1;
                        if (cpre[mid] <= t) sx = mid;
                        else shi = mid - 1;
                    }
                    ys = clo[sx] + (t - cpre[sx]);
                    yend = clo[sx] + (cpre[sx + 1] - cpre[sx]);
                    strip_consts(sx);
                    win(sx, ys - 1, Tm);
                    win(sx, ys, T0);
                    win(sx, ys + 1, Tp);
                }
                for (int it = 0; it < Q; ++it) {
                    const int j = t + it;
                    const bool live = j < tend;
                    int sn = sx, yn = ys + 1;
                    const bool more = j + 1 < tend;
                    const bool newstrip = more && yn >= yend;
                    if (newstrip) {
                        do { ++sn; } while (cpre[sn + 1] == cpre[sn]);
                        yn = clo[sn];
                    }
                    float N2[WN];
                    if (more && !newstrip) win(sn, yn + 1, N2);
                    const float ysf = (float)ys, ys2 = ysf * ysf;
#pragma unroll
                    for (int i = 0; i < kDescSW; ++i)
                        put(live, T0[i + 2] - T0[i], Tm[i + 1] - Tp[i + 1], fmaf(ysf, ar, br[i]),
                            fmaf(ysf, ac, bc[i]), kq * (ys2 + xs2[i]));
                    if (more) {
                        if (newstrip) {
                            sx = sn;
                            yend = clo[sx] + (cpre[sx + 1] - cpre[sx]);
                            strip_consts(sx);
                            win(sn, yn - 1, Tm);
                            win(sn, yn, T0);
                            win(sn, yn + 1, Tp);
                        } else {
#pragma unroll
                            for (int i = 0; i < WN; ++i) { Tm[i] = T0[i]; T0[i] = Tp[i]; Tp[i] = N2[i]; }
                        }
                        ys = yn;
                    }
                }
                if (qn > 0) drain(qn);
            }
#elif PANO_DESC_RING
            // Tap rows prefetched kRing steps ahead through an LDS ring by LDS-DMA loads
            // (global_load_lds, 2 x 12 bytes per lane and step, no VGPRs): more of each wave's
            // scattered row loads in flight than the one-step register prefetch allows (its
            // misses, not the VALU or the histogram, bound the kernel: PANO_DESC_ABL ablations).
            // The walk runs a uniform iteration count Q; a lane past its run issues its ring
            // loads from a fixed in-image address and bins nothing.  A strip change loads the
            // new strip's upper two rows directly (about once per lane run).
            {
                const int nst = tend > t ? tend - t : 0;     // this lane's steps
                int sx = 0, ys = 0, yend = 0;
                if (nst > 0) {
                    int shi = nstrip - 1;                    // largest strip with cpre[sx] <= t
                    while (sx < shi) {
                        const int mid = (sx + shi + 1) >> 1;
                        if (cpre[mid] <= t) sx = mid;
                        else shi = mid - 1;
                    }
                    ys = clo[sx] + (t - cpre[sx]);
                    yend = clo[sx] + (cpre[sx + 1] - cpre[sx]);
                }
                constexpr int WN = kDescSW + 2;
                static_assert(WN == 6, "the ring moves 2 x 3 floats per lane and step");
                auto rowp = [&](int sxx, int y) {
                    return img + (size_t)(py + y) * cols + (px + sxx * kDescSS + sub * kDescSW - half) - 1;
                };
                const float *dummy = img + (size_t)py * cols + px - 1;
                float *rw = &ring[wv][0][0][0];
                // 16-byte LDS-DMA loads land at base + 16 lane (a 12-byte one too: measured,
                // tools/probes/glds_layout.hip), so a lane's 6 floats are two 16-byte loads,
                // floats 0-3 and 2-5 of its window
                // M0 written and read in one statement with the s_nop the M0 -> LDS-DMA hazard
                // needs (cdna_hip_programming.md, LDS-DMA recipe)
                const unsigned rw_lds = (unsigned)(uintptr_t)(__attribute__((address_space(3))) float *)rw;
                auto issue = [&](int slot, const float *q) {
                    const unsigned d0 = __builtin_amdgcn_readfirstlane(rw_lds + slot * 2048);
                    const unsigned d1 = d0 + 1024;
                    unsigned keep;
                    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                                 : "=&s"(keep) : "v"(q), "s"(d0) : "memory");
                    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                                 : "=&s"(keep) : "v"(q + 2), "s"(d1) : "memory");
                };
                // the prefetch cursor: position of step ip (ip < nst), advanced like the walk
                int psx = sx, pys = ys, pyend = yend;
                auto pf_next = [&]() {
                    ++pys;
                    if (pys >= pyend) {
                        do { ++psx; } while (psx < nstrip && cpre[psx + 1] == cpre[psx]);
                        if (psx < nstrip) {
                            pys = clo[psx];
                            pyend = clo[psx] + (cpre[psx + 1] - cpre[psx]);
                        }
                    }
                };
#pragma unroll
                for (int k = 0; k < kRing; ++k) {
                    issue(k, k < nst ? rowp(psx, pys + 1) : dummy);
                    if (k + 1 < kRing && k + 1 < nst) pf_next();     // the cursor ends on step kRing - 1
                }
                float br[kDescSW], bc[kDescSW], xs2[kDescSW];
                auto strip_consts = [&](int sxx) {
#pragma unroll
                    for (int i = 0; i < kDescSW; ++i) {
                        const int c = sxx * kDescSS + sub * kDescSW + i;
                        br[i] = cbr[c];
                        bc[i] = cbc[c];
                        xs2[i] = (float)((c - half) * (c - half));
                    }
                };
                float Tm[WN], T0[WN];
                if (nst > 0) {
                    strip_consts(sx);
                    const float *q0 = rowp(sx, ys - 1), *q1 = rowp(sx, ys);
#pragma unroll
                    for (int i = 0; i < WN; ++i) { Tm[i] = q0[i]; T0[i] = q1[i]; }
                }
                for (int it = 0; it < Q; ++it) {
                    const int slot = it % kRing;
#ifdef PANO_DESC_RING_VM0
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#else
                    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * (kRing - 1)) : "memory");
#endif
                    const bool live = it < nst;
                    float Tp[WN];
                    {
                        const float4 a = *(const float4 *)(rw + slot * 512 + lane * 4);
                        const float2 b = *(const float2 *)(rw + slot * 512 + 256 + lane * 4 + 2);
                        Tp[0] = a.x; Tp[1] = a.y; Tp[2] = a.z; Tp[3] = a.w; Tp[4] = b.x; Tp[5] = b.y;
                    }
#ifdef PANO_DESC_RING_DEBUG
                    if (live) {
                        const float *qq = rowp(sx, ys + 1);
                        bool bad = false;
                        for (int i = 0; i < WN; ++i) bad |= qq[i] != Tp[i];
                        if (bad && (it == 2 || it == 3) && blockIdx.x < 2) {
                            const float *qa = rowp(sx, ys), *qb = rowp(sx, ys + 2), *qc = rowp(sx, ys - 1);
                            printf("ring mismatch blk %d lane %d it %d nst %d sx %d ys %d: ring %g %g | row+1 %g %g | row %g %g | row+2 %g %g | row-1 %g %g\n",
                                   (int)blockIdx.x, lane, it, nst, sx, ys, Tp[0], Tp[1], qq[0], qq[1], qa[0], qa[1], qb[0], qb[1], qc[0], qc[1]);
                        }
                    }
#endif
                    if (live) {
                        const float ysf = (float)ys, ys2 = ysf * ysf;
#pragma unroll
                        for (int i = 0; i < kDescSW; ++i)
                            sample(T0[i + 2] - T0[i], Tm[i + 1] - Tp[i + 1], fmaf(ysf, ar, br[i]),
                                   fmaf(ysf, ac, bc[i]), __builtin_amdgcn_exp2f(kq * (ys2 + xs2[i])));
                    }
                    // the slot is re-filled with step it + kRing once its reads have returned
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    const int ip = it + kRing;
                    if (ip < nst) pf_next();
                    issue(slot, ip < nst ? rowp(psx, pys + 1) : dummy);
                    if (live && it + 1 < nst) {
                        int yn = ys + 1;
                        if (yn >= yend) {
                            do { ++sx; } while (cpre[sx + 1] == cpre[sx]);
                            yn = clo[sx];
                            yend = clo[sx] + (cpre[sx + 1] - cpre[sx]);
                            strip_consts(sx);
                            const float *q0 = rowp(sx, yn - 1), *q1 = rowp(sx, yn);
#pragma unroll
                            for (int i = 0; i < WN; ++i) { Tm[i] = q0[i]; T0[i] = q1[i]; }
                        } else {
#pragma unroll
                            for (int i = 0; i < WN; ++i) { Tm[i] = T0[i]; T0[i] = Tp[i]; }
                        }
                        ys = yn;
                    }
                }
                // drain: the ring's last loads land before the next keypoint reuses it
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
#else
            if (t < tend) {
                int sx = 0, shi = nstrip - 1;              // largest strip with cpre[sx] <= t
                while (sx < shi) {
                    const int mid = (sx + shi + 1) >> 1;
                    if (cpre[mid] <= t) sx = mid;
                    else shi = mid - 1;
                }
                int ys = clo[sx] + (t - cpre[sx]);
                int yend = clo[sx] + (cpre[sx + 1] - cpre[sx]);
                // columns x-1 .. x+kDescSW of image row py + y at strip sx: ONE wide load per
                // step serves the strip's kDescSW samples.  Rows stay in [0, rows - 1]; the
                // columns of a strip with an invalid column can reach kDescSW floats before or
                // after the row (the neighbouring row or level plane of the same pyramid
                // buffer: allocated), and those samples are rejected before their taps are used
                constexpr int WN = kDescSW + 2;
                auto win = [&](int sxx, int y, float (&T)[WN]) {
#if PANO_DESC_ABL == 3
                    const float *q = img + (size_t)py * cols + px + ((sxx + y) & 1) - 1;   // L1-resident
#elif PANO_DESC_ABL == 4
                    // coalesced: every lane of the wave in the first active lane's row, 16-lane
                    // groups over 64 consecutive columns (2 lines per load; values wrong)
                    const int yu = __builtin_amdgcn_readfirstlane(y);
                    const int cq = min(max(px - half - 1, 0) + (lane & 15) * 4, cols - WN);
                    const float *q = img + (size_t)(py + yu) * cols + max(cq, 0);
#elif PANO_DESC_ABL == 5
                    // each lane's own row, the whole wave in one 64-column span of it (as 4 but
                    // the rows scattered: lines per load = distinct rows)
                    const int cq = min(max(px - half - 1, 0) + (lane & 15) * 4, cols - WN);
                    const float *q = img + (size_t)(py + y) * cols + max(cq, 0);
#else
                    const float *q = img + (size_t)(py + y) * cols + (px + sxx * kDescSS + sub * kDescSW - half) - 1;
#endif
#pragma unroll
                    for (int i = 0; i < WN; ++i) T[i] = q[i];
                };
                float br[kDescSW], bc[kDescSW], xs2[kDescSW];
                auto strip_consts = [&](int sxx) {
#pragma unroll
                    for (int i = 0; i < kDescSW; ++i) {
                        const int c = sxx * kDescSS + sub * kDescSW + i;
                        br[i] = cbr[c];
                        bc[i] = cbc[c];
                        xs2[i] = (float)((c - half) * (c - half));
                    }
                };
                strip_consts(sx);
#if PANO_DESC_UNROLL
                // the three-row window rotates through four buffers with static roles (the
                // step unrolled 4x): no register moves per step
                float XA[WN], XB[WN], XC[WN], XD[WN];
                win(sx, ys - 1, XA);
                win(sx, ys, XB);
                win(sx, ys + 1, XC);
                int j = t;
                auto step = [&](float (&Tm)[WN], float (&T0)[WN], float (&Tp)[WN], float (&Nx)[WN]) -> bool {
                    if (j >= tend) return false;
                    int sn = sx, yn = ys + 1;
                    const bool more = j + 1 < tend;
                    const bool newstrip = more && yn >= yend;
                    if (newstrip) {
                        do { ++sn; } while (cpre[sn + 1] == cpre[sn]);
                        yn = clo[sn];
                    }
                    if (more && !newstrip) win(sn, yn + 1, Nx);
                    const float ysf = (float)ys, ys2 = ysf * ysf;
#pragma unroll
                    for (int i = 0; i < kDescSW; ++i)
                        sample(T0[i + 2] - T0[i], Tm[i + 1] - Tp[i + 1], fmaf(ysf, ar, br[i]),
                               fmaf(ysf, ac, bc[i]), __builtin_amdgcn_exp2f(kq * (ys2 + xs2[i])));
                    if (newstrip) {
                        sx = sn;
                        yend = clo[sx] + (cpre[sx + 1] - cpre[sx]);
                        strip_consts(sx);
                        // the next step's (Tm, T0, Tp) are this step's (T0, Tp, Nx)
                        win(sn, yn - 1, T0);
                        win(sn, yn, Tp);
                        win(sn, yn + 1, Nx);
                    }
                    ys = yn;
                    ++j;
                    return true;
                };
                for (;;) {
                    if (!step(XA, XB, XC, XD)) break;
                    if (!step(XB, XC, XD, XA)) break;
                    if (!step(XC, XD, XA, XB)) break;
                    if (!step(XD, XA, XB, XC)) break;
                }
#else
                float Tm[WN], T0[WN], Tp[WN];
                win(sx, ys - 1, Tm);
                win(sx, ys, T0);
                win(sx, ys + 1, Tp);
                for (int j = t; j < tend; ++j) {
                    // the next step's position (this strip, or the next non-empty one), its
                    // taps loaded while this step's samples are binned
                    int sn = sx, yn = ys + 1;
                    const bool more = j + 1 < tend;
                    const bool newstrip = more && yn >= yend;
                    if (newstrip) {
                        do { ++sn; } while (cpre[sn + 1] == cpre[sn]);
                        yn = clo[sn];
                    }
                    float N2[WN];
#if PANO_DESC_NS_PREFETCH
                    float N0[WN], N1[WN];
                    if (newstrip) {
                        win(sn, yn - 1, N0);
                        win(sn, yn, N1);
                    }
                    if (more) win(sn, yn + 1, N2);
#else
                    if (more && !newstrip) win(sn, yn + 1, N2);
#endif
                    const float ysf = (float)ys, ys2 = ysf * ysf;
#if PANO_DESC_COUNT
                    {
                        const unsigned long long act = __ballot(1);
                        const int first = __ffsll((long long)act) - 1;
                        unsigned long long pass = 0, blocks = 0;
                        for (int i = 0; i < kDescSW; ++i) {
                            const float rb = fmaf(ysf, ar, br[i]), cb = fmaf(ysf, ac, bc[i]);
                            const unsigned long long m = __ballot(rb > -1.0f && rb < 4.0f && cb > -1.0f && cb < 4.0f);
                            pass += __popcll(m);
                            blocks += m != 0;
                        }
                        if (lane == first) {
                            atomicAdd(&g_desc_cnt[0], (unsigned long long)__popcll(act) * kDescSW);
                            atomicAdd(&g_desc_cnt[1], pass);
                            atomicAdd(&g_desc_cnt[2], blocks);
                            atomicAdd(&g_desc_cnt[3], 1ull);
                            atomicAdd(&g_desc_cnt[4], (unsigned long long)__popcll(act));
                        }
                    }
#endif
                    // exp(-((rrot/hw)^2 + (crot/hw)^2) / 8) = exp2(kq (xs^2 + ys^2)): a rotation
                    // keeps the radius (no LDS read on the sample path)
#pragma unroll
                    for (int i = 0; i < kDescSW; ++i)
                        sample(T0[i + 2] - T0[i], Tm[i + 1] - Tp[i + 1], fmaf(ysf, ar, br[i]),
                               fmaf(ysf, ac, bc[i]), __builtin_amdgcn_exp2f(kq * (ys2 + xs2[i])));
                    if (newstrip) {
                        sx = sn;
                        yend = clo[sx] + (cpre[sx + 1] - cpre[sx]);
                        strip_consts(sx);
#if PANO_DESC_NS_PREFETCH
#pragma unroll
                        for (int i = 0; i < WN; ++i) { Tm[i] = N0[i]; T0[i] = N1[i]; Tp[i] = N2[i]; }
#else
                        // a strip change (about once per lane run) loads its three rows here
                        win(sn, yn - 1, Tm);
                        win(sn, yn, T0);
                        win(sn, yn + 1, Tp);
#endif
                    } else {
#pragma unroll
                        for (int i = 0; i < WN; ++i) { Tm[i] = T0[i]; T0[i] = Tp[i]; Tp[i] = N2[i]; }
                    }
                    ys = yn;
                }
#endif
            }
#endif
            }
#endif
        } else {
            square_walk();
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // crop the padding: element i = (r, c, o) of the 4 x 4 x 8 block
        auto interior = [&](int i) {
            const int e = ((i >> 5) + 1) * kRowC + (((i >> 3) & 3) + 1) * kCell + (i & 7);
            unsigned long long v = 0;
#pragma unroll
            for (int c = 0; c < kDescCopies; ++c) v += h0[c * kHistStride + e];
            return (float)((double)v * (1.0 / 4194304.0));
        };
        float lo = interior(lane), hi = interior(64 + lane);
        if (PANO_DESC_ABL >= 2) lo += (float)abl_sink;   // keeps the ablations' samples alive
#if PANO_DESC_ABL_NOEPI                        // timing ablation: no norms (plain scaling)
        float nv = 1.0f;
#else
        const float thr = sqrtf(sdot_skx_wave128(lo, hi)) * dp.max_value;
        lo = lo > thr ? thr : lo;
        hi = hi > thr ? thr : hi;
        float nv = sqrtf(sdot_skx_wave128(lo, hi));
#endif
        if (nv < 1e-7f) nv = 1e-7f;
        float dlo = rintf(512.0f * (lo / nv)), dhi = rintf(512.0f * (hi / nv));
        dlo = dlo < 0.0f ? 0.0f : (dlo > 255.0f ? 255.0f : dlo);
        dhi = dhi < 0.0f ? 0.0f : (dhi > 255.0f ? 255.0f : dhi);
        if constexpr (OUT_U8) {
            desc_u8[row * PANO_DESC_DIM + lane] = (uint8_t)dlo;
            desc_u8[row * PANO_DESC_DIM + 64 + lane] = (uint8_t)dhi;
            int sq = (int)dlo * (int)dlo + (int)dhi * (int)dhi;
#pragma unroll
            for (int d = 32; d > 0; d >>= 1) sq += __shfl_xor(sq, d);
            if (lane == 0) norms[row] = sq;
        } else {
            desc[row * PANO_DESC_DIM + lane] = dlo;
            desc[row * PANO_DESC_DIM + 64 + lane] = dhi;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();                   // h / column tables reused next
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#if PANO_DESC_TIMING
        ++nkp;
#endif
    }
#if PANO_DESC_TIMING
    {
        const int gw = (int)blockIdx.x * kDescWaves + wv;
        if (lane == 0 && gw < kDescClkWaves) {
            unsigned long long *o = g_desc_clk[gw];
            o[0] = t_entry;
            o[1] = (unsigned long long)__builtin_amdgcn_s_memrealtime();
            o[2] = (unsigned long long)nkp;
            o[3] = (unsigned long long)(xcd + 1);
        }
    }
#endif
}

// Processing order of the descriptor waves: keypoints are emitted x-sorted (the reference's
// order), so consecutive ones lie in different pyramid planes and rows, and concurrent waves
// miss the caches on unrelated patches.  desc_order groups each frame's keypoints by the
// plane they sample (octave + 1, layer) and a 16-row band of it (counting sort, one
// workgroup per frame: LDS histogram, scan, scatter), so the waves of an XCD walk one band of
// one plane together.  Only the ORDER of work changes: outputs stay at each keypoint's row
// and are bit-identical (integer histograms).
struct OrderArgs {
    int bstart[PANO_MAX_OCTAVES + 1];   // first bucket of plane octave O (its layers x bands)
    int nband[PANO_MAX_OCTAVES];        // 16-row bands of octave O
    int n_oct, n_lvl, nb;               // octaves, levels, buckets per frame
    int by_size;                        // 1: largest window first (buckets = kOrderHalves - half)
    float hw_mult;                      // DescParams::hw_mult (the window's half width)
};
constexpr int kOrderHalves = 128;       // size order: window half widths 0 .. 127 (larger: bucket 0)

__device__ __forceinline__ int desc_bucket(const pano_kp &kp, const OrderArgs &oa) {
    int oct = kp.octave & 255;
    if (oct >= 128) oct |= -128;
    const int lyr = (kp.octave >> 8) & 255, O = oct + 1;
    if (O < 0 || O >= oa.n_oct || lyr >= oa.n_lvl) return 0;
    const float scl = oct >= 0 ? 1.0f / (float)(1 << oct) : (float)(1 << -oct);
    if (oa.by_size) {                   // descriptor_wave's own half width, largest first
        const float hw = (oa.hw_mult * scl) * kp.size;
        const int half = (int)rint((double)hw * 1.4142135623730951 * 5.0 * 0.5);
        return kOrderHalves - 1 - min(max(half, 0), kOrderHalves - 1);
    }
    int band = (int)rint((double)scl * (double)kp.y) >> 4;
    band = band < 0 ? 0 : (band >= oa.nband[O] ? oa.nband[O] - 1 : band);
    return oa.bstart[O] + lyr * oa.nband[O] + band;
}

__global__ void __launch_bounds__(kSortThreads)
desc_order(const pano_kp *__restrict__ kps, const int32_t *__restrict__ counts, int cap, OrderArgs oa,
           int32_t *__restrict__ order) {
    __shared__ int32_t bc[kSortMaxBuckets];
    __shared__ int32_t wsum[kSortThreads / 64];
    const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int n = min(max(counts[f], 0), cap), nb = oa.nb;
    const pano_kp *kp = kps + (size_t)f * cap;
    for (int b = tid; b < nb; b += kSortThreads) bc[b] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += kSortThreads) atomicAdd(&bc[desc_bucket(kp[i], oa)], 1);
    __syncthreads();
    const int per = (nb + kSortThreads - 1) / kSortThreads, b0 = tid * per;
    int run = 0;
    for (int q = 0; q < per; ++q)
        if (b0 + q < nb) run += bc[b0 + q];
    int incl = run;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int base = incl - run;
    for (int w = 0; w < wv; ++w) base += wsum[w];
    for (int q = 0; q < per; ++q) {
        const int b = b0 + q;
        if (b >= nb) break;
        const int c = bc[b];
        bc[b] = base;
        base += c;
    }
    __syncthreads();
    int32_t *ord = order + (size_t)f * cap;
    for (int i = tid; i < n; i += kSortThreads) ord[atomicAdd(&bc[desc_bucket(kp[i], oa)], 1)] = i;
}

// find_scale_space_extrema's output order (sift_impl.py:117-140): candidates in scan order
// (octave, layer, y, x), each one's orientations in peak-bin order.  The RawKp order keys are
// that order and unique per frame, so a record's position is the number of smaller keys;
// the keys of the frame stream through LDS in tiles of 256.  Keypoints stay in base
// coordinates (no dedup, no conversion).  counts[f] = raw count (> cap: dropped entries) or
// -1 when an earlier stage overflowed its scratch.
__global__ void __launch_bounds__(256)
raw_scan_order(const RawKp *__restrict__ raw, const int32_t *__restrict__ raw_cnt, int raw_cap,
               pano_kp *__restrict__ out, int cap, int32_t *__restrict__ counts, int32_t *__restrict__ err,
               const int32_t *__restrict__ ext_cnt, int ext_cap, const int32_t *__restrict__ cand_cnt,
               int cand_cap) {
    __shared__ uint64_t keys[256];
    const int f = blockIdx.y, tid = threadIdx.x, i = blockIdx.x * 256 + tid;
    const int cnt = raw_cnt[f * kCntStride];
    if (cnt > raw_cap || ext_cnt[f * kCntStride] > ext_cap || cand_cnt[f * kCntStride] > cand_cap) {
        if (blockIdx.x == 0 && tid == 0) { err[0] = PANO_E_OVERFLOW; counts[f] = -1; }
        return;
    }
    if (blockIdx.x == 0 && tid == 0) counts[f] = cnt;
    if (blockIdx.x * 256 >= cnt) return;                 // uniform per workgroup
    const RawKp *rec = raw + (size_t)f * raw_cap;
    const uint64_t mine = i < cnt ? rec[i].order : ~0ull;
    int rank = 0;
    for (int t0 = 0; t0 < cnt; t0 += 256) {
        __syncthreads();
        keys[tid] = t0 + tid < cnt ? rec[t0 + tid].order : ~0ull;
        __syncthreads();
        const int m = min(256, cnt - t0);
        for (int j = 0; j < m; ++j) rank += keys[j] < mine;
    }
    if (i < cnt && rank < cap) {
        const RawKp q = rec[i];
        pano_kp o;
        o.x = q.x;
        o.y = q.y;
        o.size = q.size;
        o.angle = q.angle;
        o.response = q.response;
        o.octave = q.octave;
        out[(size_t)f * cap + rank] = o;
    }
}

}  // namespace

int sift_reserve_pyramid(pano_ctx *ctx, int n, int h, int w, const pano_sift_params *p);

namespace {
int launch_descriptors(pano_ctx *ctx, const pano_sift_params *p, const PyrArgs &pa, const pano_kp *kps,
                       const int32_t *counts, int cap, int32_t *desc_work, float *desc, uint8_t *desc_u8,
                       int32_t *norms, const RawKp *rawk = nullptr);

// Scratch of the keypoint stage (per-frame capacities scaled with the pyramid, see kExtMin)
// and the counter block: [err] [cand f] [raw f] [ext f] [descriptor, orientation work queues
// per XCD x 8 each], one line apiece.
struct KpBufs {
    size_t ext_cap, cand_cap, raw_cap, cnt_ints;
    uint64_t *raw_ext;
    int32_t *err, *cand_cnt, *raw_cnt, *ext_cnt, *desc_work, *ori_work;
};

int kp_bufs(pano_ctx *ctx, KpBufs &b) {
    const int n = ctx->n, no = ctx->n_oct;
    size_t spo = 0;
    for (int o = 0; o < no; ++o) spo += (size_t)ctx->oct_h[o] * ctx->oct_w[o];
    b.ext_cap = std::max<size_t>(kExtMin, ((spo / 32) + 1023) & ~size_t(1023));
    b.cand_cap = std::max<size_t>(kCandMin, b.ext_cap / 4);
    b.raw_cap = b.cand_cap;
    int rc = pano_grow(ctx, (void **)&ctx->cands, &ctx->cand_cap, b.cand_cap * n * sizeof(Cand));
    if (rc) return rc;
    rc = pano_grow(ctx, (void **)&ctx->raw, &ctx->raw_cap, b.raw_cap * n * sizeof(RawKp));
    if (rc) return rc;
    rc = pano_grow(ctx, (void **)&ctx->frame_off, &ctx->ext_bytes, b.ext_cap * n * sizeof(uint64_t));
    if (rc) return rc;
    b.raw_ext = (uint64_t *)ctx->frame_off;
    b.cnt_ints = (3 * (size_t)n + 1 + 16) * kCntStride;
    rc = pano_grow(ctx, (void **)&ctx->counters, &ctx->counters_n, b.cnt_ints * sizeof(int32_t));
    if (rc) return rc;
    b.err = ctx->counters;
    b.cand_cnt = b.err + kCntStride;
    b.raw_cnt = b.cand_cnt + (size_t)n * kCntStride;
    b.ext_cnt = b.raw_cnt + (size_t)n * kCntStride;
    b.desc_work = b.ext_cnt + (size_t)n * kCntStride;
    b.ori_work = b.desc_work + 8 * kCntStride;
    return PANO_OK;
}

// The smallest octave
// height the streaming kernel takes (0 disables it).  Measured (same box): 96 -- parrington's
// octave 3 joins the streaming launch instead of its own scan -- 164-167 us per extrema class
// against 175-178 us at 192; 48 within noise of 96.
// Output rows per extrema_stream item, by the batch's size: a wave's walk costs its first
// XPD rows of load latency and two halo rows, so taller strips are cheaper per row -- but the
// launch must still hold about two rounds of resident waves, or its last partial round leaves
// the chip idle.  The tallest of kXsrs whose item count is >= 2 rounds of resident waves (else
// the shortest).  Measured (tools/feat_time.py, profiles/r06_extrema_xsr_ab.txt): parrington
// 24 rows 0.1445 ms against 0.147 (32) and 0.151 (48); 1080p 48 rows 1.105-1.112 against
// 1.16-1.18 (32) and 1.26-1.28 (24).  PANO_EXTREMA_XSR=<one of kXsrs> forces one height.
constexpr int kXsrs[] = {24, 32, 48, 64};
int extrema_items(const pano_ctx *ctx, int border, int xsr) {
    int items = 0;
    for (int o = 0; o < ctx->n_oct; ++o) {
        const int iw = ctx->oct_w[o] - 2 * border, ih = ctx->oct_h[o] - 2 * border;
        if (iw > 0 && ih > 0) items += ((iw + XSW - 1) / XSW) * ((ih + xsr - 1) / xsr);
    }
    return items;
}
int extrema_xsr(const pano_ctx *ctx, int border) {
    static const int forced = [] {
        const char *e = getenv("PANO_EXTREMA_XSR");
        const int v = e ? atoi(e) : 0;
        for (int x : kXsrs) if (v == x) return v;
        return 0;
    }();
    if (forced) return forced;
    static long long resident = 0;                  // waves the chip holds at the kernel's occupancy
    if (!resident) {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, extrema_stream<5, 32>, 256, 0) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess ||
            per_cu <= 0 || cus <= 0)
            per_cu = 6, cus = 256;
        resident = 4LL * per_cu * cus;
    }
    int pick = kXsrs[0];
    for (int x : kXsrs)
        if ((long long)ctx->n * extrema_items(ctx, border, x) >= 2 * resident) pick = x;
    return pick;
}
int extrema_min_h() {
    static const int v = [] {
        const char *e = getenv("PANO_EXTREMA_STREAM_MIN_H");
        return e ? atoi(e) : 96;
    }();
    return v;
}

// The streaming kernel's items (strips of xsr rows) of every octave, octave-major.
XArgs x_args(const pano_ctx *ctx, int border) {
    XArgs xa{};
    // every strip height is instantiated for the default 5 DoG levels only (launch_extrema_stream)
    const int no = ctx->n_oct, nl = ctx->n_lvl, xsr = nl - 1 == 5 ? extrema_xsr(ctx, border) : 32;
    int items = 0;
    xa.sr = xsr;
    xa.n_oct = no;
    for (int o = 0; o < no; ++o) {
        xa.H[o] = ctx->oct_h[o];
        xa.W[o] = ctx->oct_w[o];
        for (int l = 0; l < nl - 1; ++l) xa.dog[o][l] = ctx->dog + ctx->dog_off[o][l];
        const int iw = xa.W[o] - 2 * border, ih = xa.H[o] - 2 * border;
        xa.item_start[o] = items;
        xa.strips_x[o] = iw > 0 ? (iw + XSW - 1) / XSW : 1;
        if (iw > 0 && ih > 0) items += xa.strips_x[o] * ((ih + xsr - 1) / xsr);
    }
    xa.item_start[no] = items;
    return xa;
}

double extrema_thresh(const pano_sift_params *p) {
    return floor(0.5 * p->contrast_threshold / p->num_intervals * 255);
}

int launch_extrema_stream(pano_ctx *ctx, const pano_sift_params *p, const XArgs &xa, const KpBufs &b,
                          int t0, int t1, hipStream_t st) {
    if (t1 <= t0) return PANO_OK;
    const int n = ctx->n, ni = p->num_intervals, xsr = xa.sr;
    const double thresh = extrema_thresh(p);
    dim3 grid((unsigned)((t1 - t0 + 3) / 4), n);
    {
        PanoProf prof_(ctx, PK_EXTREMA, st);
#define PANO_EXTREMA(NLV, SR) \
    extrema_stream<NLV, SR><<<grid, 256, 0, st>>>(xa, p->border, thresh, b.raw_ext, b.ext_cnt, (int)b.ext_cap, t0, t1)
        // every strip height for the default 5 DoG levels; the other level counts at 32 rows
        // (x_args numbered their items at xa.sr: fail rather than scan the wrong rows)
        if (ni + 2 == 5) {
            switch (xsr) {
                case 24: PANO_EXTREMA(5, 24); break;
                case 32: PANO_EXTREMA(5, 32); break;
                case 48: PANO_EXTREMA(5, 48); break;
                case 64: PANO_EXTREMA(5, 64); break;
                default: return pano_fail(ctx, PANO_E_UNSUPPORTED, "extrema strip height");
            }
        } else {
            if (xsr != 32) return pano_fail(ctx, PANO_E_UNSUPPORTED, "extrema strip height");
            switch (ni + 2) {
                case 3: PANO_EXTREMA(3, 32); break;
                case 4: PANO_EXTREMA(4, 32); break;
                case 6: PANO_EXTREMA(6, 32); break;
                case 7: PANO_EXTREMA(7, 32); break;
                default: return pano_fail(ctx, PANO_E_UNSUPPORTED, "num_intervals above 5");
            }
        }
#undef PANO_EXTREMA
    }
    PANO_LAUNCH_CHECK(ctx, "extrema_stream");
    return PANO_OK;
}

// Fraction of the resident workgroups the persistent orientation / descriptor grids take
// (PANO_PERSIST_FRAC, default 1): below 1, a stitch overlapping on another context
// (pipeline.StitchPool) keeps CU slots while they run.
// PANO_ORI_FAST_BIN=0 (read per call): every orientation bin through ori_bin_exact (A/B and
// test_orientation_fast_bin_identical)
int ori_fast_bin() {
    const char *e = getenv("PANO_ORI_FAST_BIN");
    return e && atoi(e) == 0 ? 0 : 1;
}
double persist_frac() {
    static const double v = [] {
        const char *e = getenv("PANO_PERSIST_FRAC");
        const double f = e ? atof(e) : 1.0;
        return f > 0.05 && f <= 1.0 ? f : 1.0;
    }();
    return v;
}

// PANO_EARLY_EXTREMA=1 (read per call): each large octave's extrema scan goes out on a third
// stream as soon as its DoG levels exist.  Measured on MI355X (same box): bit-exact
// but 1.44-1.46 ms per graph-replayed parrington stitch against 1.09 ms, 11.9 against 11.0 ms at
// 1080p -- the scan's waves take the CU slots the next octaves' short blur launches (the
// critical path) need -- so off by default.
bool early_extrema_enabled() {
    const char *e = getenv("PANO_EARLY_EXTREMA");
    return e && atoi(e) != 0;
}
}  // namespace

// The keypoint stage's counter block (allocated / grown here), for the pyramid's first
// kernel to zero in passing (gray_frames): the separate fill launch sat between the last
// blur and the extrema scan on the critical path.
int sift_kp_counters(pano_ctx *ctx, int32_t **p, size_t *words) {
    KpBufs b;
    const int rc = kp_bufs(ctx, b);
    if (rc) return rc;
    *p = ctx->counters;
    *words = b.cnt_ints;
    return PANO_OK;
}

int sift_early_extrema(pano_ctx *ctx, const pano_sift_params *p, int o) {
    if (!early_extrema_enabled() || o != ctx->early_oct + 1) return PANO_OK;
    if (extrema_min_h() <= 0 || ctx->oct_h[o] < extrema_min_h()) return PANO_OK;
    if (p->num_intervals + 2 < 3 || p->num_intervals + 2 > 7) return PANO_OK;   // the keypoint stage reports it
    if (ctx->h > 4096 || ctx->w > 4096) return PANO_OK;
    KpBufs b;
    int rc = kp_bufs(ctx, b);
    if (rc) return rc;
    if (ctx->early_oct < 0) {               // the counters start at zero before any scan
        rc = launch_fill(ctx, ctx->counters, 0, b.cnt_ints * sizeof(int32_t));
        if (rc) return rc;
    }
    if (!ctx->xside) {
        PANO_HIP(ctx, hipStreamCreateWithFlags(&ctx->xside, hipStreamNonBlocking));
        PANO_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_x_fork, hipEventDisableTiming));
        PANO_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_x_join, hipEventDisableTiming));
    }
    PANO_HIP(ctx, hipEventRecord(ctx->ev_x_fork, ctx->stream));
    PANO_HIP(ctx, hipStreamWaitEvent(ctx->xside, ctx->ev_x_fork, 0));
    const XArgs xa = x_args(ctx, p->border);
    rc = launch_extrema_stream(ctx, p, xa, b, xa.item_start[o], xa.item_start[o + 1], ctx->xside);
    if (rc) return rc;
    PANO_HIP(ctx, hipEventRecord(ctx->ev_x_join, ctx->xside));
    ctx->x_pending = true;
    ctx->early_oct = o;
    return PANO_OK;
}

namespace {
int launch_descriptors(pano_ctx *ctx, const pano_sift_params *p, const PyrArgs &pa, const pano_kp *kps,
                       const int32_t *counts, int cap, int32_t *desc_work, float *desc, uint8_t *desc_u8,
                       int32_t *norms, const RawKp *rawk);

// raw_out != NULL: find_scale_space_extrema only (stops after the orientations and writes the
// raw keypoints in scan order to raw_out [n][cap]; kps / desc unused)
int sift_keypoints_impl(pano_ctx *ctx, const pano_sift_params *p, pano_kp *kps, float *desc,
                        uint8_t *desc_u8, int32_t *norms, int cap, int32_t *counts, pano_kp *raw_out) {
    const int n = ctx->n, no = ctx->n_oct, nl = ctx->n_lvl, ni = p->num_intervals;
    // octaves 0 .. early whose extrema the pyramid already launched (sift_early_extrema)
    const int early = ctx->early_oct;
    ctx->early_oct = -1;
    if (cap <= 0 || !counts || (!raw_out && (!kps || (!desc && !(desc_u8 && norms)))))
        return pano_fail(ctx, PANO_E_ARG, "pano_sift: bad outputs");
    if (n > PANO_MAX_FRAMES) return pano_fail(ctx, PANO_E_ARG, "pano_sift: more than PANO_MAX_FRAMES frames");
    KpBufs kb;
    int rc = kp_bufs(ctx, kb);
    if (rc) return rc;
    const size_t ext_cap = kb.ext_cap, cand_cap = kb.cand_cap, raw_cap = kb.raw_cap;
    uint64_t *raw_ext = kb.raw_ext;
    int32_t *err = kb.err, *cand_cnt = kb.cand_cnt, *raw_cnt = kb.raw_cnt, *ext_cnt = kb.ext_cnt;
    int32_t *desc_work = kb.desc_work, *ori_work = kb.ori_work;
    if (early < 0 && !ctx->kp_zeroed) {     // else gray_frames zeroed them this call
        rc = launch_fill(ctx, ctx->counters, 0, kb.cnt_ints * sizeof(int32_t));
        if (rc) return rc;
    }
    ctx->kp_zeroed = false;

    LocParams lp;
    lp.thresh = floor(0.5 * p->contrast_threshold / ni * 255);
    lp.contrast = (float)p->contrast_threshold;
    lp.edge_lhs = (float)p->eigen_ratio;
    lp.edge_rhs = (float)((p->eigen_ratio + 1) * (p->eigen_ratio + 1));
    lp.sigma_f = (float)p->sigma;
    lp.ni = ni;
    lp.border = p->border;
    lp.max_iter = p->max_iter;
    lp.octave = 0;
    DogArgs da{};
    int tiles = 0;
    da.n_oct = no;
    for (int o = 0; o < no; ++o) {
        da.H[o] = ctx->oct_h[o];
        da.W[o] = ctx->oct_w[o];
        for (int l = 0; l < nl - 1; ++l) da.dog[o][l] = ctx->dog + ctx->dog_off[o][l];
        const int iw = da.W[o] - 2 * p->border, ih = da.H[o] - 2 * p->border;
        da.tile_start[o] = tiles;
        da.tiles_x[o] = iw > 0 ? (iw + ETX - 1) / ETX : 1;
        if (iw > 0 && ih > 0) tiles += da.tiles_x[o] * ((ih + ETY - 1) / ETY);
    }
    da.tile_start[no] = tiles;
    if (ctx->h > 4096 || ctx->w > 4096)
        return pano_fail(ctx, PANO_E_UNSUPPORTED, "frames above 4096 px per side (the keypoint sort's buckets)");
    // Extrema: the streaming kernel for the large octaves (a wave walks 32 rows of a strip),
    // the LDS-tiled scan for the small ones (few rows: more, shorter workgroups win); the
    // octaves of a pending blur tail are scanned after the join.
    if (tiles > 0) {
        const XArgs xa = x_args(ctx, p->border);
        const int xmin_h = extrema_min_h();
        const int o_split = ctx->tail_pending ? ctx->o_tail : no;
        int o_s = 0;
        while (xmin_h > 0 && o_s < o_split && da.H[o_s] >= xmin_h) ++o_s;
        auto launch_scan = [&](int t0, int t1) -> int {
            if (t1 <= t0) return PANO_OK;
            dim3 grid(t1 - t0, n);
            {
                PanoProf prof_(ctx, PK_EXTREMA);
#define PANO_EXTREMA(NLV) extrema_scan<NLV><<<grid, 256, 0, ctx->stream>>>(da, p->border, lp.thresh, \
                                                                raw_ext, ext_cnt, (int)ext_cap, t0)
                switch (ni + 2) {            // DoG levels per octave
                    case 3: PANO_EXTREMA(3); break;
                    case 4: PANO_EXTREMA(4); break;
                    case 5: PANO_EXTREMA(5); break;
                    case 6: PANO_EXTREMA(6); break;
                    case 7: PANO_EXTREMA(7); break;
                    default: return pano_fail(ctx, PANO_E_UNSUPPORTED, "num_intervals above 5");
                }
#undef PANO_EXTREMA
            }
            PANO_LAUNCH_CHECK(ctx, "extrema_scan");
            return PANO_OK;
        };
        rc = launch_extrema_stream(ctx, p, xa, kb, xa.item_start[std::min(early + 1, o_s)], xa.item_start[o_s],
                                   ctx->stream);
        if (rc) return rc;
        rc = launch_scan(da.tile_start[o_s], da.tile_start[o_split]);
        if (rc) return rc;
        sift_join_tail(ctx);
        rc = launch_scan(da.tile_start[o_split], tiles);
        if (rc) return rc;
        sift_join_x(ctx);
        dim3 g2(n, (unsigned)((ext_cap + 255) / 256));
        {
            PanoProf prof_(ctx, PK_EXTREMA);
            localize<<<g2, 256, 0, ctx->stream>>>(da, lp, raw_ext, ext_cnt, (int)ext_cap, ctx->cands,
                                                  cand_cnt, (int)cand_cap);
        }
        PANO_LAUNCH_CHECK(ctx, "localize");
    }
    sift_join_tail(ctx);                  // orientation / descriptors read every octave
    PyrArgs pa{};
    pa.n_oct = no;
    pa.n_lvl = nl;
    for (int o = 0; o < no; ++o) {
        pa.H[o] = ctx->oct_h[o];
        pa.W[o] = ctx->oct_w[o];
        for (int l = 0; l < nl; ++l) pa.gauss[o][l] = ctx->pyr + ctx->gauss_off[o][l];
    }
    OriParams op{p->scale_factor, p->radius_factor, p->peak_ratio, ori_fast_bin()};
    const int nb = ctx->oct_w[0] + 1;                   // sort: floor(x) buckets over the base width
    const size_t per = raw_cap * n;
    rc = pano_grow(ctx, (void **)&ctx->sorted, &ctx->sorted_bytes, (3 * per + (size_t)nb * n) * sizeof(uint32_t));
    if (rc) return rc;
    uint32_t *mem = ctx->sorted + per;
    int32_t *bslot = (int32_t *)(ctx->sorted + 2 * per);
    int32_t *bstart = (int32_t *)(ctx->sorted + 3 * per);
    {
        static int ori_resident = 0;
        if (!ori_resident) {
            int per_cu = 0, cus = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, orientation, 256, 0) != hipSuccess ||
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess ||
                per_cu <= 0 || cus <= 0)
                per_cu = 4, cus = 256;
            ori_resident = per_cu * cus;
        }
        const size_t slots = ((size_t)n * cand_cap + 3) / 4;
        const unsigned blocks = (unsigned)std::max<size_t>(
            8, std::min<size_t>((slots + 7) & ~size_t(7), (size_t)(ori_resident * persist_frac()) & ~size_t(7)));
        {
            PanoProf prof_(ctx, PK_ORIENT);
            orientation<<<blocks, 256, 0, ctx->stream>>>(pa, op, ctx->cands, cand_cnt, (int)cand_cap, n, ori_work,
                                                         ctx->raw, raw_cnt, (int)raw_cap);
        }
        PANO_LAUNCH_CHECK(ctx, "orientation");
    }
    if (raw_out) {
        dim3 grid((unsigned)((raw_cap + 255) / 256), n);
        {
            PanoProf prof_(ctx, PK_SORT);
            raw_scan_order<<<grid, 256, 0, ctx->stream>>>(ctx->raw, raw_cnt, (int)raw_cap, raw_out, cap, counts, err,
                                                          ext_cnt, (int)ext_cap, cand_cnt, (int)cand_cap);
        }
        PANO_LAUNCH_CHECK(ctx, "raw_scan_order");
        return PANO_OK;
    }
    // PANO_DESC_RAW=1 (read per call; u8 descriptors): the descriptors of the raw keypoints
    // in orientation's order, with the sort (bucket_build, bucket_rank) on the side stream
    // beside them; emit_keypoints then writes the kept keypoints AND their descriptor rows in
    // sorted order.  A descriptor is a function of its keypoint alone, so the bytes are the
    // sorted-order kernel's; duplicates (dropped by emit) cost a descriptor each.  Measured on
    // MI355X (graph-replayed parrington): bit-identical but 0.997-1.002 against
    // 0.986 ms -- the side-stream sort is starved by the persistent descriptor grid (bucket_rank
    // 206 us beside it), the fork and join cost ~9 us each in the replayed graph, and the
    // per-frame row copy makes emit 26 us instead of 8.5.  Off by default.
    const char *dr_env = getenv("PANO_DESC_RAW");
    const bool desc_raw = desc_u8 && norms && dr_env && atoi(dr_env) != 0;
    if (desc_raw) {
        dim3 grid(n, (unsigned)((raw_cap + 255) / 256));
        if (nb > kSortMaxBuckets) return pano_fail(ctx, PANO_E_UNSUPPORTED, "frame too wide for the keypoint sort");
        const size_t dbytes = per * PANO_DESC_DIM, nbytes = per * sizeof(int32_t);
        rc = pano_grow(ctx, (void **)&ctx->descraw, &ctx->descraw_bytes, dbytes + nbytes);
        if (rc) return rc;
        uint8_t *draw = ctx->descraw;
        int32_t *nraw = (int32_t *)(ctx->descraw + dbytes);
        if (!ctx->side) PANO_HIP(ctx, hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking));
        if (!ctx->ev_sort_fork) {
            PANO_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_sort_fork, hipEventDisableTiming));
            PANO_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_sort_join, hipEventDisableTiming));
        }
        PANO_HIP(ctx, hipEventRecord(ctx->ev_sort_fork, ctx->stream));
        PANO_HIP(ctx, hipStreamWaitEvent(ctx->side, ctx->ev_sort_fork, 0));
        {
            PanoProf prof_(ctx, PK_SORT, ctx->side);
            bucket_build<<<n, kSortThreads, 0, ctx->side>>>(ctx->raw, raw_cnt, (int)raw_cap, nb, bstart, bslot, mem);
        }
        PANO_LAUNCH_CHECK(ctx, "bucket_build");
        {
            PanoProf prof_(ctx, PK_SORT, ctx->side);
            bucket_rank<<<grid, 256, 0, ctx->side>>>(ctx->raw, raw_cnt, (int)raw_cap, nb, bstart, mem, ctx->sorted);
        }
        PANO_LAUNCH_CHECK(ctx, "bucket_rank");
        PANO_HIP(ctx, hipEventRecord(ctx->ev_sort_join, ctx->side));
        rc = launch_descriptors(ctx, p, pa, nullptr, raw_cnt, (int)raw_cap, desc_work, nullptr, draw, nraw, ctx->raw);
        if (rc) return rc;
        PANO_HIP(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_sort_join, 0));
        {
            PanoProf prof_(ctx, PK_SORT);
            // bslot (bucket_build's scratch) holds emit's position -> raw index map
            emit_keypoints<<<n, kSortThreads, 0, ctx->stream>>>(ctx->raw, raw_cnt, (int)raw_cap, ctx->sorted, kps, cap,
                                                                counts, err, ext_cnt, (int)ext_cap, cand_cnt,
                                                                (int)cand_cap, draw, nraw, desc_u8, norms, bslot);
        }
        PANO_LAUNCH_CHECK(ctx, "emit_keypoints");
        return PANO_OK;
    }
    {
        dim3 grid(n, (unsigned)((raw_cap + 255) / 256));       // bucket_rank: (frame, block)
        if (nb > kSortMaxBuckets) return pano_fail(ctx, PANO_E_UNSUPPORTED, "frame too wide for the keypoint sort");
        {
            PanoProf prof_(ctx, PK_SORT);
            bucket_build<<<n, kSortThreads, 0, ctx->stream>>>(ctx->raw, raw_cnt, (int)raw_cap, nb, bstart, bslot, mem);
        }
        PANO_LAUNCH_CHECK(ctx, "bucket_build");
        {
            PanoProf prof_(ctx, PK_SORT);
            bucket_rank<<<grid, 256, 0, ctx->stream>>>(ctx->raw, raw_cnt, (int)raw_cap, nb, bstart, mem,
                                                       ctx->sorted);
        }
        PANO_LAUNCH_CHECK(ctx, "bucket_rank");
        {
            PanoProf prof_(ctx, PK_SORT);
            emit_keypoints<<<n, kSortThreads, 0, ctx->stream>>>(ctx->raw, raw_cnt, (int)raw_cap, ctx->sorted,
                                                        kps, cap, counts, err, ext_cnt, (int)ext_cap,
                                                        cand_cnt, (int)cand_cap);
        }
        PANO_LAUNCH_CHECK(ctx, "emit_keypoints");
    }
    return launch_descriptors(ctx, p, pa, kps, counts, cap, desc_work, desc, desc_u8, norms);
}

// generate_descriptors over kps [n][cap] / counts [n] on the pyramid pa: persistent waves over
// the batch's keypoints, exactly the workgroups that are resident at once (a second partial
// round would leave the first round's CUs idle).  desc_work: 8 zeroed per-XCD queue counters.
int launch_descriptors(pano_ctx *ctx, const pano_sift_params *p, const PyrArgs &pa, const pano_kp *kps,
                       const int32_t *counts, int cap, int32_t *desc_work, float *desc, uint8_t *desc_u8,
                       int32_t *norms, const RawKp *rawk) {
    const int n = ctx->n;
    DescParams dp{(float)(p->scale_multiplier * 0.5), (float)p->descriptor_max};
    // processing order: 0 the emit order (default); 1 locality (plane + 16-row band; measured on
    // MI355X, DESIGN.md 3: 253 -> 262 us per parrington step); 2 largest window first (the
    // persistent waves' tail then holds the small keypoints)
    static const int use_order = [] {
        const char *e = getenv("PANO_DESC_ORDER");
        return e ? atoi(e) : 0;
    }();
    int32_t *order = nullptr;
    if (use_order && !rawk) {
        OrderArgs oa{};
        oa.n_oct = pa.n_oct;
        oa.n_lvl = pa.n_lvl;
        int nb = 0;
        for (int o = 0; o < pa.n_oct; ++o) {
            oa.bstart[o] = nb;
            oa.nband[o] = (pa.H[o] + 15) / 16;
            nb += pa.n_lvl * oa.nband[o];
        }
        oa.bstart[pa.n_oct] = nb;
        oa.nb = nb;
        oa.hw_mult = dp.hw_mult;
        if (use_order == 2) {
            oa.by_size = 1;
            oa.nb = nb = kOrderHalves;
        }
        if (nb <= kSortMaxBuckets) {
            int rc = pano_grow(ctx, (void **)&ctx->dorder, &ctx->dorder_bytes, (size_t)n * cap * sizeof(int32_t));
            if (rc) return rc;
            order = ctx->dorder;
            {
                PanoProf prof_(ctx, PK_DESC);
                desc_order<<<n, kSortThreads, 0, ctx->stream>>>(kps, counts, cap, oa, order);
            }
            PANO_LAUNCH_CHECK(ctx, "desc_order");
        }
    }
    const int occ = desc_occ((long long)pa.H[0] * pa.W[0]);
    static int resident[2] = {0, 0};
    int &res = resident[occ == 4];
    if (!res) {
        int per_cu = 0, cus = 0;
        const hipError_t e = occ == 4
            ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, descriptor_wave<true, 4>, 64 * kDescWaves, 0)
            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, descriptor_wave<true, 3>, 64 * kDescWaves, 0);
        if (e != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess ||
            per_cu <= 0 || cus <= 0)
            per_cu = 4, cus = 256;
        res = per_cu * cus;
    }
    const size_t slots = ((size_t)n * cap + kDescWaves - 1) / kDescWaves;
    const unsigned blocks = (unsigned)std::max<size_t>(
        8, std::min<size_t>((slots + 7) & ~size_t(7), (size_t)(res * persist_frac()) & ~size_t(7)));
    {
        PanoProf prof_(ctx, PK_DESC);
        auto go = [&](auto occ_c) {
            constexpr int O = decltype(occ_c)::value;
            if (rawk)
                descriptor_wave<true, O, true><<<blocks, 64 * kDescWaves, 0, ctx->stream>>>(
                    pa, dp, nullptr, counts, n, cap, desc_work, nullptr, desc_u8, norms, nullptr, rawk);
            else if (desc_u8)
                descriptor_wave<true, O><<<blocks, 64 * kDescWaves, 0, ctx->stream>>>(
                    pa, dp, kps, counts, n, cap, desc_work, nullptr, desc_u8, norms, order);
            else
                descriptor_wave<false, O><<<blocks, 64 * kDescWaves, 0, ctx->stream>>>(
                    pa, dp, kps, counts, n, cap, desc_work, desc, nullptr, nullptr, order);
        };
        if (occ == 4) go(std::integral_constant<int, 4>{});
        else go(std::integral_constant<int, 3>{});
    }
    PANO_LAUNCH_CHECK(ctx, "descriptor");
    return PANO_OK;
}
}  // namespace

int launch_sift_keypoints(pano_ctx *ctx, const pano_sift_params *p, pano_kp *kps, float *desc,
                          uint8_t *desc_u8, int32_t *norms, int cap, int32_t *counts) {
    return sift_keypoints_impl(ctx, p, kps, desc, desc_u8, norms, cap, counts, nullptr);
}

int launch_sift_extrema(pano_ctx *ctx, const pano_sift_params *p, pano_kp *raw, int cap, int32_t *counts) {
    if (!raw) return pano_fail(ctx, PANO_E_ARG, "pano_sift_extrema: bad outputs");
    return sift_keypoints_impl(ctx, p, nullptr, nullptr, nullptr, nullptr, cap, counts, raw);
}

int launch_sift_describe(pano_ctx *ctx, const pano_sift_params *p, const pano_kp *kps, const int32_t *counts,
                         int cap, float *desc) {
    if (!kps || !counts || !desc || cap <= 0) return pano_fail(ctx, PANO_E_ARG, "pano_sift_describe: bad arguments");
    if (!ctx->pyr || ctx->n <= 0) return pano_fail(ctx, PANO_E_ARG, "pano_sift_describe: no resident pyramid");
    if (!ctx->pyr_full)
        return pano_fail(ctx, PANO_E_UNSUPPORTED, "pano_sift_describe needs every Gaussian level (pano_sift_pyramid)");
    sift_join_tail(ctx);
    const size_t cnt_ints = (3 * (size_t)ctx->n + 1 + 16) * kCntStride;
    int rc = pano_grow(ctx, (void **)&ctx->counters, &ctx->counters_n, cnt_ints * sizeof(int32_t));
    if (rc) return rc;
    int32_t *desc_work = ctx->counters + (3 * (size_t)ctx->n + 1) * kCntStride;
    rc = launch_fill(ctx, desc_work, 0, 8 * kCntStride * sizeof(int32_t));
    if (rc) return rc;
    PyrArgs pa{};
    pa.n_oct = ctx->n_oct;
    pa.n_lvl = ctx->n_lvl;
    for (int o = 0; o < ctx->n_oct; ++o) {
        pa.H[o] = ctx->oct_h[o];
        pa.W[o] = ctx->oct_w[o];
        for (int l = 0; l < ctx->n_lvl; ++l) pa.gauss[o][l] = ctx->pyr + ctx->gauss_off[o][l];
    }
    return launch_descriptors(ctx, p, pa, kps, counts, cap, desc_work, desc, nullptr, nullptr);
}

int sift_set_attributes(pano_ctx *) { return PANO_OK; }

// pano_sift_localize / pano_sift_orient (argument checks in pano_abi.cpp)
int launch_sift_localize(pano_ctx *ctx, const pano_sift_params *p, const float *const *dog, int h, int w,
                         int octave, const int32_t *cand, int n, pano_kp *out, int32_t *layer_out) {
    if (n <= 0) return PANO_OK;
    LocParams lp;
    const int ni = p->num_intervals;
    lp.thresh = floor(0.5 * p->contrast_threshold / ni * 255);
    lp.contrast = (float)p->contrast_threshold;
    lp.edge_lhs = (float)p->eigen_ratio;
    lp.edge_rhs = (float)((p->eigen_ratio + 1) * (p->eigen_ratio + 1));
    lp.sigma_f = (float)p->sigma;
    lp.ni = ni;
    lp.border = p->border;
    lp.max_iter = p->max_iter;
    lp.octave = octave;
    DogArgs da{};
    da.n_oct = octave + 1;
    da.H[octave] = h;
    da.W[octave] = w;
    for (int l = 0; l < ni + 2; ++l) da.dog[octave][l] = dog[l];
    {
        PanoProf prof_(ctx, PK_EXTREMA);
        localize_list<<<(n + 255) / 256, 256, 0, ctx->stream>>>(da, lp, octave, cand, n, out, layer_out);
    }
    PANO_LAUNCH_CHECK(ctx, "localize_list");
    return PANO_OK;
}

int launch_sift_orient(pano_ctx *ctx, const pano_sift_params *p, const float *gauss, int h, int w, int octave,
                       const pano_kp *kps, int n, pano_kp *out, int32_t *counts) {
    if (n <= 0) return PANO_OK;
    OriParams op{p->scale_factor, p->radius_factor, p->peak_ratio, ori_fast_bin()};
    const unsigned blocks = (unsigned)std::min(4096, (n + 3) / 4);
    {
        PanoProf prof_(ctx, PK_ORIENT);
        orient_list<<<blocks, 256, 0, ctx->stream>>>(gauss, h, w, octave, op, kps, n, out, counts);
    }
    PANO_LAUNCH_CHECK(ctx, "orient_list");
    return PANO_OK;
}
