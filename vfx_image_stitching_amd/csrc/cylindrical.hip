// cylindrical.hip -- C1: cylindrical_projection (image_stitching_sift.py:117-136).
//
// The reference is a FORWARD scatter in row-major source order: out[y', x'] = in[y, x]
// with x' = round(f*atan(xd/f)) + w//2, y' = round(f*yd/sqrt(xd^2+f^2)) + h//2 (fp64,
// Python round = half-even), so for colliding destinations the last writer (largest
// row-major source index) wins and unwritten pixels stay 0.
//
// gfx950 formulation: the map is inverted instead of scattered.  Both coordinate maps are
// monotone (x' in xd through atan, y' in yd for a fixed xd), so the sources that land on a
// destination pixel form a small box of consecutive candidates around the inverse images
// f tan(k/f) and k den/f; every candidate is re-checked with the forward formula itself
// (the same f64 operations and rounding), and the winner is the candidate with the largest
// row-major index -- the reference's last writer.  cyl_columns resolves the candidate
// source columns of every destination column once per frame; cyl_inverse then writes every
// destination pixel once (no winner map, no atomics, no memset) and raises the per-column
// "any non-zero byte" flag the compositor needs (blend_two_images, :185-189).
// Roofline unit C1 = 6 B/pixel algorithmic: 3 read + 3 written.
// (The scatter form, cyl_scatter + cyl_gather over an atomicMax winner map, is kept as the
// checked alternative: PANO_CYL_SCATTER=1.)
#include "pano_internal.h"

namespace {

constexpr int kFocalChunk = 256;
struct FocalArg {
    double f[kFocalChunk];   // passed by value: no host->device copy inside the stream order
};

__global__ void __launch_bounds__(256)
cyl_scatter(int32_t *__restrict__ win, int h, int w, FocalArg focal, uint8_t *__restrict__ colnz) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int f = blockIdx.z;
    if (x >= w || y >= h) return;
    if (colnz && y == 0) colnz[(size_t)f * w + x] = 0;   // cyl_gather sets the non-zero columns
    const double fl = focal.f[f];
    const int cx = w / 2, cy = h / 2;
    const int xd = x - cx, yd = y - cy;
    const double xm_d = rint(fl * atan((double)xd / fl));
    const int xm = (int)xm_d + cx;
    const double den = sqrt((double)xd * (double)xd + fl * fl);
    const int ym = (int)rint(fl * ((double)yd / den)) + cy;
    if (xm < 0 || xm >= w || ym < 0 || ym >= h) return;
    atomicMax(&win[(size_t)f * h * w + (size_t)ym * w + xm], y * w + x);
}

__global__ void __launch_bounds__(256)
cyl_gather(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
           const int32_t *__restrict__ win, uint8_t *__restrict__ colnz, int h, int w) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int f = blockIdx.z;
    if (x >= w || y >= h) return;
    const size_t plane = (size_t)h * w;
    const int32_t s = win[f * plane + (size_t)y * w + x];
    uint8_t b = 0, g = 0, r = 0;
    if (s >= 0 && (size_t)s < plane) {
        const uint8_t *p = src + (f * plane + s) * 3;
        b = p[0];
        g = p[1];
        r = p[2];
    }
    uint8_t *q = dst + (f * plane + (size_t)y * w + x) * 3;
    q[0] = b;
    q[1] = g;
    q[2] = r;
    if (colnz && (b | g | r)) colnz[(size_t)f * w + x] = 1;
}

// Source-column range [lo, hi] of destination column x' (inclusive; empty if lo > hi),
// exact: every candidate of a conservative box around f tan((k +- 1/2)/f) is tested with
// the forward map.  Also zeroes the column's non-zero flag (cyl_inverse raises it).
__global__ void __launch_bounds__(256)
cyl_columns(int w, FocalArg focal, int2 *__restrict__ cols, uint8_t *__restrict__ colnz,
            double2 *__restrict__ colden) {
    const int xp = blockIdx.x * 256 + threadIdx.x, f = blockIdx.y;
    if (xp >= w) return;
    const double fl = focal.f[f];
    const int cx = w / 2, k = xp - cx;
    {
        // per SOURCE column x = xp: 1 / sqrt(xd^2 + f^2) and sqrt(xd^2 + f^2) / f, the row
        // map's column constants (cyl_inverse reads them instead of recomputing per pixel)
        const double den = sqrt((double)k * (double)k + fl * fl);
        colden[(size_t)f * w + xp] = make_double2(1.0 / den, den / fl);
    }
    // inverse images of k -+ 1/2 (arguments kept inside the atan range; clamped to the frame)
    const double lim = 1.5707963267948966 - 1e-12;
    const double ta = fmax(fmin((k - 0.5) / fl, lim), -lim), tb = fmax(fmin((k + 0.5) / fl, lim), -lim);
    // both ends clamped to the frame's column range before the integer conversion (near the
    // atan limit fl * tan() reaches ~fl * 1e12, outside int)
    const double lo_c = -cx - 2.0, hi_c = (double)(w - cx + 1);
    const double a = fmin(fmax(fl * tan(ta), lo_c), hi_c), b = fmin(fmax(fl * tan(tb), lo_c), hi_c);
    const int c0 = (int)floor(a) - 1, c1 = (int)ceil(b) + 1;
    int lo = 1, hi = 0;
    for (int xd = c0; xd <= c1; ++xd) {
        const int x = xd + cx;
        if (x < 0 || x >= w) continue;
        const int xm = (int)rint(fl * atan((double)xd / fl)) + cx;
        if (xm != xp) continue;
        if (lo > hi) lo = x;
        hi = x;
    }
    cols[(size_t)f * w + xp] = make_int2(lo, hi);
    if (colnz) colnz[(size_t)f * w + xp] = 0;
}

// cyl_columns by source column: the column map x' = rint(f atan(xd / f)) + w/2 is monotone
// (its slope 1 / (1 + (xd / f)^2) dwarfs any f64 rounding), so the sources of destination
// column x' are a run [lo, hi] of consecutive source columns.  Thread x evaluates the map at
// x - 1, x, x + 1 -- the same expression as cyl_columns' candidate test -- and writes lo of
// its run (and the column's zeroed non-zero flag) where the run starts, hi where it ends, and
// the empty range (1, 0) for destination columns no source reaches (the gaps after its
// value; thread 0 also the columns before the first).  One f64 atan per evaluation instead of
// a search over a candidate box per destination column; the column constants as before.
__device__ __forceinline__ int col_map(double fl, int x, int cx) {
    return (int)rint(fl * atan((double)(x - cx) / fl)) + cx;
}

__global__ void __launch_bounds__(256)
cyl_columns_run(int w, FocalArg focal, int *__restrict__ cols, uint8_t *__restrict__ colnz,
                double2 *__restrict__ colden) {
    const int x = blockIdx.x * 256 + threadIdx.x, f = blockIdx.y;
    if (x >= w) return;
    const double fl = focal.f[f];
    const int cx = w / 2, k = x - cx;
    int *fc = cols + 2 * (size_t)f * w;            // int2 [w]: .x = lo, .y = hi
    uint8_t *fz = colnz ? colnz + (size_t)f * w : nullptr;
    {
        const double den = sqrt((double)k * (double)k + fl * fl);
        colden[(size_t)f * w + x] = make_double2(1.0 / den, den / fl);
    }
    const int a = col_map(fl, x, cx);
    const int p = x > 0 ? col_map(fl, x - 1, cx) : -0x40000000;
    const int b = x + 1 < w ? col_map(fl, x + 1, cx) : 0x40000000;
    if (a >= 0 && a < w) {
        if (p != a) {
            fc[2 * a] = x;
            if (fz) fz[a] = 0;
        }
        if (b != a) fc[2 * a + 1] = x;
    }
    // destination columns strictly between a and b (and before the first source's) are empty
    const int g0 = max(x == 0 ? 0 : a + 1, 0), g1 = min(b, w);
    for (int kk = g0; kk < g1; ++kk) {
        if (kk == a) continue;
        fc[2 * kk] = 1;
        fc[2 * kk + 1] = 0;
        if (fz) fz[kk] = 0;
    }
}

// The forward row map of source row yd in source column x (xd = x - w/2): rint(f (yd / den))
// in f64.  yd * (1 / den) is within a few ulp of the quotient, so its rounding is the same
// unless the product lies within 1e-9 of a half-integer; there the exact expression decides
// (the reference's division).
__device__ __forceinline__ int row_map(double fl, int yd, double inv_den, int xd) {
    const double v = fl * ((double)yd * inv_den);
    const double t = v - floor(v);
    if (fabs(t - 0.5) < 1e-9) {
        const double den = sqrt((double)xd * (double)xd + fl * fl);
        return (int)rint(fl * ((double)yd / den));
    }
    return (int)rint(v);
}

// Largest row-major source index landing on destination pixel (xp, yp) by the per-pixel
// candidate search (cyl_inverse's form; cyl_tile's fallback for very wide column ranges).
template <typename CD>
__device__ long search_best(int2 cr, CD cd, int xp, int yp, int h, int w, double fl) {
    const int cy = h / 2, k = yp - cy;
    long best = -1;
    for (int x = cr.x; x <= cr.y; ++x) {
        const double2 ds = cd(x);
        const double s = ds.y;
        const int r1 = (int)ceil((k + 0.5) * s) + 1, r0 = (int)floor((k - 0.5) * s) - 1;
        for (int yd = r1; yd >= r0; --yd) {
            const int y = yd + cy;
            if (y < 0 || y >= h) continue;
            if (row_map(fl, yd, ds.x, x - w / 2) + cy != yp) continue;
            const long li = (long)y * w + x;
            if (li > best) best = li;
            break;
        }
    }
    return best;
}

// Tile form of the inverse map: a workgroup owns 64 x 32 destination pixels.  Their
// candidate source columns (cyl_columns) form one range of <= kTC columns; per source column
// the rows whose forward row map can reach the tile's rows are a bound from den / f; every
// such source pixel is mapped ONCE with the exact forward formula and recorded as the largest
// source row per (destination row, source column) in an LDS table (LDS atomicMax).  Each
// destination pixel then reads 1-2 table entries instead of searching ~4 rows per candidate
// column with the f64 map (cyl_inverse: ~half of its 29 us at parrington was that search).
// The winner is still the largest row-major source index: the reference's last writer.
constexpr int kTX = 64, kTY = 32, kTC = 128, kRMax = 64;

// the row map's column constants of source column x: (1 / den, den / f), den = sqrt(xd^2 + f^2)
__device__ __forceinline__ double2 col_consts(double fl, int x, int cx) {
    const int k = x - cx;
    const double den = sqrt((double)k * (double)k + fl * fl);
    return make_double2(1.0 / den, den / fl);
}

// FUSED (the default): the tile derives its destination columns' source runs and the window's
// column constants itself -- col_map at every window column (and one either side), a run's
// ends where the map changes -- instead of reading cyl_columns_run's tables: one launch per
// frame batch instead of two.  Where the window cannot hold a tile column's whole run (strong
// distortion) each run comes from two binary searches over the monotone map.  The per-column
// non-zero flag is the OR over the column strip's row tiles: each tile ORs its columns into a
// u32 flag (device atomics), counts itself in on the strip, and the strip's last tile reads the
// flags back (sc1 loads), writes colnz and re-zeroes flags and counter for the next launch.
struct CylSync {
    uint32_t *flags;                     // [n][w]
    int32_t *cnt;                        // [n][strips]
};

template <bool FUSED>
__global__ void __launch_bounds__(256)
cyl_tile(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, const int2 *__restrict__ cols,
         const double2 *__restrict__ colden, uint8_t *__restrict__ colnz, int h, int w, FocalArg focal,
         CylSync sync) {
    __shared__ int T[kTY][kTC];
    __shared__ int2 cr[kTX];
    __shared__ int ylo_s[kTC], nrow_s[kTC];
    __shared__ int xs_s[2], fb_s, cov_s, last_s;
    __shared__ unsigned char nz_s[4][kTX];
    __shared__ double2 cd_s[kTC];
    __shared__ int m_s[kTC + 2];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int f = blockIdx.z, xp0 = blockIdx.x * kTX, yp0 = blockIdx.y * kTY;
    const double fl = focal.f[f];
    const int cx = w / 2, cy = h / 2;
    const int2 *fc = FUSED ? nullptr : cols + (size_t)f * w;
    const double2 *cd = FUSED ? nullptr : colden + (size_t)f * w;
    // the source columns' constants for a window from the inverse column map of the tile's
    // first column (f tan((x' - 1/2) / f), as cyl_columns bounds it), loaded together with the
    // tile's column ranges: one global round trip instead of two
    const double lim = 1.5707963267948966 - 1e-12;
    const double ta = fmax(fmin((xp0 - cx - 0.5) / fl, lim), -lim);
    const int wx0 = max((int)fmin(fmax(floor(fl * tan(ta)), -(double)cx - 2.0), (double)w) + cx - 2, 0);
    if constexpr (FUSED) {
        // m_s[t] = col_map(window column t - 1), out-of-frame columns as +-infinity
        if (tid < kTC + 2) {
            const int x = wx0 - 1 + tid;
            m_s[tid] = x < 0 ? -0x40000000 : (x >= w ? 0x40000000 : col_map(fl, x, cx));
        }
        if (tid >= kTC + 2 && tid < kTC + 2 + kTX) cr[tid - kTC - 2] = make_int2(1, 0);
        if (tid < kTC && wx0 + tid < w) cd_s[tid] = col_consts(fl, wx0 + tid, cx);
        if (tid == 0) cov_s = 1;
        __syncthreads();
        // runs of the tile's columns inside the window; covered iff the map leaves the tile's
        // column range on both sides of the window (or the window reaches the frame's edge)
        if (tid == 0) {
            const int lo_ok = wx0 == 0 || m_s[0] < xp0;
            const int hi_ok = wx0 + kTC >= w || m_s[kTC + 1] >= min(xp0 + kTX, w);
            cov_s = lo_ok && hi_ok;
        }
        if (tid >= 1 && tid <= kTC) {
            const int x = wx0 - 1 + tid, a = m_s[tid];
            if (x < w && a >= xp0 && a < xp0 + kTX && a < w) {
                if (m_s[tid - 1] != a) cr[a - xp0].x = x;
                if (m_s[tid + 1] != a) cr[a - xp0].y = x;
            }
        }
        __syncthreads();
        if (!cov_s && tid < kTX && xp0 + tid < w) {
            // the run of column xp0 + tid by two binary searches of the monotone map
            const int a = xp0 + tid;
            int lo = 0, hi = w;                      // first x with map(x) >= a
            while (lo < hi) { const int mid = (lo + hi) >> 1; if (col_map(fl, mid, cx) >= a) hi = mid; else lo = mid + 1; }
            int lo2 = lo, hi2 = w;                   // first x with map(x) > a
            while (lo2 < hi2) { const int mid = (lo2 + hi2) >> 1; if (col_map(fl, mid, cx) > a) hi2 = mid; else lo2 = mid + 1; }
            cr[tid] = lo < lo2 ? make_int2(lo, lo2 - 1) : make_int2(1, 0);
        }
    } else {
        if (tid < kTX) cr[tid] = xp0 + tid < w ? fc[xp0 + tid] : make_int2(1, 0);
        else if (tid - kTX < kTC && wx0 + tid - kTX < w) cd_s[tid - kTX] = cd[wx0 + tid - kTX];
    }
    for (int i = tid; i < kTY * kTC; i += 256) (&T[0][0])[i] = -1;
    if (tid == 0) fb_s = 0;
    __syncthreads();
    if (wv == 0) {
        const int2 c = cr[lane];
        int lo = c.x <= c.y ? c.x : 0x7fffffff, hi = c.x <= c.y ? c.y : -1;
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) {
            lo = min(lo, __shfl_xor(lo, d));
            hi = max(hi, __shfl_xor(hi, d));
        }
        if (lane == 0) { xs_s[0] = lo; xs_s[1] = hi; }
    }
    __syncthreads();
    const int xs0 = xs_s[0], ncols = xs_s[1] >= xs0 ? xs_s[1] - xs0 + 1 : 0;
    // source column x's constants: from the LDS window when it holds them
    const bool in_win = xs0 >= wx0 && xs0 + ncols <= wx0 + kTC && xs0 + ncols <= w;
    auto cdx = [&](int x) { return in_win ? cd_s[x - wx0] : (FUSED ? col_consts(fl, x, cx) : cd[x]); };
    if (ncols > kTC) {
        if (tid == 0) fb_s = 1;
    } else {
        // per source column: the rows whose forward map can land in [yp0, yp0 + kTY)
        const int k0 = yp0 - cy, k1 = min(yp0 + kTY, h) - 1 - cy;
        for (int c = tid; c < ncols; c += 256) {
            const double sc = cdx(xs0 + c).y;                      // den / f >= 1
            const int lo = max((int)floor((k0 - 0.5) * sc) - 1 + cy, 0);
            const int hi = min((int)ceil((k1 + 0.5) * sc) + 1 + cy, h - 1);
            ylo_s[c] = lo;
            nrow_s[c] = hi >= lo ? hi - lo + 1 : 0;
            if (hi - lo + 1 > kRMax) fb_s = 1;
        }
    }
    __syncthreads();
    const bool fb = fb_s != 0;
    if (!fb && ncols > 0) {
        // every candidate source pixel once: thread -> (column tid % ncols, rows tid / ncols +
        // k * per).  The row map in f32 first: its error is below 1e-6 |v| + 1e-6, so away from
        // a half-integer its rounding is the f64 map's; within 1e-3 of one the f64 map decides
        const int per = 256 / ncols;                 // >= 2 (ncols <= kTC)
        const int c = tid % ncols, r0 = tid / ncols;
        if (r0 < per) {
            const int x = xs0 + c, nr = nrow_s[c], y0 = ylo_s[c];
            const double inv_den = cdx(x).x;
            const float inv32 = (float)inv_den, fl32 = (float)fl;
            for (int r = r0; r < nr; r += per) {
                const int y = y0 + r, yd = y - cy;
                const float v = fl32 * ((float)yd * inv32);
                const float t = v - floorf(v);
                int ym;
                if (fabsf(t - 0.5f) < fmaxf(1e-3f, fabsf(v) * 1e-6f)) ym = row_map(fl, yd, inv_den, x - cx) + cy;
                else ym = (int)rintf(v) + cy;
                if (ym >= yp0 && ym < yp0 + kTY && ym < h) atomicMax(&T[ym - yp0][c], y);
            }
        }
    }
    __syncthreads();
    // thread -> 4 consecutive columns (quad q) x rows rr and rr + 16: the 12 bytes of a quad's
    // row go out as 3 dword stores (w % 4 == 0), and when its 4 winners are consecutive source
    // pixels (the common case: one source column per destination column, same row) they come
    // in as one 16-byte aligned-down load instead of 12 byte loads
    const int q = tid & 15, rr = tid >> 4;
    const int xq = xp0 + 4 * q;
    const size_t plane3 = (size_t)h * w * 3;
    const uint8_t *fs = src + (size_t)f * plane3;
    const size_t src_end = (size_t)gridDim.z * plane3 - (size_t)f * plane3;   // bytes past fs
    const bool vec = (w & 3) == 0 && xq + 3 < w;
    int nzq[4] = {0, 0, 0, 0};
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        const int yp = yp0 + rr + 16 * half;
        if (yp >= h || xq >= w) continue;
        int best[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            long b = -1;
            const int xp = xq + j;
            if (xp < w) {
                const int2 c = cr[4 * q + j];
                if (!fb) {
                    for (int x = c.x; x <= c.y; ++x) {
                        const int y = T[yp - yp0][x - xs0];
                        const long li = (long)y * w + x;
                        if (y >= 0 && li > b) b = li;
                    }
                } else if constexpr (FUSED) {
                    b = search_best(c, [&](int x) { return col_consts(fl, x, cx); }, xp, yp, h, w, fl);
                } else {
                    b = search_best(c, [&](int x) { return cd[x]; }, xp, yp, h, w, fl);
                }
            }
            best[j] = (int)b;                        // h * w < 2^31 (launch_cylindrical)
        }
        uint8_t px[4][3];
        const size_t a = (size_t)max(best[0], 0) * 3, a4 = a & ~(size_t)3;
        const bool run = best[0] >= 0 && best[1] == best[0] + 1 && best[2] == best[0] + 2 &&
                         best[3] == best[0] + 3 && a4 + 16 <= src_end;
        if (run) {
            const uint32_t *p4 = (const uint32_t *)(fs + a4);
            const uint32_t d0 = p4[0], d1 = p4[1], d2 = p4[2], d3 = p4[3];
            const int sh = 8 * (int)(a - a4);
            const uint32_t e[3] = {(uint32_t)((((uint64_t)d1 << 32) | d0) >> sh),
                                   (uint32_t)((((uint64_t)d2 << 32) | d1) >> sh),
                                   (uint32_t)((((uint64_t)d3 << 32) | d2) >> sh)};
#pragma unroll
            for (int k = 0; k < 12; ++k) px[k / 3][k % 3] = (uint8_t)(e[k >> 2] >> (8 * (k & 3)));
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                // loads from a clamped address, zeroed afterwards (no branch per load)
                const uint8_t *p = fs + (size_t)max(best[j], 0) * 3;
                const uint8_t b0 = p[0], b1 = p[1], b2 = p[2];
                const bool hit = best[j] >= 0;
                px[j][0] = hit ? b0 : 0;
                px[j][1] = hit ? b1 : 0;
                px[j][2] = hit ? b2 : 0;
            }
        }
        uint8_t *qd = dst + (((size_t)f * h + yp) * w + xq) * 3;
        if (vec) {
            uint32_t o[3] = {0u, 0u, 0u};
#pragma unroll
            for (int k = 0; k < 12; ++k) o[k >> 2] |= (uint32_t)px[k / 3][k % 3] << (8 * (k & 3));
            uint32_t *q4 = (uint32_t *)qd;
            q4[0] = o[0];
            q4[1] = o[1];
            q4[2] = o[2];
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (xq + j < w) { qd[3 * j] = px[j][0]; qd[3 * j + 1] = px[j][1]; qd[3 * j + 2] = px[j][2]; }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) nzq[j] |= px[j][0] | px[j][1] | px[j][2];
    }
    // per-column "any non-zero byte": OR over the tile's rows in LDS (nz_s reused as flags)
    unsigned int *nzc = (unsigned int *)&nz_s[0][0];          // kTX flags (4 x kTX bytes)
    if (tid < kTX) nzc[tid] = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (nzq[j]) nzc[4 * q + j] = 1;                          // same value from every writer
    __syncthreads();
    if constexpr (FUSED) {
        if (!colnz) return;
        typedef __attribute__((address_space(1))) uint32_t g_u32;
        typedef __attribute__((address_space(1))) int g_i32;
        uint32_t *fl_f = sync.flags + (size_t)f * w;
        if (tid < kTX && xp0 + tid < w && nzc[tid]) atomicOr(fl_f + xp0 + tid, 1u);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // every wave: its ORs performed
        __syncthreads();
        int32_t *cnt = sync.cnt + (size_t)f * gridDim.x + blockIdx.x;
        if (tid == 0) {
            fold_release();
            last_s = __hip_atomic_fetch_add((g_i32 *)cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                     (int)gridDim.y - 1;
        }
        __syncthreads();
        if (!last_s) return;
        fold_acquire();
        if (tid < kTX && xp0 + tid < w) {
            const uint32_t v = __hip_atomic_load((g_u32 *)(fl_f + xp0 + tid), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            colnz[(size_t)f * w + xp0 + tid] = v ? 1 : 0;
            __hip_atomic_store((g_u32 *)(fl_f + xp0 + tid), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (tid == 0) __hip_atomic_store((g_i32 *)cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        if (colnz && tid < kTX && xp0 + tid < w && nzc[tid]) colnz[(size_t)f * w + xp0 + tid] = 1;
    }
}

__global__ void __launch_bounds__(256)
cyl_inverse(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, const int2 *__restrict__ cols,
            const double2 *__restrict__ colden, uint8_t *__restrict__ colnz, int h, int w, FocalArg focal) {
    const int xp = blockIdx.x * 64 + (threadIdx.x & 63);
    const int yp = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int f = blockIdx.z;
    if (xp >= w || yp >= h) return;
    const double fl = focal.f[f];
    const int cy = h / 2, k = yp - cy;
    const int2 cr = cols[(size_t)f * w + xp];
    long best = -1;                                   // largest row-major source index
    for (int x = cr.x; x <= cr.y; ++x) {
        const double2 ds = colden[(size_t)f * w + x];
        const double inv_den = ds.x, s = ds.y;
        // rows whose forward y' can be k: a box around [(k - 1/2) s, (k + 1/2) s], scanned
        // from the top (the first hit is this column's largest row)
        const int r1 = (int)ceil((k + 0.5) * s) + 1, r0 = (int)floor((k - 0.5) * s) - 1;
        for (int yd = r1; yd >= r0; --yd) {
            const int y = yd + cy;
            if (y < 0 || y >= h) continue;
            // the forward map rint(f (yd / den)) in f64: yd * (1 / den) is within a few ulp of
            // the quotient, so its rounding is the same unless the product lies within 1e-9 of
            // a half-integer; there the exact expression decides (the reference's division)
            const double v = fl * ((double)yd * inv_den);
            const double t = v - floor(v);
            double ymd;
            if (fabs(t - 0.5) < 1e-9) {
                const int xd = x - w / 2;
                const double den = sqrt((double)xd * (double)xd + fl * fl);
                ymd = rint(fl * ((double)yd / den));
            } else {
                ymd = rint(v);
            }
            const int ym = (int)ymd + cy;
            if (ym != yp) continue;
            const long li = (long)y * w + x;
            if (li > best) best = li;
            break;
        }
    }
    uint8_t b = 0, g = 0, r = 0;
    if (best >= 0) {
        const uint8_t *p = src + ((size_t)f * h * w + (size_t)best) * 3;
        b = p[0];
        g = p[1];
        r = p[2];
    }
    uint8_t *q = dst + (((size_t)f * h + yp) * w + xp) * 3;
    q[0] = b;
    q[1] = g;
    q[2] = r;
    if (colnz && (b | g | r)) colnz[(size_t)f * w + xp] = 1;
}

}  // namespace

int launch_cylindrical(pano_ctx *ctx, const uint8_t *src, uint8_t *dst, int n, int h, int w,
                       const double *h_focal, uint8_t *colnz) {
    if (n <= 0 || h <= 0 || w <= 0 || !src || !dst || !h_focal)
        return pano_fail(ctx, PANO_E_ARG, "pano_cylindrical: bad arguments");
    if ((long long)h * w >= (1LL << 31)) return pano_fail(ctx, PANO_E_ARG, "frame too large");
    const size_t plane = (size_t)h * w;
    static const bool scatter_form = getenv("PANO_CYL_SCATTER") != nullptr;
    // the fused tile (default; PANO_CYL_TWO=1: cyl_columns_run + cyl_tile, read per call)
    const char *two_env = getenv("PANO_CYL_TWO");
    const bool fused = !scatter_form && !(two_env && atoi(two_env) != 0) && !getenv("PANO_CYL_PIXEL") &&
                       !getenv("PANO_CYL_COLSEARCH");
    if (fused) {
        const int strips = (w + kTX - 1) / kTX;
        const size_t need = (size_t)n * w * sizeof(uint32_t) + (size_t)n * strips * sizeof(int32_t);
        if (need > ctx->cyl_sync_bytes) {
            if (ctx->capturing) return pano_fail(ctx, PANO_E_UNSUPPORTED, "cylindrical counters grown inside a graph capture");
            if (ctx->cyl_sync) {
                PANO_HIP(ctx, hipStreamSynchronize(ctx->stream));
                (void)hipFree(ctx->cyl_sync);
                ctx->cyl_sync = nullptr;
                ctx->cyl_sync_bytes = 0;
                ++ctx->generation;
            }
            PANO_HIP(ctx, hipMalloc((void **)&ctx->cyl_sync, need));
            PANO_HIP(ctx, hipMemset(ctx->cyl_sync, 0, need));      // each launch re-zeroes
            ctx->cyl_sync_bytes = need;
        }
        uint32_t *flags = (uint32_t *)ctx->cyl_sync;
        int32_t *cnt = (int32_t *)(flags + (size_t)n * w);
        for (int f0 = 0; f0 < n; f0 += kFocalChunk) {
            const int nf = n - f0 < kFocalChunk ? n - f0 : kFocalChunk;
            FocalArg fa;
            for (int i = 0; i < nf; ++i) fa.f[i] = h_focal[f0 + i];
            CylSync cs{flags + (size_t)f0 * w, cnt + (size_t)f0 * strips};
            {
                PanoProf prof_(ctx, PK_CYL_GATHER);
                cyl_tile<true><<<dim3(strips, (h + kTY - 1) / kTY, nf), 256, 0, ctx->stream>>>(
                    src + f0 * plane * 3, dst + f0 * plane * 3, nullptr, nullptr,
                    colnz ? colnz + (size_t)f0 * w : nullptr, h, w, fa, cs);
            }
            PANO_LAUNCH_CHECK(ctx, "cyl_tile");
        }
        return PANO_OK;
    }
    if (!scatter_form) {
        int rc = pano_grow(ctx, &ctx->bscratch, &ctx->bscratch_bytes, (size_t)n * w * (sizeof(int2) + sizeof(double2)));
        if (rc) return rc;
        double2 *colden = (double2 *)ctx->bscratch;                      // 16-byte aligned first
        int2 *cols = (int2 *)(colden + (size_t)n * w);
        for (int f0 = 0; f0 < n; f0 += kFocalChunk) {
            const int nf = n - f0 < kFocalChunk ? n - f0 : kFocalChunk;
            FocalArg fa;
            for (int i = 0; i < nf; ++i) fa.f[i] = h_focal[f0 + i];
            static const bool col_search = getenv("PANO_CYL_COLSEARCH") != nullptr;   // A/B
            if (col_search) {
                PanoProf prof_(ctx, PK_CYL_SCATTER);
                cyl_columns<<<dim3((w + 255) / 256, nf), 256, 0, ctx->stream>>>(
                    w, fa, cols + (size_t)f0 * w, colnz ? colnz + (size_t)f0 * w : nullptr, colden + (size_t)f0 * w);
            } else {
                PanoProf prof_(ctx, PK_CYL_SCATTER);
                cyl_columns_run<<<dim3((w + 255) / 256, nf), 256, 0, ctx->stream>>>(
                    w, fa, (int *)(cols + (size_t)f0 * w), colnz ? colnz + (size_t)f0 * w : nullptr,
                    colden + (size_t)f0 * w);
            }
            PANO_LAUNCH_CHECK(ctx, "cyl_columns");
            static const bool per_pixel = getenv("PANO_CYL_PIXEL") != nullptr;   // A/B: the search form
            if (per_pixel) {
                PanoProf prof_(ctx, PK_CYL_GATHER);
                cyl_inverse<<<dim3((w + 63) / 64, (h + 3) / 4, nf), 256, 0, ctx->stream>>>(
                    src + f0 * plane * 3, dst + f0 * plane * 3, cols + (size_t)f0 * w, colden + (size_t)f0 * w,
                    colnz ? colnz + (size_t)f0 * w : nullptr, h, w, fa);
            } else {
                PanoProf prof_(ctx, PK_CYL_GATHER);
                cyl_tile<false><<<dim3((w + kTX - 1) / kTX, (h + kTY - 1) / kTY, nf), 256, 0, ctx->stream>>>(
                    src + f0 * plane * 3, dst + f0 * plane * 3, cols + (size_t)f0 * w, colden + (size_t)f0 * w,
                    colnz ? colnz + (size_t)f0 * w : nullptr, h, w, fa, CylSync{});
            }
            PANO_LAUNCH_CHECK(ctx, "cyl_inverse");
        }
        return PANO_OK;
    }
    const size_t need = plane * n * sizeof(int32_t);
    int rc = pano_grow(ctx, &ctx->bscratch, &ctx->bscratch_bytes, need);
    if (rc) return rc;
    int32_t *win = (int32_t *)ctx->bscratch;
    rc = launch_fill(ctx, win, 0xFF, plane * n * sizeof(int32_t));
    if (rc) return rc;
    for (int f0 = 0; f0 < n; f0 += kFocalChunk) {
        const int nf = n - f0 < kFocalChunk ? n - f0 : kFocalChunk;
        FocalArg fa;
        for (int i = 0; i < nf; ++i) fa.f[i] = h_focal[f0 + i];
        dim3 grid((w + 63) / 64, (h + 3) / 4, nf);
        {
            PanoProf prof_(ctx, PK_CYL_SCATTER);
            cyl_scatter<<<grid, 256, 0, ctx->stream>>>(win + f0 * plane, h, w, fa,
                                                       colnz ? colnz + (size_t)f0 * w : nullptr);
        }
        PANO_LAUNCH_CHECK(ctx, "cyl_scatter");
        {
            PanoProf prof_(ctx, PK_CYL_GATHER);
            cyl_gather<<<grid, 256, 0, ctx->stream>>>(src + f0 * plane * 3, dst + f0 * plane * 3,
                                                      win + f0 * plane,
                                                      colnz ? colnz + (size_t)f0 * w : nullptr, h, w);
        }
        PANO_LAUNCH_CHECK(ctx, "cyl_gather");
    }
    return PANO_OK;
}
