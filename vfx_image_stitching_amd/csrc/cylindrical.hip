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
    if (!scatter_form) {
        int rc = pano_grow(ctx, &ctx->bscratch, &ctx->bscratch_bytes, (size_t)n * w * (sizeof(int2) + sizeof(double2)));
        if (rc) return rc;
        double2 *colden = (double2 *)ctx->bscratch;                      // 16-byte aligned first
        int2 *cols = (int2 *)(colden + (size_t)n * w);
        for (int f0 = 0; f0 < n; f0 += kFocalChunk) {
            const int nf = n - f0 < kFocalChunk ? n - f0 : kFocalChunk;
            FocalArg fa;
            for (int i = 0; i < nf; ++i) fa.f[i] = h_focal[f0 + i];
            {
                PanoProf prof_(ctx, PK_CYL_SCATTER);
                cyl_columns<<<dim3((w + 255) / 256, nf), 256, 0, ctx->stream>>>(
                    w, fa, cols + (size_t)f0 * w, colnz ? colnz + (size_t)f0 * w : nullptr, colden + (size_t)f0 * w);
            }
            PANO_LAUNCH_CHECK(ctx, "cyl_columns");
            {
                PanoProf prof_(ctx, PK_CYL_GATHER);
                cyl_inverse<<<dim3((w + 63) / 64, (h + 3) / 4, nf), 256, 0, ctx->stream>>>(
                    src + f0 * plane * 3, dst + f0 * plane * 3, cols + (size_t)f0 * w, colden + (size_t)f0 * w,
                    colnz ? colnz + (size_t)f0 * w : nullptr, h, w, fa);
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
