// cylindrical.hip -- C1: cylindrical_projection (image_stitching_sift.py:117-136).
//
// The reference is a FORWARD scatter in row-major source order: out[y', x'] = in[y, x]
// with x' = round(f*atan(xd/f)) + w//2, y' = round(f*yd/sqrt(xd^2+f^2)) + h//2 (fp64,
// Python round = half-even), so for colliding destinations the last writer (largest
// row-major source index) wins and unwritten pixels stay 0.
//
// gfx950 formulation: pass 1 scatters the source linear index with atomicMax into an
// int32 winner map (one 4-byte atomic per source pixel), pass 2 gathers 3 bytes per
// destination pixel and raises the per-column "any non-zero byte" flag the compositor
// needs (blend_two_images counts non-zeros per column, :185-189).
// Bytes per frame pixel: 3 read (scatter: none of the pixel data) + 4 atomic + 4 read +
// 3 gathered + 3 written  ->  roofline unit C1 = 6 B/pixel algorithmic.
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

}  // namespace

int launch_cylindrical(pano_ctx *ctx, const uint8_t *src, uint8_t *dst, int n, int h, int w,
                       const double *h_focal, uint8_t *colnz) {
    if (n <= 0 || h <= 0 || w <= 0 || !src || !dst || !h_focal)
        return pano_fail(ctx, PANO_E_ARG, "pano_cylindrical: bad arguments");
    if ((long long)h * w >= (1LL << 31)) return pano_fail(ctx, PANO_E_ARG, "frame too large");
    const size_t plane = (size_t)h * w;
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
