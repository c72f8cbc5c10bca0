// harris.hip -- H1..H3: the Harris feature path of image_stitching_harris.py.
//
//   conv2d / gradients       :49-61, :150-158  Ix = g[y,x-1]-g[y,x+1], Iy = g[y-1,x]-g[y+1,x]
//                                              (edge padding; exact integers in f64)
//   HarrisCorner             :135-185  21x21 sigma=2 Gaussian (f64, reflect-101) of Ix^2,
//                                      Iy^2, IxIy; R = det - 0.05 tr^2; 2 %-of-max threshold,
//                                      3x3 NMS with R == max; stable sort by R desc; top 200
//   calc_orientation         :63-70
//   gen_descriptor           :72-133   16x16 top-left-anchored patch, 9x9 sigma=4.5 blur,
//                                      8-bin main orientation, 4x4x8 histogram, 2x normalise
//   compute_keypoints_and_descriptors_harris :187-214  (8-px border filter AFTER the top 200)
//
// Exactness: the f64 blurs accumulate tap by tap as two roundings (multiply, add) like the
// oracle's numpy expression; the f32 histograms are updated in the reference's sequential
// order (one lane), the norms reproduce OpenBLAS's sdot order.  Only f64 atan2 ulps can
// differ from numpy, which moves a 45-degree bin only within ~1e-13 of its edge.
#include "pano_internal.h"

namespace {

constexpr int HT = 32;          // output tile of the 21x21 blur
constexpr int kSel = 8192;      // NMS candidates per frame (sort capacity)

struct Taps21 { double k[21]; };
struct Taps9 { double k[9]; };

__global__ void to_gray(const uint8_t *__restrict__ bgr, uint8_t *__restrict__ gray, size_t npx) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < npx) gray[i] = gray_u8(bgr + i * 3);
}

__device__ __forceinline__ double grad_prod(const uint8_t *g, int h, int w, int y, int x, int ch) {
    const int xl = x > 0 ? x - 1 : 0, xr = x < w - 1 ? x + 1 : w - 1;
    const int yu = y > 0 ? y - 1 : 0, yd = y < h - 1 ? y + 1 : h - 1;
    const double ix = (double)g[(size_t)y * w + xl] - (double)g[(size_t)y * w + xr];
    const double iy = (double)g[(size_t)yu * w + x] - (double)g[(size_t)yd * w + x];
    return ch == 0 ? ix * ix : (ch == 1 ? iy * iy : ix * iy);
}

// blockIdx.z = frame * 3 + channel (Ixx, Iyy, Ixy)
__global__ void __launch_bounds__(256)
structure_blur(const uint8_t *__restrict__ gray, int h, int w, Taps21 t, double *__restrict__ S) {
    constexpr int R = 10, IW = HT + 2 * R;
    __shared__ double tin[IW * IW];
    __shared__ double trow[IW * HT];
    const int f = blockIdx.z / 3, ch = blockIdx.z % 3;
    const uint8_t *g = gray + (size_t)f * h * w;
    const int x0 = blockIdx.x * HT, y0 = blockIdx.y * HT, tid = threadIdx.x;
    for (int i = tid; i < IW * IW; i += 256) {
        const int ty = i / IW, tx = i - ty * IW;
        tin[i] = grad_prod(g, h, w, reflect101(y0 - R + ty, h), reflect101(x0 - R + tx, w), ch);
    }
    __syncthreads();
    for (int i = tid; i < IW * HT; i += 256) {
        const int ty = i / HT, tx = i - ty * HT;
        double acc = 0.0;
        for (int k = 0; k < 21; ++k) acc = acc + t.k[k] * tin[ty * IW + tx + k];
        trow[i] = acc;
    }
    __syncthreads();
    for (int i = tid; i < HT * HT; i += 256) {
        const int ty = i / HT, tx = i - ty * HT;
        const int gy = y0 + ty, gx = x0 + tx;
        if (gy >= h || gx >= w) continue;
        double acc = 0.0;
        for (int k = 0; k < 21; ++k) acc = acc + t.k[k] * trow[(ty + k) * HT + tx];
        S[(((size_t)ch * gridDim.z / 3 + f) * h + gy) * w + gx] = acc;
    }
}

__device__ __forceinline__ unsigned long long dsortable(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double dunsortable(unsigned long long s) {
    const unsigned long long b = (s >> 63) ? (s & 0x7fffffffffffffffull) : ~s;
    return __longlong_as_double((long long)b);
}

__global__ void __launch_bounds__(256)
response(const double *__restrict__ S, int n, int h, int w, double k, double *__restrict__ R,
         unsigned long long *__restrict__ fmax) {
    __shared__ unsigned long long red[256];
    const int f = blockIdx.y, tid = threadIdx.x;
    const size_t plane = (size_t)h * w;
    const double *sxx = S + (size_t)f * plane;
    const double *syy = S + ((size_t)n + f) * plane;
    const double *sxy = S + ((size_t)2 * n + f) * plane;
    unsigned long long m = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + tid; i < plane; i += (size_t)gridDim.x * 256) {
        const double a = sxx[i], b = syy[i], c = sxy[i];
        const double det = (a * b) - (c * c);
        const double tr = a + b;
        const double r = det - k * (tr * tr);
        R[(size_t)f * plane + i] = r;
        const unsigned long long s = dsortable(r);
        m = s > m ? s : m;
    }
    red[tid] = m;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (tid < off) red[tid] = red[tid] > red[tid + off] ? red[tid] : red[tid + off];
        __syncthreads();
    }
    if (tid == 0) atomicMax(&fmax[f], red[0]);
}

struct HCand {
    double r;
    int32_t y, x;
};

__global__ void __launch_bounds__(256)
nms(const double *__restrict__ R, int h, int w, double ratio,
    const unsigned long long *__restrict__ frame_max, HCand *__restrict__ cands,
    int32_t *__restrict__ cnt) {
    const int f = blockIdx.z;
    const int x = 1 + blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = 1 + blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= w - 1 || y >= h - 1) return;
    const double thr = dunsortable(frame_max[f]) * ratio;
    const double *Rf = R + (size_t)f * h * w;
    const double v = Rf[(size_t)y * w + x];
    if (!(v > thr)) return;
    double mx = v;
    for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) mx = fmax(mx, Rf[(size_t)(y + dy) * w + x + dx]);
    if (!(v == mx)) return;
    const int slot = atomicAdd(&cnt[f], 1);
    if (slot < kSel) cands[(size_t)f * kSel + slot] = HCand{v, y, x};
}

// per frame: stable sort by R desc (ties: row-major scan order), top max_points, then the
// 8-pixel border filter, in that order (image_stitching_harris.py:183-209)
__global__ void __launch_bounds__(1024)
select_top(const HCand *__restrict__ cands, const int32_t *__restrict__ cnt, int h, int w,
           int max_points, int32_t *__restrict__ xy, int32_t *__restrict__ counts,
           int32_t *__restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    unsigned long long *key = (unsigned long long *)smem_raw;
    uint32_t *sec = (uint32_t *)(key + kSel);
    const int f = blockIdx.x, tid = threadIdx.x;
    const int c = cnt[f];
    if (c > kSel) {
        if (tid == 0) { err[0] = PANO_E_OVERFLOW; counts[f] = -1; }
        return;
    }
    const HCand *cf = cands + (size_t)f * kSel;
    int n2 = 1;
    while (n2 < c) n2 <<= 1;
    for (int i = tid; i < n2; i += 1024) {
        if (i < c) {
            key[i] = ~dsortable(cf[i].r);                       // R descending
            sec[i] = (uint32_t)(cf[i].y * w + cf[i].x);          // then scan order
        } else {
            key[i] = ~0ull;
            sec[i] = 0xFFFFFFFFu;
        }
    }
    __syncthreads();
    for (int kk = 2; kk <= n2; kk <<= 1)
        for (int j = kk >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < n2; i += 1024) {
                const int l = i ^ j;
                if (l <= i) continue;
                const bool asc = (i & kk) == 0;
                const bool lt = key[l] < key[i] || (key[l] == key[i] && sec[l] < sec[i]);
                if (asc == lt) {
                    const unsigned long long tk = key[i]; key[i] = key[l]; key[l] = tk;
                    const uint32_t ts = sec[i]; sec[i] = sec[l]; sec[l] = ts;
                }
            }
            __syncthreads();
        }
    if (tid == 0) {
        int m = 0;
        const int top = c < max_points ? c : max_points;
        for (int r = 0; r < top; ++r) {
            const int yy = (int)(sec[r] / w), xx = (int)(sec[r] % w);
            if (yy < 8 || yy >= h - 8 || xx < 8 || xx >= w - 8) continue;
            xy[((size_t)f * max_points + m) * 2] = xx;
            xy[((size_t)f * max_points + m) * 2 + 1] = yy;
            ++m;
        }
        counts[f] = m;
    }
}

__device__ float sdot_skx128(const float *x) {
    float a16[4][16];
    for (int k = 0; k < 4; ++k)
        for (int j = 0; j < 16; ++j) a16[k][j] = 0.0f;
    for (int i = 0; i < 128; i += 64)
        for (int k = 0; k < 4; ++k)
            for (int j = 0; j < 16; ++j) {
                const float t = x[i + 16 * k + j];
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
    float hh[4];
    for (int j = 0; j < 4; ++j) hh[j] = v[j] + v[j + 4];
    return (hh[0] + hh[1]) + (hh[2] + hh[3]);
}

__device__ __forceinline__ int hbin(double ang) {
    const double a = np_remainder(ang, 360.0);
    return ((int)((a / 360.0) * 8.0)) % 8;
}

// one wave per corner, 4 corners per workgroup
__global__ void __launch_bounds__(256)
harris_desc(const uint8_t *__restrict__ gray, int h, int w, Taps9 t9,
            const int32_t *__restrict__ xy, const int32_t *__restrict__ counts, int max_points,
            float *__restrict__ desc) {
    __shared__ double pm[4][256], pt[4][256], tmp[4][256];
    __shared__ float dsc[4][128];
    __shared__ float nrm[4];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int f = blockIdx.y;
    const int k = blockIdx.x * 4 + wv;
    const int cnt = min(counts[f], max_points);
    if ((int)blockIdx.x * 4 >= cnt) return;
    const bool active = k < cnt;
    const uint8_t *g = gray + (size_t)f * h * w;
    int cx = 0, cy = 0;
    if (active) {
        cx = min(max(xy[((size_t)f * max_points + k) * 2], 0), w - 1);
        cy = min(max(xy[((size_t)f * max_points + k) * 2 + 1], 0), h - 1);
        for (int e = lane; e < 256; e += 64) {
            const int i = e >> 4, j = e & 15;
            int yy = cy + i, xx = cx + j;
            yy = yy < h ? yy : h - 1;
            xx = xx < w ? xx : w - 1;
            const int xl = xx > 0 ? xx - 1 : 0, xr = xx < w - 1 ? xx + 1 : w - 1;
            const int yu = yy > 0 ? yy - 1 : 0, yd = yy < h - 1 ? yy + 1 : h - 1;
            const double ix = (double)g[(size_t)yy * w + xl] - (double)g[(size_t)yy * w + xr];
            const double iy = (double)g[(size_t)yu * w + xx] - (double)g[(size_t)yd * w + xx];
            pm[wv][e] = sqrt(ix * ix + iy * iy);
            const double th = atan2(iy, ix) * 180.0 / 3.141592653589793;
            pt[wv][e] = np_remainder(th + 360.0, 360.0);
        }
    }
    __syncthreads();
    if (active)
        for (int e = lane; e < 256; e += 64) {   // 9-tap row pass, reflect-101 in the patch
            const int i = e >> 4, j = e & 15;
            double acc = 0.0;
            for (int q = 0; q < 9; ++q) acc = acc + t9.k[q] * pm[wv][i * 16 + reflect101(j + q - 4, 16)];
            tmp[wv][e] = acc;
        }
    __syncthreads();
    if (active)
        for (int e = lane; e < 256; e += 64) {
            const int i = e >> 4, j = e & 15;
            double acc = 0.0;
            for (int q = 0; q < 9; ++q) acc = acc + t9.k[q] * tmp[wv][reflect101(i + q - 4, 16) * 16 + j];
            pm[wv][e] = acc;
        }
    __syncthreads();
    __shared__ double mainth[4];
    if (active && lane == 0) {
        float hst[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int e = 0; e < 256; ++e) {
            const int b = hbin(pt[wv][e]);
            hst[b] = (float)((double)hst[b] + pm[wv][e]);
        }
        int am = 0;
        for (int b = 1; b < 8; ++b)
            if (hst[b] > hst[am]) am = b;
        mainth[wv] = (am + 0.5) * (360.0 / 8);
    }
    __syncthreads();
    if (active)
        for (int e = lane; e < 256; e += 64) pt[wv][e] = np_remainder((pt[wv][e] - mainth[wv]) + 360.0, 360.0);
    __syncthreads();
    if (active && lane < 16) {
        const int by = lane >> 2, bx = lane & 3;
        float hst[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int yy = 0; yy < 4; ++yy)
            for (int xx = 0; xx < 4; ++xx) {
                const int e = (by * 4 + yy) * 16 + bx * 4 + xx;
                const int b = hbin(pt[wv][e]);
                hst[b] = (float)((double)hst[b] + pm[wv][e]);
            }
        for (int b = 0; b < 8; ++b) dsc[wv][lane * 8 + b] = hst[b];
    }
    __syncthreads();
    if (active && lane == 0) nrm[wv] = sqrtf(sdot_skx128(dsc[wv])) + 1e-7f;
    __syncthreads();
    if (active)
        for (int e = lane; e < 128; e += 64) {
            float v = dsc[wv][e] / nrm[wv];
            v = v < 0.0f ? 0.0f : (v > 0.2f ? 0.2f : v);
            dsc[wv][e] = v;
        }
    __syncthreads();
    if (active && lane == 0) nrm[wv] = sqrtf(sdot_skx128(dsc[wv])) + 1e-7f;
    __syncthreads();
    if (active)
        for (int e = lane; e < 128; e += 64)
            desc[((size_t)f * max_points + k) * PANO_DESC_DIM + e] = dsc[wv][e] / nrm[wv];
}

template <int N>
void gauss_f64(double sigma, double *out) {
    const double scale2x = -0.5 / (sigma * sigma);
    double s = 0.0;
    for (int i = 0; i < N; ++i) {
        const double x = i - (N - 1) * 0.5;
        out[i] = exp(scale2x * x * x);
        s += out[i];
    }
    s = 1.0 / s;
    for (int i = 0; i < N; ++i) out[i] = out[i] * s;
}

}  // namespace

int harris_set_attributes(pano_ctx *ctx) {
    const int sm = kSel * (sizeof(unsigned long long) + sizeof(uint32_t));
    PANO_HIP(ctx, hipFuncSetAttribute((const void *)select_top,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, sm));
    return PANO_OK;
}

int launch_harris(pano_ctx *ctx, const uint8_t *bgr, int n, int h, int w, int max_points,
                  int32_t *xy, float *desc, int32_t *counts) {
    if (n <= 0 || h < 3 || w < 3 || max_points <= 0 || !bgr || !xy || !desc || !counts)
        return pano_fail(ctx, PANO_E_ARG, "pano_harris: bad arguments");
    const size_t plane = (size_t)h * w;
    const size_t o_gray = 0;
    const size_t o_S = (o_gray + plane * n + 255) & ~size_t(255);
    const size_t o_R = o_S + 3 * plane * n * sizeof(double);
    const size_t o_max = o_R + plane * n * sizeof(double);
    const size_t o_cnt = o_max + (size_t)n * 8;
    const size_t o_err = o_cnt + (size_t)n * 4;
    const size_t o_c = (o_err + 64 + 255) & ~size_t(255);
    const size_t need = o_c + (size_t)n * kSel * sizeof(HCand);
    int rc = pano_grow(ctx, &ctx->hscratch, &ctx->hscratch_bytes, need);
    if (rc) return rc;
    char *base = (char *)ctx->hscratch;
    uint8_t *gray = (uint8_t *)(base + o_gray);
    double *S = (double *)(base + o_S);
    double *R = (double *)(base + o_R);
    unsigned long long *fmx = (unsigned long long *)(base + o_max);
    int32_t *cnt = (int32_t *)(base + o_cnt);
    int32_t *err = (int32_t *)(base + o_err);
    HCand *cands = (HCand *)(base + o_c);
    rc = launch_fill(ctx, base + o_max, 0, o_c - o_max);
    if (rc) return rc;
    {
        PanoProf prof_(ctx, PK_H_GRAY);
        to_gray<<<(unsigned)((plane * n + 255) / 256), 256, 0, ctx->stream>>>(bgr, gray, plane * n);
    }
    PANO_LAUNCH_CHECK(ctx, "to_gray");
    Taps21 t21;
    gauss_f64<21>(2.0, t21.k);
    dim3 gb((w + HT - 1) / HT, (h + HT - 1) / HT, 3 * n);
    {
        PanoProf prof_(ctx, PK_H_BLUR);
        structure_blur<<<gb, 256, 0, ctx->stream>>>(gray, h, w, t21, S);
    }
    PANO_LAUNCH_CHECK(ctx, "structure_blur");
    unsigned rb = (unsigned)((plane + 255) / 256);
    if (rb > 512) rb = 512;
    {
        PanoProf prof_(ctx, PK_H_RESP);
        response<<<dim3(rb, n), 256, 0, ctx->stream>>>(S, n, h, w, 0.05, R, fmx);
    }
    PANO_LAUNCH_CHECK(ctx, "response");
    dim3 gn((w - 2 + 63) / 64, (h - 2 + 3) / 4, n);
    {
        PanoProf prof_(ctx, PK_H_NMS);
        nms<<<gn, 256, 0, ctx->stream>>>(R, h, w, 0.02, fmx, cands, cnt);
    }
    PANO_LAUNCH_CHECK(ctx, "nms");
    const size_t sm = kSel * (sizeof(unsigned long long) + sizeof(uint32_t));
    {
        PanoProf prof_(ctx, PK_H_SELECT);
        select_top<<<n, 1024, sm, ctx->stream>>>(cands, cnt, h, w, max_points, xy, counts, err);
    }
    PANO_LAUNCH_CHECK(ctx, "select_top");
    Taps9 t9;
    gauss_f64<9>(1.5 * 3, t9.k);
    dim3 gd((max_points + 3) / 4, n);
    {
        PanoProf prof_(ctx, PK_H_DESC);
        harris_desc<<<gd, 256, 0, ctx->stream>>>(gray, h, w, t9, xy, counts, max_points, desc);
    }
    PANO_LAUNCH_CHECK(ctx, "harris_desc");
    return PANO_OK;
}
