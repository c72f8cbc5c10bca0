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
// Exactness (oracle/cv2_compat.py): taps are float32, pixels float32, so each
// product is exact in double; acc = fma(tap_i, x_i, acc) in tap order i = 0..n-1 is
// therefore bit-identical to the oracle's sequential double sum, and one rounding to f32
// per pass reproduces it exactly.  The x2 bilinear upsample of integer gray levels is exact.
#include "pano_internal.h"

namespace {

constexpr int TX = 64;
constexpr int TY = 64;

struct Taps {
    double k[PANO_MAX_TAPS];
    int n;
};

enum Mode { MODE_BASE = 0, MODE_LEVEL = 1, MODE_DOWN = 2 };

struct LoadArgs {
    const uint8_t *bgr;   // MODE_BASE: [n][sh][sw][3]
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

template <int MODE>
__device__ __forceinline__ float load_px(const LoadArgs &a, int f, int y, int x, int H, int W) {
    if constexpr (MODE == MODE_LEVEL) {
        return a.src[((size_t)f * H + y) * W + x];
    } else if constexpr (MODE == MODE_DOWN) {
        int sy = (int)floor(y * a.ify);
        int sx = (int)floor(x * a.ifx);
        sy = sy < a.sh - 1 ? sy : a.sh - 1;
        sx = sx < a.sw - 1 ? sx : a.sw - 1;
        return a.src[((size_t)f * a.sh + sy) * a.sw + sx];
    } else {
        // gray at (gy, gx) of the source frame, then x2 bilinear (exact for integers)
        int y0, y1, x0, x1;
        float wy, wx;
        lin_map(y, a.sh, y0, y1, wy);
        lin_map(x, a.sw, x0, x1, wx);
        const uint8_t *fr = a.bgr + (size_t)f * a.sh * a.sw * 3;
        const float g00 = gray_u8(fr + ((size_t)y0 * a.sw + x0) * 3);
        const float g01 = gray_u8(fr + ((size_t)y0 * a.sw + x1) * 3);
        const float g10 = gray_u8(fr + ((size_t)y1 * a.sw + x0) * 3);
        const float g11 = gray_u8(fr + ((size_t)y1 * a.sw + x1) * 3);
        const float wx0 = 1.0f - wx, wy0 = 1.0f - wy;
        const float h0 = g00 * wx0 + g01 * wx;
        const float h1 = g10 * wx0 + g11 * wx;
        return h0 * wy0 + h1 * wy;
    }
}

// Register-blocked sliding window: SEG consecutive outputs of one row (or column) from
// SEG + NT - 1 staged inputs; output j receives taps t = 0..NT-1 in order (the oracle's
// sequential sum), all index arithmetic compile-time after unrolling.
template <int NT, int SEG>
__device__ __forceinline__ void conv_seg(const float *__restrict__ p, int stride,
                                         const double *__restrict__ k, double (&acc)[SEG]) {
#pragma unroll
    for (int j = 0; j < SEG; ++j) acc[j] = 0.0;
#pragma unroll
    for (int i = 0; i < SEG + NT - 1; ++i) {
        const double v = (double)p[i * stride];
#pragma unroll
        for (int j = 0; j < SEG; ++j) {
            const int t = i - j;
            if (t >= 0 && t < NT) acc[j] = fma(k[t], v, acc[j]);
        }
    }
}

// Runtime tap count fallback (sigma values other than the reference defaults).
__device__ __forceinline__ double conv_one(const float *__restrict__ p, int stride,
                                           const double *__restrict__ k, int n) {
    double acc = 0.0;
    for (int t = 0; t < n; ++t) acc = fma(k[t], (double)p[t * stride], acc);
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
    const int x0 = blockIdx.x * TX, y0 = blockIdx.y * TY, f = blockIdx.z;
    const int tw = min(TX, W - x0), th = min(TY, H - y0);   // valid outputs of this tile
    const int IW = TX + 2 * r, IH = TY + 2 * r;
    const int IWP = IW | 1;                                  // odd row pitch: no bank conflicts
    float *tin = smem;                 // [IH][IWP]
    float *trow = smem + IH * IWP;     // [IH][TX]
    const int tid = threadIdx.x;
    const int ih = th + 2 * r, iw = tw + 2 * r;              // staged extent actually needed

    for (int i = tid; i < ih * iw; i += 256) {
        const int ty = i / iw, tx = i - ty * iw;
        const int gy = reflect101(y0 - r + ty, H);
        const int gx = reflect101(x0 - r + tx, W);
        tin[ty * IWP + tx] = load_px<MODE>(la, f, gy, gx, H, W);
    }
    __syncthreads();
    if constexpr (NT > 0) {
        // row pass: lanes walk consecutive rows (odd pitch), each SEG outputs along x
        const int nseg = (tw + SEG - 1) / SEG;
        for (int it = tid; it < ih * nseg; it += 256) {
            const int row = it % ih, sg = it / ih;
            double acc[SEG];
            conv_seg<NT, SEG>(tin + row * IWP + sg * SEG, 1, taps.k, acc);
#pragma unroll
            for (int j = 0; j < SEG; ++j) trow[row * TX + sg * SEG + j] = (float)acc[j];
        }
        __syncthreads();
        // column pass: lanes walk consecutive columns, each SEG outputs down y
        const int nrs = (th + SEG - 1) / SEG;
        for (int it = tid; it < tw * nrs; it += 256) {
            const int x = it % tw, rs = it / tw;
            double acc[SEG];
            conv_seg<NT, SEG>(trow + rs * SEG * TX + x, TX, taps.k, acc);
#pragma unroll
            for (int j = 0; j < SEG; ++j) {
                const int ty = rs * SEG + j;
                if (ty >= th) break;
                const float o = (float)acc[j];
                const size_t gi = ((size_t)f * H + y0 + ty) * W + x0 + x;
                out[gi] = o;
                const float c = tin[(ty + r) * IWP + x + r];
                if (dog) dog[gi] = o - c;
                if (in_copy) in_copy[gi] = c;
            }
        }
    } else {
        for (int i = tid; i < ih * tw; i += 256) {
            const int ty = i / tw, tx = i - ty * tw;
            trow[ty * TX + tx] = (float)conv_one(tin + ty * IWP + tx, 1, taps.k, n);
        }
        __syncthreads();
        for (int i = tid; i < th * tw; i += 256) {
            const int ty = i / tw, tx = i - ty * tw;
            const float o = (float)conv_one(trow + ty * TX + tx, TX, taps.k, n);
            const size_t gi = ((size_t)f * H + y0 + ty) * W + x0 + tx;
            out[gi] = o;
            const float c = tin[(ty + r) * IWP + tx + r];
            if (dog) dog[gi] = o - c;
            if (in_copy) in_copy[gi] = c;
        }
    }
}

// getGaussianKernel(ksize, sigma, CV_32F) (cv2_compat.getGaussianKernel): f32 taps widened.
Taps make_taps(double sigma) {
    Taps t;
    int n = (int)nearbyint(sigma * 4 * 2 + 1) | 1;
    if (n > PANO_MAX_TAPS) n = -1;
    t.n = n;
    if (n < 0) return t;
    const double scale2x = -0.5 / (sigma * sigma);
    float tf[PANO_MAX_TAPS];
    double s = 0.0;
    for (int i = 0; i < n; ++i) {
        const double x = i - (n - 1) * 0.5;
        tf[i] = (float)exp(scale2x * x * x);
        s += (double)tf[i];
    }
    s = 1.0 / s;
    for (int i = 0; i < n; ++i) t.k[i] = (double)(float)((double)tf[i] * s);
    return t;
}

size_t smem_bytes(const Taps &t) {
    const int r = (t.n - 1) / 2;
    // trow rows are read up to SEG past the valid extent by the column pass: pad them
    return (size_t)((TY + 2 * r) * ((TX + 2 * r) | 1) + (TY + 2 * r + SEG) * TX) * sizeof(float);
}

template <int MODE, int NT>
int launch_blur_nt(pano_ctx *ctx, const LoadArgs &la, float *out, float *dog, float *in_copy,
                   int n, int H, int W, const Taps &t) {
    dim3 grid((W + TX - 1) / TX, (H + TY - 1) / TY, n);
    const size_t sm = smem_bytes(t);
    if (sm > 65536)
        PANO_HIP(ctx, hipFuncSetAttribute((const void *)blur_level<MODE, NT>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm));
    {
        PanoProf prof_(ctx, PK_BLUR);
        blur_level<MODE, NT><<<grid, 256, sm, ctx->stream>>>(la, out, dog, in_copy, H, W, t);
    }
    PANO_LAUNCH_CHECK(ctx, "blur_level");
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

int sift_reserve_pyramid(pano_ctx *ctx, int n, int h, int w, const pano_sift_params *p) {
    int no, nl;
    double sb, sl[PANO_MAX_LEVELS];
    int rc = sift_plan(p, h, w, &no, &nl, &sb, sl);
    if (rc) return pano_fail(ctx, rc, "unsupported SIFT parameters");
    size_t goff = 0, doff = 0;
    int oh = 2 * h, ow = 2 * w;
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
        if (ctx->pyr) (void)hipFree(ctx->pyr);
        ctx->pyr = nullptr;
        ctx->pyr_bytes = 0;
        PANO_HIP(ctx, hipMalloc((void **)&ctx->pyr, need));
        ctx->pyr_bytes = need;
    }
    ctx->dog = ctx->pyr + goff;
    ctx->n = n;
    ctx->h = h;
    ctx->w = w;
    return PANO_OK;
}

int launch_sift_pyramid(pano_ctx *ctx, const uint8_t *bgr, int n, int h, int w,
                        const pano_sift_params *p) {
    int no, nl;
    double sb, sl[PANO_MAX_LEVELS];
    int rc = sift_plan(p, h, w, &no, &nl, &sb, sl);
    if (rc) return pano_fail(ctx, rc, "unsupported SIFT parameters");
    rc = sift_reserve_pyramid(ctx, n, h, w, p);
    if (rc) return rc;
    no = ctx->n_oct;
    Taps tb = make_taps(sb);
    Taps tl[PANO_MAX_LEVELS];
    for (int l = 1; l < nl; ++l) tl[l] = make_taps(sl[l]);
    if (tb.n < 0) return pano_fail(ctx, PANO_E_UNSUPPORTED, "Gaussian kernel too wide");
    for (int l = 1; l < nl; ++l)
        if (tl[l].n < 0) return pano_fail(ctx, PANO_E_UNSUPPORTED, "Gaussian kernel too wide");
    float *G = ctx->pyr, *D = ctx->dog;
    // octave 0, level 0: base image
    {
        LoadArgs la{};
        la.bgr = bgr;
        la.sh = h;
        la.sw = w;
        rc = launch_blur<MODE_BASE>(ctx, la, G + ctx->gauss_off[0][0], nullptr, nullptr, n,
                                    ctx->oct_h[0], ctx->oct_w[0], tb);
        if (rc) return rc;
    }
    for (int o = 0; o < no; ++o) {
        const int H = ctx->oct_h[o], W = ctx->oct_w[o];
        for (int l = 1; l < nl; ++l) {
            float *out = G + ctx->gauss_off[o][l];
            float *dg = D + ctx->dog_off[o][l - 1];
            LoadArgs la{};
            if (l == 1 && o > 0) {
                // next-octave base = INTER_NEAREST (w//2, h//2) of level nl-3 of octave o-1,
                // materialised as G[o][0] by the same launch
                la.src = G + ctx->gauss_off[o - 1][nl - 3];
                la.sh = ctx->oct_h[o - 1];
                la.sw = ctx->oct_w[o - 1];
                la.ifx = 1.0 / ((double)W / la.sw);
                la.ify = 1.0 / ((double)H / la.sh);
                rc = launch_blur<MODE_DOWN>(ctx, la, out, dg, G + ctx->gauss_off[o][0], n, H, W,
                                            tl[l]);
            } else {
                la.src = G + ctx->gauss_off[o][l - 1];
                rc = launch_blur<MODE_LEVEL>(ctx, la, out, dg, nullptr, n, H, W, tl[l]);
            }
            if (rc) return rc;
        }
    }
    return PANO_OK;
}
