// blend.hip -- B1: pad_image + blend_two_images (image_stitching_sift.py:139-202), the
// mosaic loop of run_panorama (:369-381) and rectangle_crop's bbox (:208-247).
//
// The reference re-allocates and rewrites the whole mosaic every step (O(N^2 H W)).  Here
// the final canvas is sized up front (pano_plan_composite replays the integer geometry of
// every step on the host) and each step touches only the columns of the new frame: all
// other columns of the step's result are "B only" / "neither" columns, whose values the
// reference copies unchanged.  Per step and column:
//   fF = frame column has a non-zero byte, fM = mosaic column has a non-zero byte
//   both   -> out = f32(1-a) * A + f32(a) * B over the WHOLE step-canvas column,
//             a = (#both columns to the left) / overlap_range (double), uint8 truncation
//   fF only-> the frame column (zeros outside its rows)
// with A/B = (new frame, mosaic) in the dx < 0 (swap) branch, (mosaic, frame) otherwise.
// Column flags ping-pong between two arrays so a step reads the previous step's flags
// while writing its own (columns of the previous frame range are carried across).
#include "pano_internal.h"
#include "plan_core.h"

namespace {

constexpr int CPB = 4;   // columns per workgroup

__device__ __forceinline__ uint8_t blend_px(float a32, float b32, uint8_t A, uint8_t B) {
    const float v = a32 * (float)A + b32 * (float)B;
    return (uint8_t)(int)v;   // astype(np.uint8) on a non-negative float: truncation
}

__device__ __forceinline__ void box_init_slot(int32_t *b) {
    b[0] = 0x7fffffff; b[1] = -1; b[2] = 0x7fffffff; b[3] = -1;
}
// one workgroup's box into slot (workgroup id mod PANO_BBOX_SLOTS)
__device__ __forceinline__ void box_commit(int32_t *slots, int ymin, int ymax, int xmin, int xmax) {
    int32_t *b = slots + 4 * (linear_block_id() % PANO_BBOX_SLOTS);
    atomicMin(&b[0], ymin);
    atomicMax(&b[1], ymax);
    atomicMin(&b[2], xmin);
    atomicMax(&b[3], xmax);
}

__global__ void __launch_bounds__(256)
place_first(const uint8_t *__restrict__ frame, const uint8_t *__restrict__ colnz, int h, int w,
            uint8_t *__restrict__ canvas, int W, int fy, int fx, uint8_t *__restrict__ F0,
            uint8_t *__restrict__ F1) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= w || y >= h) return;
    const uint8_t *s = frame + ((size_t)y * w + x) * 3;
    uint8_t *d = canvas + ((size_t)(fy + y) * W + fx + x) * 3;
    d[0] = s[0];
    d[1] = s[1];
    d[2] = s[2];
    if (y == 0) {
        F0[fx + x] = colnz[x] ? 1 : 0;
        F1[fx + x] = colnz[x] ? 1 : 0;
    }
}

struct StepArg {
    int fx, fy;             // frame content top-left (final canvas)
    int cy, ch;             // step canvas rows [cy, cy + ch)
    int prev_fx;            // previous step's frame column start (-1: none)
    int frame_is_a;
    double overlap;
};

__global__ void __launch_bounds__(256)
composite_step(const uint8_t *__restrict__ frame, const uint8_t *__restrict__ colnz, int h,
               int w, uint8_t *__restrict__ canvas, int W, StepArg s,
               const uint8_t *__restrict__ Fin, uint8_t *__restrict__ Fout) {
    __shared__ int red[256];
    __shared__ int rank_sh[CPB];
    __shared__ int any_sh[CPB];
    const int tid = threadIdx.x;
    const int c0 = blockIdx.x * CPB;
    // carry the previous step's frame-range flags that this step does not rewrite
    if (tid < CPB && s.prev_fx >= 0) {
        const int X = s.prev_fx + c0 + tid;
        if (c0 + tid < w && X >= 0 && X < W && !(X >= s.fx && X < s.fx + w)) Fout[X] = Fin[X];
    }
    // number of "both" columns left of c0 (redundant per workgroup, <= w flags)
    int cntb = 0;
    for (int c = tid; c < c0; c += 256) cntb += (colnz[c] && Fin[s.fx + c]) ? 1 : 0;
    red[tid] = cntb;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (tid < off) red[tid] += red[tid + off];
        __syncthreads();
    }
    if (tid == 0) {
        int r = red[0];
        for (int q = 0; q < CPB; ++q) {
            const int c = c0 + q;
            rank_sh[q] = r;
            any_sh[q] = 0;
            if (c < w && colnz[c] && Fin[s.fx + c]) ++r;
        }
    }
    __syncthreads();
    for (int q = 0; q < CPB; ++q) {
        const int c = c0 + q;
        if (c >= w) break;
        const int X = s.fx + c;
        const bool fF = colnz[c] != 0;
        const bool fM = Fin[X] != 0;
        if (!fF) {
            if (tid == 0) Fout[X] = fM ? 1 : 0;
            continue;
        }
        if (!fM) {
            // frame-only column: copy the frame column (the mosaic column is all zero)
            for (int e = tid; e < h * 3; e += 256) {
                const int y = e / 3, ch = e - y * 3;
                canvas[((size_t)(s.fy + y) * W + X) * 3 + ch] = frame[((size_t)y * w + c) * 3 + ch];
            }
            if (tid == 0) Fout[X] = 1;
            continue;
        }
        const double alpha = s.overlap != 0.0 ? (double)rank_sh[q] / s.overlap : 0.0;
        const float a32 = (float)(1.0 - alpha), b32 = (float)alpha;
        int any = 0;
        for (int e = tid; e < s.ch * 3; e += 256) {
            const int y = s.cy + e / 3, ch = e % 3;
            const int fyl = y - s.fy;
            const uint8_t Fv = (fyl >= 0 && fyl < h) ? frame[((size_t)fyl * w + c) * 3 + ch] : 0;
            uint8_t *pm = canvas + ((size_t)y * W + X) * 3 + ch;
            const uint8_t Mv = *pm;
            const uint8_t o = s.frame_is_a ? blend_px(a32, b32, Fv, Mv) : blend_px(a32, b32, Mv, Fv);
            *pm = o;
            any |= o;
        }
        if (any) any_sh[q] = 1;   // benign race: every writer stores 1
        __syncthreads();
        if (tid == 0) Fout[X] = any_sh[q] ? 1 : 0;
    }
}

// ------------------------------------------------------------------ parallel composite
// Valid when frame i's columns never meet frame j <= i-2 (pano_plan_composite geometry,
// checked on the host): then at step i the mosaic in frame i's columns is exactly frame
// i-1's raw pixels (its A-only region of step i-1), the mosaic column flags there are
// frame i-1's own flags, and every canvas column's final value is written by the LAST
// step whose frame has a non-zero byte in it.  So the fold needs no sequential pass:
//   composite_tables  per (step, frame column): mode (0 none, 1 frame only, 2 both) and
//                     the f32 blend weights of the overlap ramp (block scan for the rank)
//   composite_owner   per canvas column: owning step
//   composite_pixels  per canvas pixel: copy or blend from the raw frames, and the
//                     rectangle_crop bounding box of gray > thr (fused)
constexpr int kMaxSeq = 256;
struct SeqArg {
    int fx[kMaxSeq], fy[kMaxSeq];
    unsigned char is_a[kMaxSeq];
    double overlap[kMaxSeq];
};

// Device-planned stitch (pano_plan_device): the plan kernel writes the sequence table and
// the canvas size to HBM, so the composite launches read them there and the whole stitch is
// one launch chain (one hipGraph, one device->host read at the end).
#ifndef PANO_PLAN_CLOCK
#define PANO_PLAN_CLOCK 0        // 1: s_memtime stamps of plan_device's phases in DevPlan::clk
#endif
struct DevPlan {
    int32_t status, H, W, n;            // status: PANO_OK, PANO_E_NOMATCH, or PANO_E_OVERFLOW
    int32_t first_x, first_y, pad0, pad1;   //   (-> the host plan path)
    SeqArg sa;
    pano_step steps[kMaxSeq];
    long long clk[8];                   // PANO_PLAN_CLOCK timing builds (tools/plan_clock.py); last
};
#ifndef PANO_PLAN_FAST
#define PANO_PLAN_FAST 1         // 0: plan_core over LDS state by one thread (the A/B reference)
#endif
#if PANO_PLAN_CLOCK
#define PLAN_STAMP(k) do { if (threadIdx.x == 0 && blockIdx.x == 0) dp->clk[k] = (long long)__builtin_amdgcn_s_memtime(); } while (0)
#else
#define PLAN_STAMP(k) do { } while (0)
#endif

template <bool DEV>
__global__ void __launch_bounds__(256)
composite_tables(const uint8_t *__restrict__ colnz, int w, SeqArg sa_arg, const DevPlan *__restrict__ dp,
                 uint8_t *__restrict__ mode, float2 *__restrict__ wgt, int32_t *__restrict__ bbox) {
    if (DEV && bbox && blockIdx.x == 0 && threadIdx.x < PANO_BBOX_SLOTS)   // crop-box slots init
        box_init_slot(bbox + 4 * threadIdx.x);
    if (DEV && (dp->status != PANO_OK || (int)blockIdx.x >= dp->n)) return;
    const SeqArg &sa = DEV ? dp->sa : sa_arg;
    __shared__ int sh[256];
    const int i = blockIdx.x, tid = threadIdx.x;
    int carry = 0;
    for (int base = 0; base < w; base += 256) {
        const int c = base + tid;
        int fF = 0, fM = 0;
        if (c < w) {
            fF = colnz[(size_t)i * w + c] != 0;
            if (i > 0) {
                const int xm = sa.fx[i] + c - sa.fx[i - 1];
                fM = (xm >= 0 && xm < w) ? colnz[(size_t)(i - 1) * w + xm] != 0 : 0;
            }
        }
        const int both = fF && fM;
        sh[tid] = both;
        __syncthreads();
        for (int off = 1; off < 256; off <<= 1) {
            const int t = tid >= off ? sh[tid - off] : 0;
            __syncthreads();
            sh[tid] += t;
            __syncthreads();
        }
        if (c < w) {
            const int rank = carry + sh[tid] - both;
            mode[(size_t)i * w + c] = (uint8_t)(fF ? (both ? 2 : 1) : 0);
            const double ov = sa.overlap[i];
            const double alpha = ov != 0.0 ? (double)rank / ov : 0.0;
            wgt[(size_t)i * w + c] = make_float2((float)(1.0 - alpha), (float)alpha);
        }
        carry += sh[255];
        __syncthreads();
    }
}

// Per canvas column: the owning step and everything composite_pixels needs about it
// (source columns, row offsets, mode, blend weights) -- one coalesced 32-byte record.
struct ColInfo {
    int32_t i;          // owning frame (-1: no frame covers the column)
    int32_t c, fy;      // frame column, frame top row on the canvas
    int32_t cm, fym;    // previous frame's column (-1: outside it) and top row
    float w0, w1;       // f32(1 - alpha), f32(alpha)
    uint8_t mode, is_a, pad0, pad1;
};

template <bool DEV>
__global__ void composite_owner(const uint8_t *__restrict__ mode, const float2 *__restrict__ wgt,
                                int n, int w, int W, SeqArg sa_arg, const DevPlan *__restrict__ dp,
                                ColInfo *__restrict__ info) {
    if (DEV) {
        if (dp->status != PANO_OK) return;
        n = dp->n;
        W = dp->W;
    }
    const SeqArg &sa = DEV ? dp->sa : sa_arg;
    const int X = blockIdx.x * blockDim.x + threadIdx.x;
    if (X >= W) return;
    int o = -1;
    for (int i = n - 1; i >= 0; --i) {
        const int c = X - sa.fx[i];
        if (c >= 0 && c < w && mode[(size_t)i * w + c]) { o = i; break; }
    }
    ColInfo ci{};
    ci.i = o;
    if (o >= 0) {
        ci.c = X - sa.fx[o];
        ci.fy = sa.fy[o];
        ci.mode = mode[(size_t)o * w + ci.c];
        ci.is_a = sa.is_a[o];
        const float2 ab = wgt[(size_t)o * w + ci.c];
        ci.w0 = ab.x;
        ci.w1 = ab.y;
        ci.cm = -1;
        if (o > 0) {
            const int cm = X - sa.fx[o - 1];
            ci.cm = (cm >= 0 && cm < w) ? cm : -1;
            ci.fym = sa.fy[o - 1];
        }
    }
    info[X] = ci;
}

// Workgroup = 64 canvas columns x 32 rows: lane = column (its ColInfo record read once),
// each thread walks 8 rows; byte loads / stores are contiguous across the wave.  One bbox
// atomic per workgroup.
constexpr int kCompRows = 8;
// The owner record of canvas column X (composite_owner's per-column work), for the
// device-planned composite, which computes it in composite_pixels itself: the owner is
// usually the last or second-to-last frame tried, and the recomputation per 32-row block
// costs less than a launch.
__device__ __forceinline__ ColInfo column_owner(const uint8_t *__restrict__ mode, const float2 *__restrict__ wgt,
                                                int n, int w, const SeqArg &sa, int X) {
    int o = -1;
    for (int i = n - 1; i >= 0; --i) {
        const int c = X - sa.fx[i];
        if (c >= 0 && c < w && mode[(size_t)i * w + c]) { o = i; break; }
    }
    ColInfo ci{};
    ci.i = o;
    if (o >= 0) {
        ci.c = X - sa.fx[o];
        ci.fy = sa.fy[o];
        ci.mode = mode[(size_t)o * w + ci.c];
        ci.is_a = sa.is_a[o];
        const float2 ab = wgt[(size_t)o * w + ci.c];
        ci.w0 = ab.x;
        ci.w1 = ab.y;
        ci.cm = -1;
        if (o > 0) {
            const int cm = X - sa.fx[o - 1];
            ci.cm = (cm >= 0 && cm < w) ? cm : -1;
            ci.fym = sa.fy[o - 1];
        }
    }
    return ci;
}

template <bool DEV>
__global__ void __launch_bounds__(256)
composite_pixels(const uint8_t *__restrict__ frames, int h, int w, const ColInfo *__restrict__ info,
                 uint8_t *__restrict__ canvas, int H, int W, int thr, int32_t *__restrict__ bbox,
                 const DevPlan *__restrict__ dp, const uint8_t *__restrict__ mode = nullptr,
                 const float2 *__restrict__ wgt = nullptr) {
    __shared__ int r[4][256];
    const int tid = threadIdx.x;
    int bx = blockIdx.x, by = blockIdx.y;
    if (DEV) {
        // grid sized for the capacity; the planned canvas is [H][W] inside it.  The linear
        // block id is remapped onto the planned canvas's blocks, so the live blocks are the
        // first ones dispatched (not interleaved with the empty capacity columns of each row)
        H = dp->status == PANO_OK ? dp->H : 0;
        W = dp->status == PANO_OK ? dp->W : 0;
        const int nbx = (W + 63) / 64, nby = (H + 4 * kCompRows - 1) / (4 * kCompRows);
        const int b = blockIdx.x + gridDim.x * blockIdx.y;
        if (b >= nbx * nby) return;
        by = b / nbx;
        bx = b - by * nbx;
    }
    int ymin = 0x7fffffff, ymax = -1, xmin = 0x7fffffff, xmax = -1;
    const int X = bx * 64 + (tid & 63);
    const int y0 = (by * 4 + (tid >> 6)) * kCompRows;
    if (X < W) {
        const ColInfo ci = DEV ? column_owner(mode, wgt, dp->n, w, dp->sa, X) : info[X];
        // all rows' source bytes first (loads in flight together), then blend and store
        uint8_t F[kCompRows][3], M[kCompRows][3];
        const uint8_t *fp = frames + (((size_t)max(ci.i, 0) * h) * w + ci.c) * 3;
        const uint8_t *mp = frames + (((size_t)max(ci.i - 1, 0) * h) * w + max(ci.cm, 0)) * 3;
        const bool blend = ci.i >= 0 && ci.mode == 2;
        // every load is issued unconditionally from a clamped (in-frame) address and the
        // out-of-frame bytes are zeroed afterwards: predicated loads compiled to a branch and
        // a wait per byte, serialising the 48 loads of a thread
#pragma unroll
        for (int k = 0; k < kCompRows; ++k) {
            const int y = y0 + k;
            const int fyl = y - ci.fy, ym = y - ci.fym;
            const bool fin = ci.i >= 0 && y < H && fyl >= 0 && fyl < h;
            const bool min_ = blend && y < H && ci.cm >= 0 && ym >= 0 && ym < h;
            const size_t fo = (size_t)min(max(fyl, 0), h - 1) * w * 3;
            const size_t mo = (size_t)min(max(ym, 0), h - 1) * w * 3;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const uint8_t fv = fp[fo + c], mv = mp[mo + c];
                F[k][c] = fin ? fv : 0;
                M[k][c] = min_ ? mv : 0;
            }
        }
#pragma unroll
        for (int k = 0; k < kCompRows; ++k) {
            const int y = y0 + k;
            if (y >= H) break;
            uint8_t o[3];
#pragma unroll
            for (int c = 0; c < 3; ++c)
                o[c] = !blend ? F[k][c]
                              : (ci.is_a ? blend_px(ci.w0, ci.w1, F[k][c], M[k][c])
                                         : blend_px(ci.w0, ci.w1, M[k][c], F[k][c]));
            uint8_t *d = canvas + ((size_t)y * W + X) * 3;
            d[0] = o[0]; d[1] = o[1]; d[2] = o[2];
            if (bbox && gray_u8(o) > thr) {
                ymin = min(ymin, y); ymax = max(ymax, y);
                xmin = min(xmin, X); xmax = max(xmax, X);
            }
        }
    }
    if (!bbox) return;
    r[0][tid] = ymin; r[1][tid] = ymax; r[2][tid] = xmin; r[3][tid] = xmax;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (tid < off) {
            r[0][tid] = min(r[0][tid], r[0][tid + off]);
            r[1][tid] = max(r[1][tid], r[1][tid + off]);
            r[2][tid] = min(r[2][tid], r[2][tid + off]);
            r[3][tid] = max(r[3][tid], r[3][tid + off]);
        }
        __syncthreads();
    }
    if (tid == 0 && r[1][0] >= 0) box_commit(bbox, r[0][0], r[1][0], r[2][0], r[3][0]);
}

// ------------------------------------------------------------------ generic blend_two_images
__global__ void col_flags2(const uint8_t *__restrict__ A, int hA, int wA, int ayA, int axA,
                           const uint8_t *__restrict__ B, int hB, int wB, int ayB, int axB,
                           int WW, uint8_t *__restrict__ fa, uint8_t *__restrict__ fb) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= WW) return;
    int ra = 0, rb = 0;
    const int ca = c - axA, cb = c - axB;
    if (ca >= 0 && ca < wA)
        for (int y = 0; y < hA && !ra; ++y) {
            const uint8_t *p = A + ((size_t)y * wA + ca) * 3;
            ra = (p[0] | p[1] | p[2]) != 0;
        }
    if (cb >= 0 && cb < wB)
        for (int y = 0; y < hB && !rb; ++y) {
            const uint8_t *p = B + ((size_t)y * wB + cb) * 3;
            rb = (p[0] | p[1] | p[2]) != 0;
        }
    fa[c] = (uint8_t)ra;
    fb[c] = (uint8_t)rb;
}

__global__ void __launch_bounds__(1024)
both_rank(const uint8_t *__restrict__ fa, const uint8_t *__restrict__ fb, int WW,
          int32_t *__restrict__ rank) {
    __shared__ int sh[1024];
    int carry = 0;
    const int tid = threadIdx.x;
    for (int base = 0; base < WW; base += 1024) {
        const int c = base + tid;
        const int v = (c < WW && fa[c] && fb[c]) ? 1 : 0;
        sh[tid] = v;
        __syncthreads();
        for (int off = 1; off < 1024; off <<= 1) {
            const int t = tid >= off ? sh[tid - off] : 0;
            __syncthreads();
            sh[tid] += t;
            __syncthreads();
        }
        if (c < WW) rank[c] = carry + sh[tid] - v;
        const int tot = sh[1023];
        __syncthreads();
        carry += tot;
    }
}

__global__ void __launch_bounds__(256)
blend_two(const uint8_t *__restrict__ A, int hA, int wA, int ayA, int axA,
          const uint8_t *__restrict__ B, int hB, int wB, int ayB, int axB, int HH, int WW,
          const uint8_t *__restrict__ fa, const uint8_t *__restrict__ fb,
          const int32_t *__restrict__ rank, double overlap, uint8_t *__restrict__ out) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= WW || y >= HH) return;
    const int ya = y - ayA, xa = x - axA, yb = y - ayB, xb = x - axB;
    const bool ina = ya >= 0 && ya < hA && xa >= 0 && xa < wA;
    const bool inb = yb >= 0 && yb < hB && xb >= 0 && xb < wB;
    uint8_t *o = out + ((size_t)y * WW + x) * 3;
    const uint8_t *pa = ina ? A + ((size_t)ya * wA + xa) * 3 : nullptr;
    const uint8_t *pb = inb ? B + ((size_t)yb * wB + xb) * 3 : nullptr;
    if (fa[x] && fb[x]) {
        const double alpha = overlap != 0.0 ? (double)rank[x] / overlap : 0.0;
        const float a32 = (float)(1.0 - alpha), b32 = (float)alpha;
        for (int ch = 0; ch < 3; ++ch)
            o[ch] = blend_px(a32, b32, pa ? pa[ch] : 0, pb ? pb[ch] : 0);
    } else if (fa[x]) {
        for (int ch = 0; ch < 3; ++ch) o[ch] = pa ? pa[ch] : 0;
    } else if (fb[x]) {
        for (int ch = 0; ch < 3; ++ch) o[ch] = pb ? pb[ch] : 0;
    } else {
        o[0] = o[1] = o[2] = 0;
    }
}

// ------------------------------------------------------------------ rectangle_crop bbox

__global__ void __launch_bounds__(256)
gray_bbox(const uint8_t *__restrict__ img, int H, int W, int thr, int32_t *__restrict__ bbox) {
    __shared__ int r[4][256];
    const int tid = threadIdx.x;
    int ymin = 0x7fffffff, ymax = -1, xmin = 0x7fffffff, xmax = -1;
    const size_t total = (size_t)H * W;
    for (size_t i = (size_t)blockIdx.x * 256 + tid; i < total; i += (size_t)gridDim.x * 256) {
        if (gray_u8(img + i * 3) > thr) {
            const int y = (int)(i / W), x = (int)(i % W);
            ymin = min(ymin, y); ymax = max(ymax, y);
            xmin = min(xmin, x); xmax = max(xmax, x);
        }
    }
    r[0][tid] = ymin; r[1][tid] = ymax; r[2][tid] = xmin; r[3][tid] = xmax;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (tid < off) {
            r[0][tid] = min(r[0][tid], r[0][tid + off]);
            r[1][tid] = max(r[1][tid], r[1][tid + off]);
            r[2][tid] = min(r[2][tid], r[2][tid + off]);
            r[3][tid] = max(r[3][tid], r[3][tid + off]);
        }
        __syncthreads();
    }
    if (tid == 0 && r[1][0] >= 0) box_commit(bbox, r[0][0], r[1][0], r[2][0], r[3][0]);
}

__global__ void bbox_init(int32_t *slots) {   // PANO_BBOX_SLOTS threads
    box_init_slot(slots + 4 * threadIdx.x);
}

// slots -> the 4-int box, -1s when no pixel passed (one wave)
__global__ void bbox_fix(const int32_t *__restrict__ slots, int32_t *__restrict__ bbox) {
    const int t = threadIdx.x;
    int a = 0x7fffffff, b = -1, c = 0x7fffffff, d = -1;
    if (t < PANO_BBOX_SLOTS) { a = slots[4 * t]; b = slots[4 * t + 1]; c = slots[4 * t + 2]; d = slots[4 * t + 3]; }
    for (int o = 32; o > 0; o >>= 1) {
        a = min(a, __shfl_xor(a, o)); b = max(b, __shfl_xor(b, o));
        c = min(c, __shfl_xor(c, o)); d = max(d, __shfl_xor(d, o));
    }
    if (t == 0) {
        if (b < 0) a = b = c = d = -1;
        bbox[0] = a; bbox[1] = b; bbox[2] = c; bbox[3] = d;
    }
}

}  // namespace

extern "C" int pano_blend_geometry(double dx, double dy, const double *ref4, int hA, int wA,
                                   int hB, int wB, int32_t *geom, double *overlap) {
    if (!ref4 || !geom || !overlap) return PANO_E_ARG;
    return blend_geometry(dx, dy, ref4, hA, wA, hB, wB, geom, overlap);
}

extern "C" int pano_plan_composite(const double *shifts, const double *pairs, int n, int h, int w,
                                   pano_step *steps, int32_t *first_xy, int32_t *canvas_hw) {
    if (n < 1 || h <= 0 || w <= 0 || !first_xy || !canvas_hw || (n > 1 && (!shifts || !pairs || !steps)))
        return PANO_E_ARG;
    std::vector<int32_t> tmp(5 * (size_t)n);
    return plan_core([&](int k, double *d) { d[0] = shifts[2 * k]; d[1] = shifts[2 * k + 1]; },
                     [&](int k, double *d) { for (int q = 0; q < 4; ++q) d[q] = pairs[4 * k + q]; },
                     n, h, w, steps, first_xy, canvas_hw, tmp.data());
}

namespace {


// run_panorama's record -> shift conversion (floats for SIFT, int() for Harris), drift
// correction (:336-365) and the whole composite plan, in the host code's exact double
// arithmetic.  The plan is a sequential scalar chain: the records are staged in LDS and ONE
// thread runs it over LDS state (a global-memory chain would pay an HBM round trip per
// dependent access); the parallel-composite check and the write-out use every thread.
// TABLES (plan_tables): grid = n workgroups; every workgroup replays the (cheap, serial) plan
// itself, workgroup 0 publishes it (and initialises the crop-box slots), and workgroup i then
// builds composite_tables' mode / weight row of frame i from its own copy -- the plan and the
// tables in one launch, no cross-workgroup hand-off.
template <bool TABLES>
__global__ void __launch_bounds__(256)
plan_device(const pano_pair_rec *__restrict__ recs, int n, int h, int w, int int_shifts, int Hcap,
            int Wcap, DevPlan *__restrict__ dp, const uint8_t *__restrict__ colnz = nullptr,
            uint8_t *__restrict__ mode = nullptr, float2 *__restrict__ wgt = nullptr,
            int32_t *__restrict__ bbox = nullptr) {
    __shared__ double rv[6][kMaxSeq];           // dx dy xA yA xB yB per pair (converted)
    __shared__ pano_step st[kMaxSeq];
    __shared__ int32_t tmp[8 * kMaxSeq];           // plan scratch (plan_core: 5 n; the fast path: 8 rows)
    __shared__ int32_t fx[kMaxSeq];
    __shared__ int32_t hdr[6];                  // status H W first_x first_y, bands flag
    __shared__ int bad;
    const int tid = threadIdx.x, P = n - 1;
    const bool lead = blockIdx.x == 0;          // the workgroup that publishes the plan
    PLAN_STAMP(0);
    if (TABLES && lead && bbox && tid < PANO_BBOX_SLOTS) box_init_slot(bbox + 4 * tid);
    auto conv = [&](double v) { return int_shifts ? (double)(long long)v : v; };   // int() truncates
    if (tid == 0) bad = 0;
    __syncthreads();
    for (int k = tid; k < P; k += blockDim.x) {
        const pano_pair_rec r = recs[k];
        if (r.status != PANO_OK) atomicOr(&bad, 1);
        rv[0][k] = conv(r.dx); rv[1][k] = conv(r.dy);
        rv[2][k] = conv(r.xA); rv[3][k] = conv(r.yA); rv[4][k] = conv(r.xB); rv[5][k] = conv(r.yB);
    }
    __syncthreads();
    PLAN_STAMP(1);
#if PANO_PLAN_FAST
    // Wave 0: the per-step constants (plan_step_const) one step per lane; the serial part --
    // the drift sum in pair order and the mosaic-size chain (plan_chain_hw) -- with each
    // step's constants broadcast by readlane; then every lane finishes its own step
    // (plan_chain_step from the sizes the chain handed it) and the origins are suffix sums
    // across the lanes.  Same numbers as plan_core (plan_fast, tools/host_fuzz.cpp).  Per step
    // the chain costs ~490 cycles (PANO_PLAN_CLOCK): plan_core over LDS state by one thread
    // ~1,200; the same chain on LDS broadcast reads ~650.
    if (tid < 64) {
        const int lane = tid;
        auto rl = [](int v, int j) { return __builtin_amdgcn_readlane(v, j); };
        auto rld = [](double v, int j) {
            const long long b = __double_as_longlong(v);
            const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), j);
            const int hi = __builtin_amdgcn_readlane((int)(b >> 32), j);
            return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
        };
        int rc = bad ? PANO_E_NOMATCH : PANO_OK;
        int Hm = h, Wm = w, oy = 0, ox = 0;
        if (rc == PANO_OK) {
            // drift correction: the sum in pair order, as Python's
            double tot = 0.0;
            long long itot = 0;
            for (int k = 0; k < P; ++k) {
                if (int_shifts) itot += (long long)rv[1][k];
                else tot = tot + rv[1][k];
            }
            const double avg = int_shifts ? (double)itot / (double)P : tot / (double)P;
            PLAN_STAMP(2);
            if (h <= 0 || w <= 0 || h > kPlanMaxSide / 2 || w > kPlanMaxSide / 2) rc = PANO_E_ARG;
            int32_t *yM = tmp, *xM = tmp + kMaxSeq, *yF = tmp + 2 * kMaxSeq, *xF = tmp + 3 * kMaxSeq,
                    *ptop = tmp + 4 * kMaxSeq;          // by step k = i - 1
            for (int c0 = 0; c0 < P && rc == PANO_OK; c0 += 64) {
                const int k = c0 + lane;
                PlanStepConst c{};
                if (k < P) {
                    const double pd[4] = {rv[2][k], rv[3][k], rv[4][k], rv[5][k]};
                    c = plan_step_const(rv[0][k], rv[1][k] - avg, pd);
                }
                // the serial part: only the mosaic size; lane j keeps the size its step starts
                // from and computes the rest of its step afterwards
                int Hin = Hm, Win = Wm;
                const int m = min(64, P - c0);
                for (int j = 0; j < m; ++j) {
                    PlanStepConst cj;
                    cj.bad = rl(c.bad, j);
                    if (cj.bad) { rc = PANO_E_ARG; break; }
                    cj.r00 = rld(c.r00, j);
                    cj.r10 = rld(c.r10, j);
                    cj.swapped = rl(c.swapped, j);
                    cj.myA = rl(c.myA, j);
                    cj.myB = rl(c.myB, j);
                    cj.mxB = rl(c.mxB, j);
                    int H1, W1;
                    plan_chain_hw(cj, Hm, Wm, h, w, H1, W1);
                    if (H1 > kPlanMaxSide || W1 > kPlanMaxSide) { rc = PANO_E_OVERFLOW; break; }
                    if (lane == j) { Hin = Hm; Win = Wm; }
                    Hm = H1;
                    Wm = W1;
                }
                const PlanStepOut mine = plan_chain_step(c, Hin, Win, h, w);
                if (k < P && rc == PANO_OK) {
                    pano_step &q = st[k];
                    q.canvas_h = mine.H;
                    q.canvas_w = mine.W;
                    q.frame_is_a = c.swapped;
                    q.pad = 0;
                    q.overlap_range = mine.ov;
                    yM[k] = mine.yM; xM[k] = mine.xM; yF[k] = mine.yF; xF[k] = mine.xF; ptop[k] = mine.ptop;
                }
            }
            PLAN_STAMP(7);
            if (rc == PANO_OK) {
                // origins: step k's mosaic sits at the sum of yM / xM over the later steps
                for (int c0 = (P - 1) / 64 * 64; c0 >= 0; c0 -= 64) {
                    const int k = c0 + lane;
                    const int vy = k < P ? yM[k] : 0, vx = k < P ? xM[k] : 0;
                    int iy = vy, ix = vx;            // inclusive prefix over the lanes
#pragma unroll
                    for (int d = 1; d < 64; d <<= 1) {
                        const int ty = __shfl_up(iy, d), tx = __shfl_up(ix, d);
                        if (lane >= d) { iy += ty; ix += tx; }
                    }
                    const int ty = __shfl(iy, 63), tx = __shfl(ix, 63);
                    if (k < P) {
                        pano_step &q = st[k];
                        q.canvas_y = oy + ty - iy;   // later steps of this chunk + later chunks
                        q.canvas_x = ox + tx - ix;
                        q.frame_y = q.canvas_y + yF[k] + ptop[k];
                        q.frame_x = q.canvas_x + xF[k];
                    }
                    oy += ty;
                    ox += tx;
                }
            }
        }
        if (lane == 0) {
            hdr[0] = rc;
            hdr[1] = rc == PANO_OK ? Hm : 0;
            hdr[2] = rc == PANO_OK ? Wm : 0;
            hdr[3] = ox;
            hdr[4] = oy;
            if (rc == PANO_OK && !(ox >= 0 && oy >= 0 && ox + w <= Wm && oy + h <= Hm && Hm <= Hcap && Wm <= Wcap))
                hdr[0] = PANO_E_OVERFLOW;
        }
        PLAN_STAMP(3);
    }
#else
    if (tid == 0) {
        hdr[0] = PANO_OK;
        if (bad) {
            hdr[0] = PANO_E_NOMATCH;
        } else {
            double avg = 0.0;
            if (int_shifts) {           // Python int sum, then true division
                long long tot = 0;
                for (int k = 0; k < P; ++k) tot += (long long)rv[1][k];
                avg = (double)tot / (double)P;
            } else {
                double tot = 0.0;
                for (int k = 0; k < P; ++k) tot = tot + rv[1][k];
                avg = tot / (double)P;
            }
            int32_t first[2], hw[2];
            PLAN_STAMP(2);
            const int rc = plan_core([&](int k, double *d) { d[0] = rv[0][k]; d[1] = rv[1][k] - avg; },
                                     [&](int k, double *d) { for (int q = 0; q < 4; ++q) d[q] = rv[2 + q][k]; },
                                     n, h, w, st, first, hw, tmp);
            PLAN_STAMP(3);
            hdr[0] = rc ? rc : PANO_OK;
            hdr[1] = hw[0];
            hdr[2] = hw[1];
            hdr[3] = first[0];
            hdr[4] = first[1];
            if (!rc && !(first[0] >= 0 && first[1] >= 0 && first[0] + w <= hw[1] && first[1] + h <= hw[0] &&
                         hw[0] <= Hcap && hw[1] <= Wcap))
                hdr[0] = PANO_E_OVERFLOW;
        }
    }
#endif
    __syncthreads();
    const int status = hdr[0];
    PLAN_STAMP(4);
    if (status == PANO_OK) {
        const int H = hdr[1], W = hdr[2];
        for (int i = tid; i < n; i += blockDim.x) fx[i] = i ? st[i - 1].frame_x : hdr[3];
        __syncthreads();
        if (TABLES) {
            // composite_tables' row of frame i = blockIdx.x from this workgroup's plan copy
            const int i = blockIdx.x;
            const double ov = i ? st[i - 1].overlap_range : 0.0;
            int carry = 0;
            int *sh = tmp;                       // the plan's scratch, free now
            for (int base = 0; base < w; base += 256) {
                const int c = base + tid;
                int fF = 0, fM = 0;
                if (c < w) {
                    fF = colnz[(size_t)i * w + c] != 0;
                    if (i > 0) {
                        const int xm = fx[i] + c - fx[i - 1];
                        fM = (xm >= 0 && xm < w) ? colnz[(size_t)(i - 1) * w + xm] != 0 : 0;
                    }
                }
                const int both = fF && fM;
                // exclusive rank of `both` (ballot per wave, wave totals through LDS)
                const unsigned long long m = __ballot(both);
                const int lane = tid & 63, wv = tid >> 6;
                if (lane == 0) sh[wv] = __popcll(m);
                __syncthreads();
                int wbase = 0, tot = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    wbase += q < wv ? sh[q] : 0;
                    tot += sh[q];
                }
                if (c < w) {
                    const int rank = carry + wbase + __popcll(m & ((1ull << lane) - 1ull));
                    mode[(size_t)i * w + c] = (uint8_t)(fF ? (both ? 2 : 1) : 0);
                    const double alpha = ov != 0.0 ? (double)rank / ov : 0.0;
                    wgt[(size_t)i * w + c] = make_float2((float)(1.0 - alpha), (float)alpha);
                }
                carry += tot;
                __syncthreads();
            }
            PLAN_STAMP(5);
            if (!lead) return;
        }
        for (int i = tid; i < n; i += blockDim.x) {
            bool ok = true;
            if (i) {
                const pano_step &q = st[i - 1];
                ok = q.frame_x >= 0 && q.frame_x + w <= W && q.frame_y >= 0 && q.frame_y + h <= H &&
                     q.canvas_y >= 0 && q.canvas_y + q.canvas_h <= H;
            }
            const int xi = fx[i];
            for (int j = 0; j <= i - 2; ++j)            // frame i never meets a frame j <= i - 2
                ok &= xi + w <= fx[j] || fx[j] + w <= xi;
            if (!ok) atomicOr(&bad, 2);
            dp->sa.fx[i] = fx[i];
            dp->sa.fy[i] = i ? st[i - 1].frame_y : hdr[4];
            dp->sa.is_a[i] = i ? (unsigned char)st[i - 1].frame_is_a : 0;
            dp->sa.overlap[i] = i ? st[i - 1].overlap_range : 0.0;
            if (i) dp->steps[i - 1] = st[i - 1];
        }
        __syncthreads();
    }
    if (TABLES && !lead) return;
    PLAN_STAMP(6);
    if (tid == 0) {
        dp->status = (status == PANO_OK && (bad & 2)) ? PANO_E_OVERFLOW : status;
        dp->n = n;
        dp->H = status == PANO_OK ? hdr[1] : 0;
        dp->W = status == PANO_OK ? hdr[2] : 0;
        dp->first_x = hdr[3];
        dp->first_y = hdr[4];
    }
}

// One rank's band of a sharded stitch, from the GLOBAL device plan: the rank holds
// frames f0 .. f0 + n_local - 1 (its pairs plus the boundary frame f0) and owns the canvas
// columns whose last covering frame is one of its frames after f0 (plus frame 0's columns on
// the first band).  With no column covered by three frames -- which plan_device checks: its
// status is PANO_OK only then -- a column's final value depends on its last covering frame
// and that frame's predecessor, both held by the owning band, so the band composites exactly
// like the whole canvas.  Writes a LOCAL plan over the band's frames whose canvas is the
// owned column range (frame positions shifted by its first column, possibly negative), for
// pano_composite_planned, and band = {status, own_lo, own_hi, global W}.
__global__ void band_plan(const DevPlan *__restrict__ g, int f0, int n_local, int w, int Wcap,
                          DevPlan *__restrict__ l, int32_t *__restrict__ band) {
    __shared__ int32_t hdr[3];
    const int tid = threadIdx.x;
    if (tid == 0) {
        int st = g->status, lo = 0, hi = 0;
        const int n = g->n;
        if (st == PANO_OK && (f0 < 0 || n_local < 1 || f0 + n_local > n)) st = PANO_E_ARG;
        if (st == PANO_OK) {
            // owned pieces: last_cover(i) = frame i's span minus frame i+1's span (at most two
            // pieces each; disjoint across frames because frame i+2 never meets frame i), so
            // their union is one interval iff its span equals their total length
            lo = 0x7fffffff;
            hi = -0x7fffffff;
            long long total = 0;
            const int i0 = f0 == 0 ? 0 : f0 + 1;
            for (int i = i0; i <= f0 + n_local - 1; ++i) {
                const int a = g->sa.fx[i], b = a + w;
                int pc[2][2] = {{a, b}, {0, 0}};
                if (i + 1 < n) {
                    const int na = g->sa.fx[i + 1], nb = na + w;
                    pc[0][1] = min(b, na);
                    pc[1][0] = max(a, nb);
                    pc[1][1] = b;
                }
                for (int q = 0; q < 2; ++q)
                    if (pc[q][0] < pc[q][1]) {
                        lo = min(lo, pc[q][0]);
                        hi = max(hi, pc[q][1]);
                        total += pc[q][1] - pc[q][0];
                    }
            }
            if (lo > hi) { lo = 0; hi = 0; }
            else if (total != (long long)(hi - lo)) st = PANO_E_UNSUPPORTED;
            if (st == PANO_OK && hi - lo > Wcap) st = PANO_E_OVERFLOW;
        }
        hdr[0] = st; hdr[1] = lo; hdr[2] = hi;
    }
    __syncthreads();
    const int st = hdr[0], lo = hdr[1], hi = hdr[2];
    for (int k = tid; k < n_local && st == PANO_OK; k += blockDim.x) {
        l->sa.fx[k] = g->sa.fx[f0 + k] - lo;
        l->sa.fy[k] = g->sa.fy[f0 + k];
        l->sa.is_a[k] = k == 0 ? 0 : g->sa.is_a[f0 + k];
        l->sa.overlap[k] = k == 0 ? 0.0 : g->sa.overlap[f0 + k];
    }
    if (tid == 0) {
        l->status = st;
        l->n = n_local;
        l->H = st == PANO_OK ? g->H : 0;
        l->W = st == PANO_OK ? hi - lo : 0;
        l->first_x = l->first_y = 0;
        band[0] = st;
        band[1] = lo;
        band[2] = hi;
        band[3] = g->W;
    }
}

// The rank's row of the N > 1 layout exchange, on the device (so the all_gather of the rows
// needs no host round trip): {ymin, ymax, xmin, xmax} of the band's crop-box partials in
// GLOBAL columns (NO_BOX when no pixel passed), own_lo, own_hi, fallback (the global plan or
// the band plan refused), the global plan's status.
__global__ void band_layout_row(const DevPlan *__restrict__ g, const int32_t *__restrict__ band,
                                const int32_t *__restrict__ slots, long long *__restrict__ row) {
    const int t = threadIdx.x;                   // one wave
    int a = 0x7fffffff, b = -1, c = 0x7fffffff, d = -1;
    if (t < PANO_BBOX_SLOTS) { a = slots[4 * t]; b = slots[4 * t + 1]; c = slots[4 * t + 2]; d = slots[4 * t + 3]; }
    for (int o = 32; o > 0; o >>= 1) {
        a = min(a, __shfl_xor(a, o)); b = max(b, __shfl_xor(b, o));
        c = min(c, __shfl_xor(c, o)); d = max(d, __shfl_xor(d, o));
    }
    if (t == 0) {
        const int gst = g->status, bst = band[0];
        const bool ok = gst == PANO_OK && bst == PANO_OK;
        const long long lo = ok ? band[1] : 0, hi = ok ? band[2] : 0;
        const bool box = ok && b >= 0;
        row[0] = box ? a : (1ll << 30);
        row[1] = box ? b : -1;
        row[2] = box ? c + lo : (1ll << 30);
        row[3] = box ? d + lo : -1;
        row[4] = lo;
        row[5] = hi;
        row[6] = ok ? 0 : 1;
        row[7] = gst;
    }
}

}  // namespace

int launch_band_layout_row(pano_ctx *ctx, const void *plan, const int32_t *band, const int32_t *slots,
                           long long *row) {
    if (!plan || !band || !slots || !row) return pano_fail(ctx, PANO_E_ARG, "pano_band_layout_row: bad arguments");
    band_layout_row<<<1, 64, 0, ctx->stream>>>((const DevPlan *)plan, band, slots, row);
    PANO_LAUNCH_CHECK(ctx, "band_layout_row");
    return PANO_OK;
}

int launch_band_plan(pano_ctx *ctx, const void *plan, int f0, int n_local, int w, int Wcap,
                     void *local_plan, int32_t *band) {
    if (!plan || !local_plan || !band || n_local < 1 || n_local > kMaxSeq || f0 < 0 || w <= 0)
        return pano_fail(ctx, PANO_E_ARG, "pano_band_plan: bad arguments");
    {
        PanoProf prof_(ctx, PK_COMPOSITE);
        band_plan<<<1, 256, 0, ctx->stream>>>((const DevPlan *)plan, f0, n_local, w, Wcap,
                                             (DevPlan *)local_plan, band);
    }
    PANO_LAUNCH_CHECK(ctx, "band_plan");
    return PANO_OK;
}

size_t plan_device_bytes() { return sizeof(DevPlan); }

int launch_plan_device(pano_ctx *ctx, const pano_pair_rec *recs, int n, int h, int w, int int_shifts,
                       int Hcap, int Wcap, void *plan) {
    if (n < 2 || n > kMaxSeq || h <= 0 || w <= 0 || !recs || !plan)
        return pano_fail(ctx, PANO_E_ARG, "pano_plan_device: bad arguments");
    {
        PanoProf prof_(ctx, PK_COMPOSITE);
        plan_device<false><<<1, 256, 0, ctx->stream>>>(recs, n, h, w, int_shifts, Hcap, Wcap, (DevPlan *)plan);
    }
    PANO_LAUNCH_CHECK(ctx, "plan_device");
    return PANO_OK;
}

int launch_composite_planned(pano_ctx *ctx, const uint8_t *frames, const uint8_t *colnz, int n, int h,
                             int w, const void *plan, uint8_t *canvas, int Hcap, int Wcap, int thr,
                             int32_t *bbox) {
    if (n < 2 || n > kMaxSeq || !frames || !colnz || !canvas || !plan)
        return pano_fail(ctx, PANO_E_ARG, "pano_composite_planned: bad arguments");
    const DevPlan *dp = (const DevPlan *)plan;
    const size_t o_w = ((size_t)n * w + 255) & ~size_t(255);
    const size_t o_own = o_w + (((size_t)n * w * sizeof(float2) + 255) & ~size_t(255));
    int rc = pano_grow(ctx, (void **)&ctx->flags, &ctx->flags_bytes, o_own + (size_t)Wcap * sizeof(ColInfo));
    if (rc) return rc;
    uint8_t *mode = ctx->flags;
    float2 *wgt = (float2 *)(ctx->flags + o_w);
    ColInfo *info = (ColInfo *)(ctx->flags + o_own);
    static const SeqArg none{};
    {
        PanoProf prof_(ctx, PK_COMPOSITE);
        composite_tables<true><<<n, 256, 0, ctx->stream>>>(colnz, w, none, dp, mode, wgt, bbox);
    }
    PANO_LAUNCH_CHECK(ctx, "composite_tables");
    (void)info;                                  // the owner records: computed per column in composite_pixels
    {
        dim3 grid((Wcap + 63) / 64, (Hcap + 4 * kCompRows - 1) / (4 * kCompRows));
        PanoProf prof_(ctx, PK_COMPOSITE);
        composite_pixels<true><<<grid, 256, 0, ctx->stream>>>(frames, h, w, nullptr, canvas, Hcap, Wcap, thr,
                                                              bbox, dp, mode, wgt);
    }
    PANO_LAUNCH_CHECK(ctx, "composite_pixels");
    return PANO_OK;
}

// pano_plan_device + pano_composite_planned as two launches: plan_device<true> (the plan in
// every workgroup, the composite tables of frame i in workgroup i, the crop-box slots) and
// composite_pixels.  Same bytes as the three-launch form (the tables are the same arithmetic).
int launch_plan_composite_device(pano_ctx *ctx, const pano_pair_rec *recs, const uint8_t *frames,
                                 const uint8_t *colnz, int n, int h, int w, int int_shifts, void *plan,
                                 uint8_t *canvas, int Hcap, int Wcap, int thr, int32_t *bbox) {
    if (n < 2 || n > kMaxSeq || h <= 0 || w <= 0 || !recs || !plan || !frames || !colnz || !canvas)
        return pano_fail(ctx, PANO_E_ARG, "pano_plan_composite_device: bad arguments");
    const DevPlan *dp = (const DevPlan *)plan;
    const size_t o_w = ((size_t)n * w + 255) & ~size_t(255);
    const size_t o_own = o_w + (((size_t)n * w * sizeof(float2) + 255) & ~size_t(255));
    int rc = pano_grow(ctx, (void **)&ctx->flags, &ctx->flags_bytes, o_own + (size_t)Wcap * sizeof(ColInfo));
    if (rc) return rc;
    uint8_t *mode = ctx->flags;
    float2 *wgt = (float2 *)(ctx->flags + o_w);
    {
        PanoProf prof_(ctx, PK_COMPOSITE);
        plan_device<true><<<n, 256, 0, ctx->stream>>>(recs, n, h, w, int_shifts, Hcap, Wcap, (DevPlan *)plan,
                                                      colnz, mode, wgt, bbox);
    }
    PANO_LAUNCH_CHECK(ctx, "plan_device");
    {
        dim3 grid((Wcap + 63) / 64, (Hcap + 4 * kCompRows - 1) / (4 * kCompRows));
        PanoProf prof_(ctx, PK_COMPOSITE);
        composite_pixels<true><<<grid, 256, 0, ctx->stream>>>(frames, h, w, nullptr, canvas, Hcap, Wcap, thr,
                                                              bbox, dp, mode, wgt);
    }
    PANO_LAUNCH_CHECK(ctx, "composite_pixels");
    return PANO_OK;
}

// Host check of the parallel-composite condition: frame i never shares a column with a
// frame j <= i - 2.
static bool bands_independent(const pano_step *steps, const int32_t *first_xy, int n, int w) {
    auto fx = [&](int i) { return i == 0 ? first_xy[0] : steps[i - 1].frame_x; };
    for (int i = 2; i < n; ++i)
        for (int j = 0; j <= i - 2; ++j)
            if (!(fx(i) + w <= fx(j) || fx(j) + w <= fx(i))) return false;
    return true;
}

static int composite_sequential(pano_ctx *ctx, const uint8_t *frames, const uint8_t *colnz, int n,
                                int h, int w, const pano_step *steps, const int32_t *first_xy,
                                uint8_t *canvas, int H, int W) {
    int rc = pano_grow(ctx, (void **)&ctx->flags, &ctx->flags_bytes, 2 * (size_t)W + 64);
    if (rc) return rc;
    uint8_t *F[2] = {ctx->flags, ctx->flags + W};
    rc = launch_fill(ctx, canvas, 0, (size_t)H * W * 3);
    if (rc) return rc;
    rc = launch_fill(ctx, ctx->flags, 0, 2 * (size_t)W);
    if (rc) return rc;
    dim3 g0((w + 63) / 64, (h + 3) / 4);
    {
        PanoProf prof_(ctx, PK_COMPOSITE);
        place_first<<<g0, 256, 0, ctx->stream>>>(frames, colnz, h, w, canvas, W, first_xy[1],
                                                 first_xy[0], F[0], F[1]);
    }
    PANO_LAUNCH_CHECK(ctx, "place_first");
    int prev_fx = -1;
    for (int i = 1; i < n; ++i) {
        const pano_step &st = steps[i - 1];
        StepArg s;
        s.fx = st.frame_x;
        s.fy = st.frame_y;
        s.cy = st.canvas_y;
        s.ch = st.canvas_h;
        s.prev_fx = prev_fx;
        s.frame_is_a = st.frame_is_a;
        s.overlap = st.overlap_range;
        const uint8_t *fr = frames + (size_t)i * h * w * 3;
        {
            PanoProf prof_(ctx, PK_COMPOSITE);
            composite_step<<<(w + CPB - 1) / CPB, 256, 0, ctx->stream>>>(
                fr, colnz + (size_t)i * w, h, w, canvas, W, s, F[(i - 1) & 1], F[i & 1]);
        }
        PANO_LAUNCH_CHECK(ctx, "composite_step");
        prev_fx = st.frame_x;
    }
    return PANO_OK;
}

static int check_geometry(pano_ctx *ctx, int n, int h, int w, const pano_step *steps,
                          const int32_t *first_xy, int H, int W) {
    if (first_xy[0] < 0 || first_xy[1] < 0 || first_xy[0] + w > W || first_xy[1] + h > H)
        return pano_fail(ctx, PANO_E_ARG, "pano_composite: frame 0 outside canvas");
    for (int i = 1; i < n; ++i) {
        const pano_step &st = steps[i - 1];
        if (st.frame_x < 0 || st.frame_x + w > W || st.frame_y < 0 || st.frame_y + h > H ||
            st.canvas_y < 0 || st.canvas_y + st.canvas_h > H)
            return pano_fail(ctx, PANO_E_ARG, "pano_composite: step outside canvas");
    }
    return PANO_OK;
}

int launch_composite_bbox(pano_ctx *ctx, const uint8_t *frames, const uint8_t *colnz, int n,
                          int h, int w, const pano_step *steps, const int32_t *first_xy,
                          uint8_t *canvas, int H, int W, int thr, int32_t *bbox) {
    if (n < 1 || !frames || !colnz || !canvas || !first_xy || (n > 1 && !steps))
        return pano_fail(ctx, PANO_E_ARG, "pano_composite: bad arguments");
    int rc = check_geometry(ctx, n, h, w, steps, first_xy, H, W);
    if (rc) return rc;
    if (n > kMaxSeq || !bands_independent(steps, first_xy, n, w)) {
        rc = composite_sequential(ctx, frames, colnz, n, h, w, steps, first_xy, canvas, H, W);
        if (rc || !bbox) return rc;
        return launch_gray_bbox(ctx, canvas, H, W, thr, bbox);
    }
    SeqArg sa;
    for (int i = 0; i < n; ++i) {
        sa.fx[i] = i == 0 ? first_xy[0] : steps[i - 1].frame_x;
        sa.fy[i] = i == 0 ? first_xy[1] : steps[i - 1].frame_y;
        sa.is_a[i] = i == 0 ? 0 : (unsigned char)steps[i - 1].frame_is_a;
        sa.overlap[i] = i == 0 ? 0.0 : steps[i - 1].overlap_range;
    }
    const size_t o_mode = 0;
    const size_t o_w = ((size_t)n * w + 255) & ~size_t(255);
    const size_t o_own = o_w + (((size_t)n * w * sizeof(float2) + 255) & ~size_t(255));
    rc = pano_grow(ctx, (void **)&ctx->flags, &ctx->flags_bytes, o_own + (size_t)W * sizeof(ColInfo));
    if (rc) return rc;
    uint8_t *mode = ctx->flags + o_mode;
    float2 *wgt = (float2 *)(ctx->flags + o_w);
    ColInfo *info = (ColInfo *)(ctx->flags + o_own);
    int32_t *slots = nullptr;
    if (bbox) {
        rc = pano_grow(ctx, (void **)&ctx->boxslots, &ctx->boxslots_bytes, 4 * PANO_BBOX_SLOTS * sizeof(int32_t));
        if (rc) return rc;
        slots = ctx->boxslots;
        PanoProf prof_(ctx, PK_BBOX);
        bbox_init<<<1, PANO_BBOX_SLOTS, 0, ctx->stream>>>(slots);
    }
    {
        PanoProf prof_(ctx, PK_COMPOSITE);
        composite_tables<false><<<n, 256, 0, ctx->stream>>>(colnz, w, sa, nullptr, mode, wgt, nullptr);
    }
    PANO_LAUNCH_CHECK(ctx, "composite_tables");
    {
        PanoProf prof_(ctx, PK_COMPOSITE);
        composite_owner<false><<<(W + 255) / 256, 256, 0, ctx->stream>>>(mode, wgt, n, w, W, sa, nullptr, info);
    }
    PANO_LAUNCH_CHECK(ctx, "composite_owner");
    {
        dim3 grid((W + 63) / 64, (H + 4 * kCompRows - 1) / (4 * kCompRows));
        PanoProf prof_(ctx, PK_COMPOSITE);
        composite_pixels<false><<<grid, 256, 0, ctx->stream>>>(frames, h, w, info, canvas, H, W, thr, slots, nullptr);
    }
    PANO_LAUNCH_CHECK(ctx, "composite_pixels");
    if (bbox) {
        PanoProf prof_(ctx, PK_BBOX);
        bbox_fix<<<1, 64, 0, ctx->stream>>>(slots, bbox);
    }
    return PANO_OK;
}

int launch_composite(pano_ctx *ctx, const uint8_t *frames, const uint8_t *colnz, int n, int h,
                     int w, const pano_step *steps, const int32_t *first_xy, uint8_t *canvas,
                     int H, int W) {
    return launch_composite_bbox(ctx, frames, colnz, n, h, w, steps, first_xy, canvas, H, W, 0,
                                 nullptr);
}

int launch_composite_seq(pano_ctx *ctx, const uint8_t *frames, const uint8_t *colnz, int n, int h,
                         int w, const pano_step *steps, const int32_t *first_xy, uint8_t *canvas,
                         int H, int W) {
    if (n < 1 || !frames || !colnz || !canvas || !first_xy || (n > 1 && !steps))
        return pano_fail(ctx, PANO_E_ARG, "pano_composite: bad arguments");
    int rc = check_geometry(ctx, n, h, w, steps, first_xy, H, W);
    if (rc) return rc;
    return composite_sequential(ctx, frames, colnz, n, h, w, steps, first_xy, canvas, H, W);
}

int launch_blend_two(pano_ctx *ctx, const uint8_t *A, int hA, int wA, const uint8_t *B, int hB,
                     int wB, const int32_t *g, double overlap, uint8_t *out) {
    if (!A || !B || !g || !out) return pano_fail(ctx, PANO_E_ARG, "pano_blend_two: bad arguments");
    const int HH = g[4], WW = g[5];
    const size_t need = 2 * (size_t)WW + (size_t)WW * 4 + 64;
    int rc = pano_grow(ctx, (void **)&ctx->flags, &ctx->flags_bytes, need);
    if (rc) return rc;
    uint8_t *fa = ctx->flags, *fb = ctx->flags + WW;
    int32_t *rank = (int32_t *)(ctx->flags + ((2 * (size_t)WW + 15) & ~size_t(15)));
    col_flags2<<<(WW + 255) / 256, 256, 0, ctx->stream>>>(A, hA, wA, g[0], g[1], B, hB, wB, g[2],
                                                          g[3], WW, fa, fb);
    PANO_LAUNCH_CHECK(ctx, "col_flags2");
    {
        PanoProf prof_(ctx, PK_COMPOSITE);
        both_rank<<<1, 1024, 0, ctx->stream>>>(fa, fb, WW, rank);
    }
    PANO_LAUNCH_CHECK(ctx, "both_rank");
    dim3 grid((WW + 63) / 64, (HH + 3) / 4);
    {
        PanoProf prof_(ctx, PK_COMPOSITE);
        blend_two<<<grid, 256, 0, ctx->stream>>>(A, hA, wA, g[0], g[1], B, hB, wB, g[2], g[3], HH, WW,
                                                 fa, fb, rank, overlap, out);
    }
    PANO_LAUNCH_CHECK(ctx, "blend_two");
    return PANO_OK;
}

int launch_gray_bbox(pano_ctx *ctx, const uint8_t *img, int H, int W, int thr, int32_t *bbox) {
    if (!img || !bbox || H <= 0 || W <= 0) return pano_fail(ctx, PANO_E_ARG, "pano_gray_bbox");
    int rc = pano_grow(ctx, (void **)&ctx->boxslots, &ctx->boxslots_bytes, 4 * PANO_BBOX_SLOTS * sizeof(int32_t));
    if (rc) return rc;
    int32_t *slots = ctx->boxslots;
    bbox_init<<<1, PANO_BBOX_SLOTS, 0, ctx->stream>>>(slots);
    const size_t total = (size_t)H * W;
    unsigned blocks = (unsigned)((total + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    {
        PanoProf prof_(ctx, PK_BBOX);
        gray_bbox<<<blocks, 256, 0, ctx->stream>>>(img, H, W, thr, slots);
    }
    bbox_fix<<<1, 64, 0, ctx->stream>>>(slots, bbox);
    PANO_LAUNCH_CHECK(ctx, "gray_bbox");
    return PANO_OK;
}
