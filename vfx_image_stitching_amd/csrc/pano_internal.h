// pano_internal.h -- shared declarations of the gfx950 kernels behind include/pano.h.
//
// Numerics policy (DESIGN.md "Parity"): every translation unit is compiled with
// -ffp-contract=off so that a*b+c is two roundings unless a kernel asks for fma()
// explicitly.  fma() is used only where the reference's own arithmetic is an FMA (OpenCV's
// float32 separable Gaussian under FMA3, the OpenBLAS sdot order numpy uses) or where the
// product is exact.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <vector>

#include "../../include/pano.h"

#define PANO_MAX_OCTAVES 16
#define PANO_MAX_LEVELS 8      // num_intervals + 3 <= 8  -> num_intervals <= 5
#define PANO_MAX_TAPS 64
#define PANO_MAX_FRAMES 1024   // frames per pano_sift batch
// SIFT per-frame counters: one 128-byte line each (no false sharing between frames).
// Layout of pano_ctx::counters: [err] [cand f=0..n) [raw f] [ext f], kCntStride ints apiece.
constexpr int kCntStride = 32;
#define PANO_ORI_BINS 36

// Cross-workgroup hand-off of the last-arriver folds (dist_i8 -> reduce, pair_votes ->
// select, cyl_tile<true> -> column flags): the partials are stored at
// agent scope, every wave drains them (s_waitcnt vmcnt(0)) before the barrier, one lane counts
// the workgroup in with an agent-scope add, and the last arriver reads the partials with
// agent-scope loads.  On gfx950 (and gfx942) agent-scope relaxed stores and loads bypass the
// XCD's private L2 (sc1), so drained partials are visible to the last arriver; the HIP / LLVM
// memory model only promises that with a release before the add and an acquire after it.
// PANO_FOLD_FENCE=1 inserts exactly those fences (fold_release / fold_acquire); any other
// target must build with it.
#ifndef PANO_FOLD_FENCE
#define PANO_FOLD_FENCE 0
#endif
#if defined(__HIP_DEVICE_COMPILE__) && !PANO_FOLD_FENCE && !defined(__gfx950__) && !defined(__gfx942__)
#error "the relaxed last-arriver folds rely on gfx950 / gfx942 sc1 semantics: build with -DPANO_FOLD_FENCE=1"
#endif
__device__ __forceinline__ void fold_release() {
#if PANO_FOLD_FENCE
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
#endif
}
__device__ __forceinline__ void fold_acquire() {
#if PANO_FOLD_FENCE
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#endif
}

// Raw keypoint produced by the orientation kernel (before sort/dedup/convert), in base
// (2x upsampled) coordinates, exactly the fields sift_impl.py:206-210/290 stores, plus a
// deterministic scan-order tie-break.
struct RawKp {
    float x, y, size, angle, response;
    int32_t octave;       // packed cv2 octave field
    int32_t frame;
    int32_t pad;
    uint64_t order;       // scan-order tie-break: (candidate scan order << 6) | peak bin
};

// Localised extremum (sift_impl.py:169-211 output) waiting for orientation assignment.
struct Cand {
    float x, y, size, response;   // KeyPoint fields (base coordinates)
    int32_t octave_field;
    int16_t octave, layer;        // octave index and localised layer
    int32_t frame;
    int32_t pad;
    uint64_t order;               // scan order key (octave*8 + layer0) << 32 | y << 16 | x
};

// Device-side view of one pyramid level of a frame batch.
struct LevelView {
    float *ptr;      // [n][h][w]
    int h, w;
};

// Kernel classes for the live HIP-event profiler (pano_prof_enable / pano_prof_read).
enum PanoKernel {
    PK_CYL_SCATTER = 0, PK_CYL_GATHER, PK_BLUR, PK_EXTREMA, PK_ORIENT, PK_SORT, PK_DESC,
    PK_NORMS, PK_DIST_MFMA, PK_DIST_DIRECT, PK_REDUCE, PK_PAIR_SHIFTS, PK_COMPOSITE, PK_BBOX,
    PK_H_GRAY, PK_H_BLUR, PK_H_RESP, PK_H_NMS, PK_H_SELECT, PK_H_DESC, PK_JPEG, PK_COUNT
};

struct ProfState {
    int kernel = -1;                 // -1 off, PK_COUNT = every kernel
    std::vector<hipEvent_t> ev;      // pairs (start, stop)
    std::vector<int> kid;            // kernel class of each pair
    size_t used = 0;                 // events used
};

struct pano_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // ---- SIFT scratch (grown on demand by reserve)
    int n = 0, h = 0, w = 0, cap = 0;
    int n_oct = 0, n_lvl = 0;           // octaves, Gaussian levels per octave
    int oct_h[PANO_MAX_OCTAVES], oct_w[PANO_MAX_OCTAVES];
    size_t pyr_bytes = 0;
    float *pyr = nullptr;                // Gaussian levels, all octaves
    float *dog = nullptr;                // DoG levels, all octaves
    size_t gauss_off[PANO_MAX_OCTAVES][PANO_MAX_LEVELS];
    size_t dog_off[PANO_MAX_OCTAVES][PANO_MAX_LEVELS];
    Cand *cands = nullptr;   size_t cand_cap = 0;
    RawKp *raw = nullptr;    size_t raw_cap = 0;
    int32_t *counters = nullptr;         // [0]=cands [1]=raw [2..2+n) per-frame raw counts
    size_t counters_n = 0;
    int32_t *frame_off = nullptr;        // raw extrema (scan keys) before localisation
    size_t ext_bytes = 0;
    RawKp *raw_sorted = nullptr;
    uint32_t *sorted = nullptr; size_t sorted_bytes = 0;   // per-frame sorted raw indices
    int32_t *dorder = nullptr; size_t dorder_bytes = 0;    // descriptor processing order
    float *taps = nullptr;               // device Gaussian taps (f32), per level [L][PANO_MAX_TAPS]
    float taps_host[PANO_MAX_LEVELS * PANO_MAX_TAPS];    // what *taps holds
    bool taps_valid = false;
    int32_t *match_sync = nullptr; size_t match_sync_bytes = 0; // dist_i8 fold arrival counters (zeroed)
    int32_t *sel_sync = nullptr; size_t sel_sync_bytes = 0;     // pair_votes fold arrival counters (zeroed)
    void *cyl_sync = nullptr; size_t cyl_sync_bytes = 0;        // cyl_tile column flags + strip counters (zeroed)
    uint8_t *gray = nullptr; size_t gray_bytes = 0;   // u8 gray frames (base blur input)
    int32_t *boxslots = nullptr; size_t boxslots_bytes = 0;   // crop-box partials (kBoxSlots x 4)
    // ---- match / ransac scratch
    void *mscratch = nullptr; size_t mscratch_bytes = 0;
    // ---- homography scratch
    void *hmscratch = nullptr; size_t hmscratch_bytes = 0;
    // ---- composite scratch
    uint8_t *flags = nullptr; size_t flags_bytes = 0;
    // ---- harris scratch
    void *hscratch = nullptr; size_t hscratch_bytes = 0;
    // ---- blend scratch
    void *bscratch = nullptr; size_t bscratch_bytes = 0;
    // ---- JPEG decode (jpeg.hip): device scratch, two pinned upload staging buffers used in
    // turn, and per buffer the event that says when the upload out of it has completed (the
    // host fills one while the other's upload may still be queued)
    void *jscratch = nullptr; size_t jscratch_bytes = 0;
    void *jpin[2] = {nullptr, nullptr}; size_t jpin_bytes[2] = {0, 0};
    void *epin = nullptr;                // pinned: the encoder's tables (H2D) and totals (D2H)
    hipEvent_t jev[2] = {nullptr, nullptr};
    int jslot = 0;
    int32_t *jstats = nullptr; int jstats_n = 0;   // last decode's per-frame sync statistics
    // ---- side stream: the small-octave blur tail runs there, overlapped with the extrema
    // scan of the large octaves (fork / join by events; see launch_sift_pyramid)
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    bool tail_pending = false;           // blur_tail enqueued on `side`, not yet joined
    // second side stream: levels nl-2.. of an octave (PANO_OCT_FORK) beside the next octave's
    // first levels, which need only level nl-3; joined before anything reads them
    hipStream_t lvl_side = nullptr;
    // the keypoint sort beside the raw-order descriptors (PANO_DESC_RAW): fork / join on `side`
    hipEvent_t ev_sort_fork = nullptr, ev_sort_join = nullptr;
    uint8_t *descraw = nullptr; size_t descraw_bytes = 0;   // raw-order descriptors + norms
    hipEvent_t ev_lvl[PANO_MAX_OCTAVES] = {};
    hipEvent_t ev_lvl_join = nullptr;
    // third stream: the extrema scan of an octave launched right after its blur (early
    // extrema, PANO_EARLY_EXTREMA), beside the next octaves' blur; joined before localize
    hipStream_t xside = nullptr;
    hipEvent_t ev_x_fork = nullptr, ev_x_join = nullptr;
    bool x_pending = false;              // extrema enqueued on `xside`, not yet joined
    bool early_armed = false;            // pano_sift(_u8): the pyramid may start the extrema
    bool kp_zeroed = false;              // the pyramid's gray_frames zeroed the keypoint counters
    int flags_opt = 0;                   // pano_ctx_set_flags (PANO_CTX_*)
    int early_oct = -1;                  // last octave whose extrema went out early (-1: none)
    int o_tail = 0;                      // first octave of the tail
    bool pyr_full = false;               // every Gaussian level materialised (see launch_sift_pyramid)
    // ---- hipGraph capture (pano_graph_begin / end)
    bool capturing = false;
    size_t cap_prof_start = 0;           // first profiler event of the capture
    // bumped whenever scratch is freed and re-allocated (pano_grow): a graph captured under
    // an older generation holds dangling scratch pointers (pano_ctx_generation)
    uint64_t generation = 1;
    // ---- live profiler
    ProfState prof;
};

// Make ctx->stream wait for a pending blur tail (no-op otherwise).
inline void sift_join_tail(pano_ctx *ctx) {
    if (!ctx->tail_pending) return;
    (void)hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0);
    ctx->tail_pending = false;
}

// Make ctx->stream wait for pending early extrema (no-op otherwise).
inline void sift_join_x(pano_ctx *ctx) {
    if (!ctx->x_pending) return;
    (void)hipStreamWaitEvent(ctx->stream, ctx->ev_x_join, 0);
    ctx->x_pending = false;
}

// RAII: records a start/stop hipEvent pair on the context's stream around one launch
// when the profiler is enabled for this kernel class.
struct PanoProf {
    pano_ctx *ctx;
    hipStream_t st;
    bool on;
    PanoProf(pano_ctx *c, int kid, hipStream_t s = nullptr) : ctx(c), st(s ? s : c->stream), on(false) {
        ProfState &p = c->prof;
        if (p.kernel != kid && p.kernel != PK_COUNT) return;
        if (p.used + 2 > p.ev.size()) {
            for (int i = 0; i < 64; ++i) {
                hipEvent_t e;
                if (hipEventCreate(&e) != hipSuccess) return;
                p.ev.push_back(e);
            }
        }
        p.kid.resize(p.ev.size() / 2);
        p.kid[p.used / 2] = kid;
        on = hipEventRecord(p.ev[p.used], st) == hipSuccess;
    }
    ~PanoProf() {
        if (!on) return;
        ProfState &p = ctx->prof;
        (void)hipEventRecord(p.ev[p.used + 1], st);
        p.used += 2;
    }
};

int pano_fail(pano_ctx *ctx, int code, const std::string &msg);
int pano_hip_check(pano_ctx *ctx, hipError_t e, const char *what);
int pano_grow(pano_ctx *ctx, void **p, size_t *have, size_t need);

#define PANO_HIP(ctx, call)                                                  \
    do {                                                                     \
        hipError_t e__ = (call);                                             \
        if (e__ != hipSuccess) return pano_hip_check((ctx), e__, #call);     \
    } while (0)

#define PANO_LAUNCH_CHECK(ctx, what)                                         \
    do {                                                                     \
        hipError_t e__ = hipGetLastError();                                  \
        if (e__ != hipSuccess) return pano_hip_check((ctx), e__, (what));    \
    } while (0)

// ---- host launchers implemented in the .hip translation units
int launch_fill(pano_ctx *ctx, void *dst, uint8_t value, size_t bytes);   // graph-safe memset
int launch_copy(pano_ctx *ctx, void *dst, const void *src, size_t bytes);  // kernel copy (device-addressable)
int launch_cylindrical(pano_ctx *ctx, const uint8_t *src, uint8_t *dst, int n, int h, int w,
                       const double *h_focal, uint8_t *colnz);
// full = true materialises every Gaussian level (stage access, pano_sift_pyramid); the
// hot path (pano_sift) skips the planes nothing downstream reads: level 0 of octaves > 0 and
// the top level (only its DoG is used).
int sift_kp_counters(pano_ctx *ctx, int32_t **p, size_t *words);   // keypoint counter block
int launch_sift_pyramid(pano_ctx *ctx, const uint8_t *bgr, int n, int h, int w,
                        const pano_sift_params *p, bool defer_tail = false, bool full = true);
// Pyramid input of the stage functions (sift_impl.py:45-97): exactly one source is set.
struct PyrSource {
    const uint8_t *bgr = nullptr;    // [n][h][w][3] u8 BGR (compute_keypoints_and_descriptors)
    const float *grayf = nullptr;    // [n][h][w] f32 gray (generate_base_image)
    const float *base = nullptr;     // [n][h][w] f32 base = octave 0, level 0 (generate_gaussian_images)
    int max_oct = 0;                 // base source: the caller's num_octaves
    bool base_only = false;          // stop after level 0 of octave 0 (generate_base_image)
    const double *sig = nullptr;     // base source: the caller's kernel list (level l blurs level
    int n_sig = 0;                   // l - 1 by sig[l]; n_sig levels), else the parameters' list
};
int launch_sift_pyramid_src(pano_ctx *ctx, const PyrSource &src, int n, int h, int w,
                            const pano_sift_params *p, bool defer_tail, bool full);
// The extrema scan of octave o on the xside stream, forked from ctx->stream (whose work up to
// here wrote octave o's DoG levels); called by the pyramid when early_armed.  The octaves must
// come in order from 0; the keypoint stage then skips them and joins before localize.
int sift_early_extrema(pano_ctx *ctx, const pano_sift_params *p, int o);
int sift_reserve_dims(pano_ctx *ctx, int n, int H0, int W0, int max_oct, int nl);
int launch_sift_dog(pano_ctx *ctx);
// Raw oriented keypoints (find_scale_space_extrema) of the resident pyramid in the
// reference's scan order, base coordinates: d_raw [n][cap], d_counts [n].
int launch_sift_extrema(pano_ctx *ctx, const pano_sift_params *p, pano_kp *raw, int cap, int32_t *counts);
// generate_descriptors for caller keypoints on the resident pyramid: d_desc f32 [n][cap][128].
int launch_sift_localize(pano_ctx *ctx, const pano_sift_params *p, const float *const *dog, int h, int w,
                         int octave, const int32_t *cand, int n, pano_kp *out, int32_t *layer_out);
int launch_sift_orient(pano_ctx *ctx, const pano_sift_params *p, const float *gauss, int h, int w, int octave,
                       const pano_kp *kps, int n, pano_kp *out, int32_t *counts);
int launch_sift_describe(pano_ctx *ctx, const pano_sift_params *p, const pano_kp *kps,
                         const int32_t *counts, int cap, float *desc);
// desc: f32 [n][cap][128] (drop-in form) or, when NULL, desc_u8 [n][cap][128] + norms [n][cap]
int launch_sift_keypoints(pano_ctx *ctx, const pano_sift_params *p, pano_kp *kps, float *desc,
                          uint8_t *desc_u8, int32_t *norms, int cap, int32_t *counts);
int launch_harris(pano_ctx *ctx, const uint8_t *bgr, int n, int h, int w, int max_points,
                  int32_t *xy, float *desc, int32_t *counts);
int launch_match(pano_ctx *ctx, const float *desc, const int32_t *counts, int cap,
                 const int32_t *h_pairs, int n_pairs, int exact_int, int32_t *best, float *d1,
                 float *d2);
int launch_match_u8(pano_ctx *ctx, const uint8_t *desc, const int32_t *norms, const int32_t *counts,
                    int cap, const int32_t *h_pairs, int n_pairs, int32_t *best, float *d1, float *d2);
int launch_pair_shifts(pano_ctx *ctx, const pano_kp *kps, const int32_t *xy_i32,
                       const int32_t *counts, int cap, const int32_t *h_pairs, int n_pairs,
                       const int32_t *best, const float *d1, const float *d2,
                       double desc_thresh, double ratio, double thr, pano_pair_rec *recs);
int launch_ransac_translate(pano_ctx *ctx, const double *moves, int k, double thr,
                            int32_t *out);
int launch_match_compact(pano_ctx *ctx, const pano_kp *kps, const int32_t *counts, int cap,
                         const int32_t *fa, const int32_t *fb, int np, const int32_t *best,
                         const float *d1, const float *d2, double desc_thresh, double ratio,
                         void *moves, int32_t *midx, int32_t *kcount);
int launch_pair_homography(pano_ctx *ctx, const pano_kp *kps, const int32_t *counts, int cap,
                           const int32_t *h_pairs, int n_pairs, const int32_t *best, const float *d1,
                           const float *d2, double desc_thresh, double ratio, double reproj_thr,
                           int n_hyp, unsigned long long seed, int min_good,
                           pano_homography_rec *recs, uint8_t *mask);
int launch_composite(pano_ctx *ctx, const uint8_t *frames, const uint8_t *colnz, int n, int h,
                     int w, const pano_step *steps, const int32_t *first_xy, uint8_t *canvas,
                     int H, int W);
size_t plan_device_bytes();
int launch_plan_device(pano_ctx *ctx, const pano_pair_rec *recs, int n, int h, int w, int int_shifts,
                       int Hcap, int Wcap, void *plan);
int launch_band_layout_row(pano_ctx *ctx, const void *plan, const int32_t *band, const int32_t *slots,
                           long long *row);
int launch_band_plan(pano_ctx *ctx, const void *plan, int f0, int n_local, int w, int Wcap,
                     void *local_plan, int32_t *band);
int launch_composite_planned(pano_ctx *ctx, const uint8_t *frames, const uint8_t *colnz, int n, int h,
                             int w, const void *plan, uint8_t *canvas, int Hcap, int Wcap, int thr,
                             int32_t *bbox);
int launch_plan_composite_device(pano_ctx *ctx, const pano_pair_rec *recs, const uint8_t *frames,
                                 const uint8_t *colnz, int n, int h, int w, int int_shifts, void *plan,
                                 uint8_t *canvas, int Hcap, int Wcap, int thr, int32_t *bbox);
int launch_composite_bbox(pano_ctx *ctx, const uint8_t *frames, const uint8_t *colnz, int n,
                          int h, int w, const pano_step *steps, const int32_t *first_xy,
                          uint8_t *canvas, int H, int W, int thr, int32_t *bbox);
int launch_composite_seq(pano_ctx *ctx, const uint8_t *frames, const uint8_t *colnz, int n, int h,
                         int w, const pano_step *steps, const int32_t *first_xy, uint8_t *canvas,
                         int H, int W);
int launch_blend_two(pano_ctx *ctx, const uint8_t *A, int hA, int wA, const uint8_t *B, int hB,
                     int wB, const int32_t *geom, double overlap, uint8_t *out);
int launch_gray_bbox(pano_ctx *ctx, const uint8_t *img, int H, int W, int thr, int32_t *bbox);
// Baseline JPEG files in host memory -> u8 BGR [n][h][w][3] on the device (jpeg.hip).
int launch_jpeg_decode(pano_ctx *ctx, int n, const uint8_t *const *bufs, const size_t *lens, uint8_t *bgr,
                       int h, int w, int32_t *status);
int jpeg_last_stats(pano_ctx *ctx, int32_t *h, int n);
// u8 BGR rows on the device -> a baseline JPEG file in host memory (jpeg_enc.hip).
int launch_jpeg_encode(pano_ctx *ctx, const uint8_t *bgr, int h, int w, int64_t pitch, int quality,
                       uint8_t *h_out, size_t cap, size_t *out_len);

// ---- device helpers
// XCD-aware workgroup order (MI355X_MICROARCH.md "Workgroup dispatch, XCD placement"):
// workgroups are dealt round-robin over the 8 XCDs, so linear id b runs on the XCD labelled
// b % 8.  Returns a bijective remap giving each XCD label a CONTIGUOUS range of tile ids, so
// neighbouring tiles (shared halos, overlapping patches) hit the same XCD's L2.  Speed only.
__device__ __forceinline__ unsigned xcd_swizzle(unsigned b, unsigned n) {
    const unsigned q = n / 8, r = n % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}
// Chunked variant for grids with uneven work per tile (per-frame keypoint counts): runs of
// CH consecutive tiles stay on one XCD (locality) while the runs rotate over the XCDs
// (balance).  Bijective: the tail that does not fill 8 * CH tiles maps to itself.
template <unsigned CH>
__device__ __forceinline__ unsigned xcd_swizzle_chunked(unsigned b, unsigned n) {
    const unsigned head = n / (8 * CH) * (8 * CH);
    if (b >= head) return b;
    const unsigned i = b / 8;
    return (i / CH) * (8 * CH) + (b % 8) * CH + i % CH;
}
__device__ __forceinline__ unsigned linear_block_id() {
    return blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
}
__device__ __forceinline__ int reflect101(int i, int n) {
    // BORDER_REFLECT_101, periodic beyond one reflection (cv2_compat.reflect101).
    if (n == 1) return 0;
    const int period = 2 * n - 2;
    int m = i % period;
    if (m < 0) m += period;
    return m >= n ? period - m : m;
}

__device__ __forceinline__ uint8_t gray_u8(const uint8_t *p) {
    // OpenCV fixed-point BGR->GRAY (cv2_compat.bgr_to_gray_u8).
    return (uint8_t)((p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + 8192) >> 14);
}

// numpy.round / Python round: half to even.
__device__ __forceinline__ float round_half_even_f(float v) { return rintf(v); }
__device__ __forceinline__ double round_half_even(double v) { return rint(v); }

// numpy float remainder (npy_divmod): result has the sign of the divisor.
__device__ __forceinline__ float np_remainder_f(float a, float b) {
    float m = fmodf(a, b);
    if (m != 0.0f) {
        if ((b < 0.0f) != (m < 0.0f)) m += b;
    } else {
        m = copysignf(0.0f, b);
    }
    return m;
}
// np_remainder_f for b > 0 with the common |a| < b case first: fmod(a, b) == a exactly
// there, so the result is a, a + b (a < 0, rounded as numpy rounds it) or +0.
__device__ __forceinline__ float np_remainder_pos_f(float a, float b) {
    if (fabsf(a) < b) return a < 0.0f ? a + b : (a == 0.0f ? 0.0f : a);
    return np_remainder_f(a, b);
}
__device__ __forceinline__ double np_remainder(double a, double b) {
    double m = fmod(a, b);
    if (m != 0.0) {
        if ((b < 0.0) != (m < 0.0)) m += b;
    } else {
        m = copysign(0.0, b);
    }
    return m;
}
