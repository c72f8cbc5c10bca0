// pano_abi.cpp -- the extern "C" surface declared in include/pano.h.
//
// Thin: argument checks, the per-device context (stream + scratch), and dispatch to the
// launchers of the .hip translation units.  Nothing here computes image data.
#include <cstdio>
#include <cstring>

#include "jpeg_core.h"
#include "pano_internal.h"

int sift_reserve_pyramid(pano_ctx *ctx, int n, int h, int w, const pano_sift_params *p);
int sift_plan(const pano_sift_params *p, int h, int w, int *n_oct, int *n_lvl, double *sig_base,
              double *sig_lvl);
int sift_set_attributes(pano_ctx *ctx);
int harris_set_attributes(pano_ctx *ctx);
int match_set_attributes(pano_ctx *ctx);

int pano_fail(pano_ctx *ctx, int code, const std::string &msg) {
    if (ctx) ctx->err = msg;
    return code;
}

int pano_hip_check(pano_ctx *ctx, hipError_t e, const char *what) {
    char buf[512];
    snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    return pano_fail(ctx, PANO_E_HIP, buf);
}

int pano_grow(pano_ctx *ctx, void **p, size_t *have, size_t need) {
    if (need <= *have && *p) return PANO_OK;
    if (ctx->capturing)
        return pano_fail(ctx, PANO_E_UNSUPPORTED,
                         "scratch growth inside a graph capture: run the sequence once eagerly first");
    if (*p) {
        hipError_t e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) return pano_hip_check(ctx, e, "grow sync");
        (void)hipFree(*p);
        *p = nullptr;
        *have = 0;
        ++ctx->generation;               // graphs captured before this point are stale
    }
    size_t sz = need + need / 4 + 4096;
    hipError_t e = hipMalloc(p, sz);
    if (e != hipSuccess) return pano_hip_check(ctx, e, "hipMalloc scratch");
    *have = sz;
    return PANO_OK;
}

// The device address of p when the GPU may dereference it (device memory, or pinned host
// memory mapped into the device's address space), else nullptr.
static void *device_address(void *p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();               // pageable host memory: clear the sticky error
        return nullptr;
    }
    if (a.type == hipMemoryTypeDevice) return p;
    // pinned host memory: only when the GPU sees it at the same address (no offset to trust)
    if (a.type == hipMemoryTypeHost && a.devicePointer == p) return p;
    return nullptr;
}

extern "C" {

const char *pano_version(void) { return "libpano 0.1 gfx950"; }

void pano_sift_default_params(pano_sift_params *p) {
    p->sigma = 1.6;
    p->num_intervals = 3;
    p->assumed_blur = 0.5;
    p->border = 5;
    p->contrast_threshold = 0.04;
    p->eigen_ratio = 10;
    p->max_iter = 5;
    p->radius_factor = 3;
    p->peak_ratio = 0.8;
    p->scale_factor = 1.5;
    p->scale_multiplier = 3;
    p->descriptor_max = 0.2;
}

// Host-only: the scalar plan of a SIFT run (octaves, per-level sigmas) -- CPU-testable.
int pano_sift_plan(const pano_sift_params *p, int h, int w, int *n_oct, int *n_lvl,
                   double *sig_base, double *sig_lvl) {
    if (!p || !n_oct || !n_lvl || !sig_base || !sig_lvl || h <= 0 || w <= 0) return PANO_E_ARG;
    return sift_plan(p, h, w, n_oct, n_lvl, sig_base, sig_lvl);
}

int pano_ctx_create(int device, void *stream, pano_ctx **out) {
    if (!out) return PANO_E_ARG;
    *out = nullptr;
    pano_ctx *ctx = new pano_ctx();
    ctx->device = device;
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) {
        delete ctx;
        return PANO_E_HIP;
    }
    ctx->stream = (hipStream_t)stream;
    int rc = sift_set_attributes(ctx);
    if (!rc) rc = harris_set_attributes(ctx);
    if (!rc) rc = match_set_attributes(ctx);
    if (rc) {
        delete ctx;
        return rc;
    }
    *out = ctx;
    return PANO_OK;
}

int pano_ctx_destroy(pano_ctx *ctx) {
    if (!ctx) return PANO_OK;
    sift_join_tail(ctx);
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->side) (void)hipStreamSynchronize(ctx->side);
    if (ctx->side) (void)hipStreamDestroy(ctx->side);
    if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
    if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
    if (ctx->xside) (void)hipStreamSynchronize(ctx->xside);
    if (ctx->xside) (void)hipStreamDestroy(ctx->xside);
    if (ctx->ev_x_fork) (void)hipEventDestroy(ctx->ev_x_fork);
    if (ctx->ev_x_join) (void)hipEventDestroy(ctx->ev_x_join);
    if (ctx->lvl_side) (void)hipStreamSynchronize(ctx->lvl_side);
    if (ctx->lvl_side) (void)hipStreamDestroy(ctx->lvl_side);
    for (hipEvent_t e : ctx->ev_lvl)
        if (e) (void)hipEventDestroy(e);
    if (ctx->ev_lvl_join) (void)hipEventDestroy(ctx->ev_lvl_join);
    if (ctx->ev_sort_fork) (void)hipEventDestroy(ctx->ev_sort_fork);
    if (ctx->ev_sort_join) (void)hipEventDestroy(ctx->ev_sort_join);
    void *bufs[] = {ctx->pyr, ctx->cands, ctx->raw, ctx->counters, ctx->frame_off, ctx->raw_sorted,
                    ctx->taps, ctx->mscratch, ctx->flags, ctx->hscratch, ctx->bscratch, ctx->gray, ctx->sorted,
                    ctx->boxslots, ctx->hmscratch, ctx->dorder, ctx->match_sync, ctx->sel_sync, ctx->descraw, ctx->cyl_sync};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    if (ctx->jscratch) (void)hipFree(ctx->jscratch);
    for (int i = 0; i < 2; ++i) {
        if (ctx->jpin[i]) (void)hipHostFree(ctx->jpin[i]);
        if (ctx->jev[i]) (void)hipEventDestroy(ctx->jev[i]);
    }
    if (ctx->epin) (void)hipHostFree(ctx->epin);
    for (hipEvent_t e : ctx->prof.ev) (void)hipEventDestroy(e);
    delete ctx;
    return PANO_OK;
}

int pano_ctx_release_scratch(pano_ctx *ctx) {
    if (!ctx) return PANO_E_ARG;
    if (ctx->capturing) return pano_fail(ctx, PANO_E_UNSUPPORTED, "pano_ctx_release_scratch inside a graph capture");
    sift_join_tail(ctx);
    sift_join_x(ctx);
    hipError_t e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return pano_hip_check(ctx, e, "release sync");
    struct Slot { void **p; size_t *bytes; };
    size_t dummy = 0;
    const Slot slots[] = {
        {(void **)&ctx->pyr, &ctx->pyr_bytes},           {(void **)&ctx->cands, &ctx->cand_cap},
        {(void **)&ctx->raw, &ctx->raw_cap},             {(void **)&ctx->counters, &ctx->counters_n},
        {(void **)&ctx->frame_off, &ctx->ext_bytes},     {(void **)&ctx->sorted, &ctx->sorted_bytes},
        {(void **)&ctx->dorder, &ctx->dorder_bytes},     {(void **)&ctx->gray, &ctx->gray_bytes},
        {(void **)&ctx->boxslots, &ctx->boxslots_bytes}, {&ctx->mscratch, &ctx->mscratch_bytes},
        {&ctx->hmscratch, &ctx->hmscratch_bytes},        {(void **)&ctx->flags, &ctx->flags_bytes},
        {&ctx->hscratch, &ctx->hscratch_bytes},          {&ctx->bscratch, &ctx->bscratch_bytes},
        {&ctx->jscratch, &ctx->jscratch_bytes},          {(void **)&ctx->raw_sorted, &dummy},
        {(void **)&ctx->descraw, &ctx->descraw_bytes},   {&ctx->cyl_sync, &ctx->cyl_sync_bytes},
        // arrival counters: zeroed when (re)allocated, so a released one comes back zeroed
        {(void **)&ctx->match_sync, &ctx->match_sync_bytes},
        {(void **)&ctx->sel_sync, &ctx->sel_sync_bytes},
    };
    for (const Slot &s : slots) {
        if (*s.p) (void)hipFree(*s.p);
        *s.p = nullptr;
        *s.bytes = 0;
    }
    for (int i = 0; i < 2; ++i) {
        if (ctx->jev[i]) (void)hipEventSynchronize(ctx->jev[i]);
        if (ctx->jpin[i]) (void)hipHostFree(ctx->jpin[i]);
        ctx->jpin[i] = nullptr;
        ctx->jpin_bytes[i] = 0;
    }
    ctx->dog = nullptr;
    ctx->jstats = nullptr;
    ctx->jstats_n = 0;
    ctx->n = ctx->h = ctx->w = 0;
    ++ctx->generation;                   // every captured graph points at freed memory now
    return PANO_OK;
}

int pano_ctx_set_stream(pano_ctx *ctx, void *stream) {
    if (!ctx) return PANO_E_ARG;
    sift_join_tail(ctx);
    ctx->stream = (hipStream_t)stream;
    return PANO_OK;
}

int pano_ctx_set_flags(pano_ctx *ctx, int flags) {
    if (!ctx || (flags & ~(PANO_CTX_TAIL_MAIN | PANO_CTX_MATCH_WHOLE))) return PANO_E_ARG;
    ctx->flags_opt = flags;
    return PANO_OK;
}

int pano_ctx_reserve(pano_ctx *ctx, int n, int h, int w, int cap) {
    if (!ctx || n <= 0 || h <= 0 || w <= 0 || cap <= 0) return PANO_E_ARG;
    pano_sift_params p;
    pano_sift_default_params(&p);
    return sift_reserve_pyramid(ctx, n, h, w, &p);
}

int pano_sync(pano_ctx *ctx) {
    if (!ctx) return PANO_E_ARG;
    hipError_t e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return pano_hip_check(ctx, e, "pano_sync");
    if (ctx->counters && ctx->n > 0) {
        int32_t err = 0;
        e = hipMemcpy(&err, ctx->counters, sizeof err, hipMemcpyDeviceToHost);
        if (e == hipSuccess && err) return pano_fail(ctx, PANO_E_OVERFLOW, "keypoint capacity exceeded");
    }
    return PANO_OK;
}

const char *pano_last_error(pano_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

uint64_t pano_ctx_generation(pano_ctx *ctx) { return ctx ? ctx->generation : 0; }

int pano_cylindrical(pano_ctx *ctx, const uint8_t *src, uint8_t *dst, int n, int h, int w,
                     const double *focal, uint8_t *colnz) {
    if (!ctx) return PANO_E_ARG;
    return launch_cylindrical(ctx, src, dst, n, h, w, focal, colnz);
}

int pano_sift_pyramid(pano_ctx *ctx, const uint8_t *bgr, int n, int h, int w,
                      const pano_sift_params *params) {
    if (!ctx || !bgr || n <= 0 || h <= 0 || w <= 0) return ctx ? pano_fail(ctx, PANO_E_ARG, "pano_sift_pyramid") : PANO_E_ARG;
    pano_sift_params p;
    if (params) p = *params; else pano_sift_default_params(&p);
    return launch_sift_pyramid(ctx, bgr, n, h, w, &p);
}

int pano_sift(pano_ctx *ctx, const uint8_t *bgr, int n, int h, int w,
              const pano_sift_params *params, pano_kp *kps, float *desc, int cap,
              int32_t *counts) {
    if (!ctx) return PANO_E_ARG;
    pano_sift_params p;
    if (params) p = *params; else pano_sift_default_params(&p);
    ctx->early_armed = true;
    int rc = launch_sift_pyramid(ctx, bgr, n, h, w, &p, /*defer_tail=*/true, /*full=*/false);
    ctx->early_armed = false;
    if (rc != PANO_OK) ctx->kp_zeroed = false;        // no keypoint stage follows
    if (rc == PANO_OK) rc = launch_sift_keypoints(ctx, &p, kps, desc, nullptr, nullptr, cap, counts);
    sift_join_tail(ctx);
    sift_join_x(ctx);
    ctx->early_oct = -1;                  // no-op unless an error left the tail unjoined
    return rc;
}

int pano_sift_u8(pano_ctx *ctx, const uint8_t *bgr, int n, int h, int w,
                 const pano_sift_params *params, pano_kp *kps, uint8_t *desc_u8, int32_t *norms,
                 int cap, int32_t *counts) {
    if (!ctx) return PANO_E_ARG;
    if (!desc_u8 || !norms) return pano_fail(ctx, PANO_E_ARG, "pano_sift_u8: bad outputs");
    pano_sift_params p;
    if (params) p = *params; else pano_sift_default_params(&p);
    ctx->early_armed = true;
    int rc = launch_sift_pyramid(ctx, bgr, n, h, w, &p, /*defer_tail=*/true, /*full=*/false);
    ctx->early_armed = false;
    if (rc != PANO_OK) ctx->kp_zeroed = false;        // no keypoint stage follows
    if (rc == PANO_OK) rc = launch_sift_keypoints(ctx, &p, kps, nullptr, desc_u8, norms, cap, counts);
    sift_join_tail(ctx);
    sift_join_x(ctx);
    ctx->early_oct = -1;
    return rc;
}

int pano_sift_base(pano_ctx *ctx, const float *gray, int n, int h, int w, const pano_sift_params *params,
                   float *base) {
    if (!ctx || !gray || !base || n <= 0 || h <= 0 || w <= 0)
        return ctx ? pano_fail(ctx, PANO_E_ARG, "pano_sift_base") : PANO_E_ARG;
    pano_sift_params p;
    if (params) p = *params; else pano_sift_default_params(&p);
    PyrSource src;
    src.grayf = gray;
    src.base_only = true;
    int rc = launch_sift_pyramid_src(ctx, src, n, h, w, &p, false, false);
    if (rc) return rc;
    PANO_HIP(ctx, hipMemcpyAsync(base, ctx->pyr + ctx->gauss_off[0][0],
                                 (size_t)n * ctx->oct_h[0] * ctx->oct_w[0] * sizeof(float),
                                 hipMemcpyDeviceToDevice, ctx->stream));
    return PANO_OK;
}

int pano_sift_pyramid_base(pano_ctx *ctx, const float *base, int n, int H0, int W0, int n_octaves,
                           const pano_sift_params *params) {
    if (!ctx || !base || n <= 0 || H0 <= 0 || W0 <= 0 || n_octaves <= 0)
        return ctx ? pano_fail(ctx, PANO_E_ARG, "pano_sift_pyramid_base") : PANO_E_ARG;
    if (n_octaves > PANO_MAX_OCTAVES)
        return pano_fail(ctx, PANO_E_UNSUPPORTED, "pano_sift_pyramid_base: more than PANO_MAX_OCTAVES octaves");
    pano_sift_params p;
    if (params) p = *params; else pano_sift_default_params(&p);
    PyrSource src;
    src.base = base;
    src.max_oct = n_octaves;
    return launch_sift_pyramid_src(ctx, src, n, H0, W0, &p, false, true);
}

int pano_sift_pyramid_kernels(pano_ctx *ctx, const float *base, int n, int H0, int W0, int n_octaves,
                              const double *kernels, int n_kernels) {
    if (!ctx || !base || !kernels || n <= 0 || H0 <= 0 || W0 <= 0 || n_octaves <= 0)
        return ctx ? pano_fail(ctx, PANO_E_ARG, "pano_sift_pyramid_kernels") : PANO_E_ARG;
    if (n_octaves > PANO_MAX_OCTAVES)
        return pano_fail(ctx, PANO_E_UNSUPPORTED, "pano_sift_pyramid_kernels: more than PANO_MAX_OCTAVES octaves");
    // the level count first: kernels[] is read only up to a valid n_kernels
    if (n_kernels < 3 || n_kernels > PANO_MAX_LEVELS)
        return pano_fail(ctx, PANO_E_UNSUPPORTED, "pano_sift_pyramid_kernels: 3 <= n_kernels <= PANO_MAX_LEVELS");
    // every sigma finite, >= 0 and narrow enough for PANO_MAX_TAPS taps (rint(8 s + 1) | 1 <= 63)
    for (int l = 1; l < n_kernels; ++l)
        if (!(kernels[l] >= 0.0 && kernels[l] * 8.0 + 1.0 < (double)PANO_MAX_TAPS))
            return pano_fail(ctx, PANO_E_UNSUPPORTED,
                             "pano_sift_pyramid_kernels: sigma negative, NaN, infinite or wider than PANO_MAX_TAPS taps");
    pano_sift_params p;
    pano_sift_default_params(&p);
    PyrSource src;
    src.base = base;
    src.max_oct = n_octaves;
    src.sig = kernels;
    src.n_sig = n_kernels;
    return launch_sift_pyramid_src(ctx, src, n, H0, W0, &p, false, true);
}

int pano_sift_reserve_levels(pano_ctx *ctx, int n, int H0, int W0, int n_octaves, int n_levels) {
    if (!ctx || n <= 0 || H0 <= 0 || W0 <= 0 || n_octaves <= 0 || n_levels < 3 || n_levels > PANO_MAX_LEVELS)
        return ctx ? pano_fail(ctx, PANO_E_ARG, "pano_sift_reserve_levels") : PANO_E_ARG;
    if (n_octaves > PANO_MAX_OCTAVES)
        return pano_fail(ctx, PANO_E_UNSUPPORTED, "pano_sift_reserve_levels: more than PANO_MAX_OCTAVES octaves");
    sift_join_tail(ctx);
    const int rc = sift_reserve_dims(ctx, n, H0, W0, n_octaves, n_levels);
    if (rc == PANO_OK) ctx->pyr_full = true;
    return rc;
}

int pano_sift_set_level(pano_ctx *ctx, int frame, int octave, int level, int dog, const float *in) {
    if (!ctx || !in || frame < 0 || frame >= ctx->n || octave < 0 || octave >= ctx->n_oct) return PANO_E_ARG;
    const int nl = dog ? ctx->n_lvl - 1 : ctx->n_lvl;
    if (level < 0 || level >= nl) return PANO_E_ARG;
    const size_t plane = (size_t)ctx->oct_h[octave] * ctx->oct_w[octave];
    float *dst = dog ? ctx->dog + ctx->dog_off[octave][level] : ctx->pyr + ctx->gauss_off[octave][level];
    PANO_HIP(ctx, hipMemcpyAsync(dst + (size_t)frame * plane, in, plane * sizeof(float),
                                 hipMemcpyDeviceToDevice, ctx->stream));
    return PANO_OK;
}

int pano_sift_dog(pano_ctx *ctx) {
    if (!ctx) return PANO_E_ARG;
    sift_join_tail(ctx);
    return launch_sift_dog(ctx);
}

int pano_sift_extrema(pano_ctx *ctx, const pano_sift_params *params, pano_kp *raw, int cap, int32_t *counts) {
    if (!ctx) return PANO_E_ARG;
    if (!ctx->pyr || ctx->n <= 0) return pano_fail(ctx, PANO_E_ARG, "pano_sift_extrema: no resident pyramid");
    pano_sift_params p;
    if (params) p = *params; else pano_sift_default_params(&p);
    if (p.num_intervals + 3 != ctx->n_lvl)
        return pano_fail(ctx, PANO_E_ARG, "pano_sift_extrema: num_intervals does not match the pyramid");
    const int rc = launch_sift_extrema(ctx, &p, raw, cap, counts);
    sift_join_tail(ctx);
    return rc;
}

int pano_sift_describe(pano_ctx *ctx, const pano_sift_params *params, const pano_kp *kps, const int32_t *counts,
                       int cap, float *desc) {
    if (!ctx) return PANO_E_ARG;
    pano_sift_params p;
    if (params) p = *params; else pano_sift_default_params(&p);
    return launch_sift_describe(ctx, &p, kps, counts, cap, desc);
}

int pano_sift_localize(pano_ctx *ctx, const pano_sift_params *params, const float *const *dog, int n_dog, int h,
                       int w, int octave, const int32_t *cand, int n, pano_kp *out, int32_t *layer) {
    if (!ctx) return PANO_E_ARG;
    pano_sift_params p;
    if (params) p = *params; else pano_sift_default_params(&p);
    if (n < 0 || (n > 0 && (!cand || !out || !layer || !dog)))
        return pano_fail(ctx, PANO_E_ARG, "pano_sift_localize: bad arguments");
    if (p.num_intervals < 1 || p.num_intervals + 3 > PANO_MAX_LEVELS || n_dog != p.num_intervals + 2)
        return pano_fail(ctx, PANO_E_ARG, "pano_sift_localize: needs num_intervals + 2 DoG levels");
    if (octave < 0 || octave >= PANO_MAX_OCTAVES || h < 3 || w < 3 || h > 65535 || w > 65535 || p.border < 1 ||
        p.max_iter < 1)
        return pano_fail(ctx, PANO_E_ARG, "pano_sift_localize: bad octave, level shape, border or max_iter");
    for (int l = 0; l < n_dog && n > 0; ++l)
        if (!dog[l]) return pano_fail(ctx, PANO_E_ARG, "pano_sift_localize: null DoG level");
    return launch_sift_localize(ctx, &p, dog, h, w, octave, cand, n, out, layer);
}

int pano_sift_orient(pano_ctx *ctx, const pano_sift_params *params, const float *gauss, int h, int w, int octave,
                     const pano_kp *kps, int n, pano_kp *out, int32_t *counts) {
    if (!ctx) return PANO_E_ARG;
    pano_sift_params p;
    if (params) p = *params; else pano_sift_default_params(&p);
    if (n < 0 || (n > 0 && (!gauss || !kps || !out || !counts)) || h < 1 || w < 1 || octave < 0 || octave > 30)
        return pano_fail(ctx, PANO_E_ARG, "pano_sift_orient: bad arguments");
    return launch_sift_orient(ctx, &p, gauss, h, w, octave, kps, n, out, counts);
}

int pano_sift_level_shape(pano_ctx *ctx, int octave, int *h_out, int *w_out, int *n_octaves) {
    if (!ctx || octave < 0 || octave >= ctx->n_oct) return PANO_E_ARG;
    if (h_out) *h_out = ctx->oct_h[octave];
    if (w_out) *w_out = ctx->oct_w[octave];
    if (n_octaves) *n_octaves = ctx->n_oct;
    return PANO_OK;
}

int pano_sift_copy_level(pano_ctx *ctx, int frame, int octave, int level, int dog, float *out) {
    if (!ctx || !out || frame < 0 || frame >= ctx->n || octave < 0 || octave >= ctx->n_oct)
        return PANO_E_ARG;
    const int nl = dog ? ctx->n_lvl - 1 : ctx->n_lvl;
    if (level < 0 || level >= nl) return PANO_E_ARG;
    if (!dog && !ctx->pyr_full && (level == 0 || level > nl - 3))
        return pano_fail(ctx, PANO_E_UNSUPPORTED,
                         "pano_sift does not materialise this Gaussian level; use pano_sift_pyramid");
    const size_t plane = (size_t)ctx->oct_h[octave] * ctx->oct_w[octave];
    const float *src = dog ? ctx->dog + ctx->dog_off[octave][level] : ctx->pyr + ctx->gauss_off[octave][level];
    PANO_HIP(ctx, hipMemcpyAsync(out, src + (size_t)frame * plane, plane * sizeof(float),
                                 hipMemcpyDeviceToDevice, ctx->stream));
    return PANO_OK;
}

int pano_harris(pano_ctx *ctx, const uint8_t *bgr, int n, int h, int w, int max_points,
                int32_t *xy, float *desc, int32_t *counts) {
    if (!ctx) return PANO_E_ARG;
    return launch_harris(ctx, bgr, n, h, w, max_points, xy, desc, counts);
}

int pano_match(pano_ctx *ctx, const float *desc, const int32_t *counts, int cap,
               const int32_t *pairs, int n_pairs, int exact_int, int32_t *best, float *d1,
               float *d2) {
    if (!ctx || !pairs) return PANO_E_ARG;
    return launch_match(ctx, desc, counts, cap, pairs, n_pairs, exact_int, best, d1, d2);
}

int pano_match_u8(pano_ctx *ctx, const uint8_t *desc_u8, const int32_t *norms, const int32_t *counts,
                  int cap, const int32_t *pairs, int n_pairs, int32_t *best, float *d1, float *d2) {
    if (!ctx || !pairs) return PANO_E_ARG;
    return launch_match_u8(ctx, desc_u8, norms, counts, cap, pairs, n_pairs, best, d1, d2);
}

int pano_pair_shifts(pano_ctx *ctx, const pano_kp *kps, const int32_t *xy_i32,
                     const int32_t *counts, int cap, const int32_t *pairs, int n_pairs,
                     const int32_t *best, const float *d1, const float *d2, double desc_thresh,
                     double ratio, double ransac_thr, pano_pair_rec *recs) {
    if (!ctx || !pairs) return PANO_E_ARG;
    return launch_pair_shifts(ctx, kps, xy_i32, counts, cap, pairs, n_pairs, best, d1, d2,
                              desc_thresh, ratio, ransac_thr, recs);
}

int pano_pair_homography(pano_ctx *ctx, const pano_kp *kps, const int32_t *counts, int cap,
                         const int32_t *pairs, int n_pairs, const int32_t *best, const float *d1,
                         const float *d2, double desc_thresh, double ratio, double reproj_thr, int n_hyp,
                         uint64_t seed, int min_good, pano_homography_rec *recs, uint8_t *mask) {
    if (!ctx || !pairs) return PANO_E_ARG;
    return launch_pair_homography(ctx, kps, counts, cap, pairs, n_pairs, best, d1, d2, desc_thresh, ratio,
                                  reproj_thr, n_hyp, seed, min_good, recs, mask);
}

int pano_ransac_translate(pano_ctx *ctx, const double *moves, int k, double thr, int32_t *out) {
    if (!ctx) return PANO_E_ARG;
    return launch_ransac_translate(ctx, moves, k, thr, out);
}

int pano_composite(pano_ctx *ctx, const uint8_t *frames, const uint8_t *colnz, int n, int h,
                   int w, const pano_step *steps, const int32_t *first_xy, uint8_t *canvas, int H,
                   int W) {
    if (!ctx) return PANO_E_ARG;
    return launch_composite(ctx, frames, colnz, n, h, w, steps, first_xy, canvas, H, W);
}

int pano_composite_bbox(pano_ctx *ctx, const uint8_t *frames, const uint8_t *colnz, int n,
                        int h, int w, const pano_step *steps, const int32_t *first_xy,
                        uint8_t *canvas, int H, int W, int black_threshold, int32_t *bbox) {
    if (!ctx) return PANO_E_ARG;
    return launch_composite_bbox(ctx, frames, colnz, n, h, w, steps, first_xy, canvas, H, W,
                                 black_threshold, bbox);
}

size_t pano_plan_device_bytes(void) { return plan_device_bytes(); }

int pano_plan_device(pano_ctx *ctx, const pano_pair_rec *recs, int n, int h, int w, int int_shifts,
                     int Hcap, int Wcap, void *plan) {
    if (!ctx) return PANO_E_ARG;
    return launch_plan_device(ctx, recs, n, h, w, int_shifts, Hcap, Wcap, plan);
}

int pano_band_layout_row(pano_ctx *ctx, const void *plan, const int32_t *band, const int32_t *bbox,
                         int64_t *row) {
    if (!ctx) return PANO_E_ARG;
    return launch_band_layout_row(ctx, plan, band, bbox, (long long *)row);
}

int pano_band_plan(pano_ctx *ctx, const void *plan, int f0, int n_local, int w, int Wcap,
                   void *local_plan, int32_t *band) {
    if (!ctx) return PANO_E_ARG;
    return launch_band_plan(ctx, plan, f0, n_local, w, Wcap, local_plan, band);
}

int pano_composite_planned(pano_ctx *ctx, const uint8_t *frames, const uint8_t *colnz, int n, int h,
                           int w, const void *plan, uint8_t *canvas, int Hcap, int Wcap,
                           int black_threshold, int32_t *bbox) {
    if (!ctx) return PANO_E_ARG;
    return launch_composite_planned(ctx, frames, colnz, n, h, w, plan, canvas, Hcap, Wcap,
                                    black_threshold, bbox);
}

int pano_plan_composite_device(pano_ctx *ctx, const pano_pair_rec *recs, const uint8_t *frames,
                               const uint8_t *colnz, int n, int h, int w, int int_shifts, void *plan,
                               uint8_t *canvas, int Hcap, int Wcap, int black_threshold, int32_t *bbox) {
    if (!ctx) return PANO_E_ARG;
    return launch_plan_composite_device(ctx, recs, frames, colnz, n, h, w, int_shifts, plan, canvas, Hcap,
                                        Wcap, black_threshold, bbox);
}

int pano_composite_sequential(pano_ctx *ctx, const uint8_t *frames, const uint8_t *colnz, int n,
                              int h, int w, const pano_step *steps, const int32_t *first_xy,
                              uint8_t *canvas, int H, int W) {
    if (!ctx) return PANO_E_ARG;
    return launch_composite_seq(ctx, frames, colnz, n, h, w, steps, first_xy, canvas, H, W);
}

int pano_blend_two(pano_ctx *ctx, const uint8_t *A, int hA, int wA, const uint8_t *B, int hB,
                   int wB, const int32_t *geom, double overlap, uint8_t *out) {
    if (!ctx) return PANO_E_ARG;
    return launch_blend_two(ctx, A, hA, wA, B, hB, wB, geom, overlap, out);
}

int pano_gray_bbox(pano_ctx *ctx, const uint8_t *img, int H, int W, int thr, int32_t *bbox) {
    if (!ctx) return PANO_E_ARG;
    return launch_gray_bbox(ctx, img, H, W, thr, bbox);
}

int pano_jpeg_info(const uint8_t *buf, size_t len, int *h, int *w, int *ncomp) {
    pj::Parsed P;
    std::string err;
    int rc = pj::parse(buf, len, &P, &err);
    if (rc) return rc;
    pj::Frame F;
    rc = pj::plan_frame(P, &F, &err);
    if (rc) return rc;
    if (h) *h = P.h;
    if (w) *w = P.w;
    if (ncomp) *ncomp = P.ncomp;
    return PANO_OK;
}

int pano_jpeg_decode(pano_ctx *ctx, int n, const uint8_t *const *bufs, const size_t *lens, uint8_t *bgr,
                     int h, int w, int32_t *status) {
    if (!ctx) return PANO_E_ARG;
    if (n <= 0 || !bufs || !lens || !bgr || h <= 0 || w <= 0)
        return pano_fail(ctx, PANO_E_ARG, "pano_jpeg_decode: bad arguments");
    if (ctx->capturing)
        return pano_fail(ctx, PANO_E_UNSUPPORTED, "pano_jpeg_decode reads host files: not capturable");
    return launch_jpeg_decode(ctx, n, bufs, lens, bgr, h, w, status);
}

int pano_jpeg_stats(pano_ctx *ctx, int32_t *h_stats, int n) {
    if (!ctx || !h_stats || n <= 0) return PANO_E_ARG;
    return jpeg_last_stats(ctx, h_stats, n);
}

int pano_jpeg_encode(pano_ctx *ctx, const uint8_t *bgr, int h, int w, int64_t pitch, int quality,
                     uint8_t *h_out, size_t cap, size_t *out_len) {
    if (!ctx) return PANO_E_ARG;
    if (!bgr || h <= 0 || w <= 0 || h > 65535 || w > 65535 || pitch < 3 * (int64_t)w || quality < 1 || quality > 100)
        return pano_fail(ctx, PANO_E_ARG, "pano_jpeg_encode: bad arguments");
    if (ctx->capturing)
        return pano_fail(ctx, PANO_E_UNSUPPORTED, "pano_jpeg_encode writes host memory: not capturable");
    return launch_jpeg_encode(ctx, bgr, h, w, pitch, quality, h_out, cap, out_len);
}

int pano_prof_enable(pano_ctx *ctx, int kernel_class) {
    if (!ctx || kernel_class < -1 || kernel_class > PK_COUNT) return PANO_E_ARG;
    ctx->prof.kernel = kernel_class;
    ctx->prof.used = 0;
    return PANO_OK;
}

int pano_prof_read(pano_ctx *ctx, int kernel_class, int *launches, double *total_ms,
                   double *min_ms, double *max_ms) {
    if (!ctx || !launches || !total_ms) return PANO_E_ARG;
    PANO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    int n = 0;
    double tot = 0.0, mn = 1e30, mx = 0.0;
    for (size_t i = 0; i + 1 < ctx->prof.used; i += 2) {
        if (kernel_class != PK_COUNT && ctx->prof.kid[i / 2] != kernel_class) continue;
        float ms = 0.0f;
        PANO_HIP(ctx, hipEventElapsedTime(&ms, ctx->prof.ev[i], ctx->prof.ev[i + 1]));
        ++n;
        tot += ms;
        mn = ms < mn ? ms : mn;
        mx = ms > mx ? ms : mx;
    }
    *launches = n;
    *total_ms = tot;
    if (min_ms) *min_ms = n ? mn : 0.0;
    if (max_ms) *max_ms = mx;
    ctx->prof.used = 0;
    return PANO_OK;
}

// ------------------------------------------------------------------ hipGraph capture
struct pano_graph {
    hipGraphExec_t exec = nullptr;
    std::vector<hipEvent_t> ev;          // profiler event pairs captured into the graph
    std::vector<int> kid;
};

int pano_graph_begin(pano_ctx *ctx) {
    if (!ctx || ctx->capturing) return PANO_E_ARG;
    sift_join_tail(ctx);
    sift_join_x(ctx);
    ctx->cap_prof_start = ctx->prof.used;
    PANO_HIP(ctx, hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeRelaxed));
    ctx->capturing = true;
    return PANO_OK;
}

int pano_graph_end(pano_ctx *ctx, pano_graph **out) {
    if (!ctx || !out || !ctx->capturing) return PANO_E_ARG;
    *out = nullptr;
    sift_join_tail(ctx);
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(ctx->stream, &g);
    ctx->capturing = false;
    ProfState &p = ctx->prof;
    const size_t a = ctx->cap_prof_start, b = p.used;
    if (e != hipSuccess || !g) {
        p.used = a;
        return pano_hip_check(ctx, e != hipSuccess ? e : hipErrorUnknown, "hipStreamEndCapture");
    }
    pano_graph *pg = new pano_graph;
    e = hipGraphInstantiate(&pg->exec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) {
        delete pg;
        p.used = a;
        return pano_hip_check(ctx, e, "hipGraphInstantiate");
    }
    // the graph owns the event pairs recorded during capture (they are re-recorded on
    // every replay); take them out of the context's pool
    for (size_t i = a; i + 1 < b; i += 2) {
        pg->ev.push_back(p.ev[i]);
        pg->ev.push_back(p.ev[i + 1]);
        pg->kid.push_back(p.kid[i / 2]);
    }
    p.ev.erase(p.ev.begin() + a, p.ev.begin() + b);
    p.kid.erase(p.kid.begin() + a / 2, p.kid.begin() + b / 2);
    p.used = a;
    *out = pg;
    return PANO_OK;
}

int pano_graph_launch(pano_ctx *ctx, pano_graph *g) {
    if (!ctx || !g) return PANO_E_ARG;
    PANO_HIP(ctx, hipGraphLaunch(g->exec, ctx->stream));
    return PANO_OK;
}

int pano_graph_launch_stream(pano_ctx *ctx, pano_graph *g, void *stream) {
    if (!ctx || !g) return PANO_E_ARG;
    PANO_HIP(ctx, hipGraphLaunch(g->exec, stream ? (hipStream_t)stream : ctx->stream));
    return PANO_OK;
}

int pano_graph_launch_sync(pano_ctx *ctx, pano_graph *g, void *stream) {
    if (!ctx || !g) return PANO_E_ARG;
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    PANO_HIP(ctx, hipGraphLaunch(g->exec, s));
    PANO_HIP(ctx, hipStreamSynchronize(s));
    return PANO_OK;
}

int pano_copy_async(pano_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (!ctx || (bytes && (!dst || !src))) return PANO_E_ARG;
    // small copies run as a kernel: a graph kernel node, no blit / SDMA node; large ones stay
    // hipMemcpyAsync.  Only when both pointers are device memory or registered (pinned) host
    // memory with a device address -- anything else (pageable memory) takes the memcpy path
    if (bytes && bytes <= (1u << 20)) {
        void *dd = device_address(dst), *ds = device_address(const_cast<void *>(src));
        if (dd && ds) return launch_copy(ctx, dd, ds, bytes);
    }
    if (bytes) PANO_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, ctx->stream));
    return PANO_OK;
}

int pano_graph_prof(pano_graph *g, int kernel_class, int *launches, double *total_ms) {
    if (!g || !launches || !total_ms) return PANO_E_ARG;
    int n = 0;
    double tot = 0.0;
    for (size_t i = 0; i + 1 < g->ev.size(); i += 2) {
        if (kernel_class != PK_COUNT && g->kid[i / 2] != kernel_class) continue;
        float ms = 0.0f;
        const hipError_t e = hipEventElapsedTime(&ms, g->ev[i], g->ev[i + 1]);
        if (e != hipSuccess) return PANO_E_HIP - 100 * (int)e;   // caller decodes the HIP code
        ++n;
        tot += ms;
    }
    *launches = n;
    *total_ms = tot;
    return PANO_OK;
}

int pano_graph_destroy(pano_graph *g) {
    if (!g) return PANO_OK;
    if (g->exec) (void)hipGraphExecDestroy(g->exec);
    for (hipEvent_t e : g->ev) (void)hipEventDestroy(e);
    delete g;
    return PANO_OK;
}

}  // extern "C"
