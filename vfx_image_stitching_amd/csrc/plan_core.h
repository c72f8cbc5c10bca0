// plan_core.h -- the composite geometry of the reference's mosaic loop, shared by the host plan
// (pano_plan_composite), the device plan kernel (plan_device, blend.hip) and the host sanitizer
// harness (tools/host_fuzz.cpp).  Exact replay of the Python scalar arithmetic of
// blend_two_images (image_stitching_sift.py:156-202), pad_image (:139-153) and run_panorama's
// top padding (:374-376).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/pano.h"

// plan inputs beyond +-2^24 px (non-finite ones included) are refused; canvases beyond 2^30 px
// per side overflow
constexpr double kPlanMaxOffset = 16777216.0;
constexpr int kPlanMaxSide = 1 << 30;

static __host__ __device__ void pad_place(long long mx, long long my, int h, int w, int *top, int *left, int *ph,
                      int *pw) {
    *left = mx >= 0 ? (int)mx : 0;
    *top = my >= 0 ? (int)my : 0;
    *pw = w + (int)(mx >= 0 ? mx : -mx);
    *ph = h + (int)(my >= 0 ? my : -my);
}

static __host__ __device__ int blend_geometry(double dx, double dy, const double *ref4, int hA, int wA,
                                              int hB, int wB, int32_t *geom, double *overlap) {
    double r00 = ref4[0], r01 = ref4[1], r10 = ref4[2], r11 = ref4[3];
    const int swapped = dx < 0;
    if (swapped) {
        dx = -dx;
        dy = -dy;
        double t0 = r00, t1 = r01;
        r00 = r10; r01 = r11; r10 = t0; r11 = t1;
        int th = hA, tw = wA;
        hA = hB; wA = wB; hB = th; wB = tw;
    }
    (void)r01; (void)r11;
    const double padA_x = ((double)(wB - wA) + r00) - r10;
    const double padB_x = r00 - r10;
    *overlap = (r10 - r00) + wA;
    const long long mxA = (long long)nearbyint(-padA_x), myA = (long long)nearbyint(-dy);
    const long long mxB = (long long)nearbyint(padB_x), myB = (long long)nearbyint(dy);
    int tA, lA, hhA, wwA, tB, lB, hhB, wwB;
    pad_place(mxA, myA, hA, wA, &tA, &lA, &hhA, &wwA);
    pad_place(mxB, myB, hB, wB, &tB, &lB, &hhB, &wwB);
    // geom: ayA axA ayB axB HH WW swapped (A/B are the post-swap roles)
    geom[0] = tA; geom[1] = lA; geom[2] = tB; geom[3] = lB;
    geom[4] = hhA > hhB ? hhA : hhB;
    geom[5] = wwA > wwB ? wwA : wwB;
    geom[6] = swapped;
    geom[7] = 0;
    return PANO_OK;
}

// shifts / pairs: element i - 1 of step i, read through the accessors (host arrays, or the
// device records with drift correction applied on the fly); tmp: 5 x n ints of scratch
template <typename SH, typename PR>
static __host__ __device__ int plan_core(SH shift, PR pair, int n, int h, int w, pano_step *steps,
                                         int32_t *first_xy, int32_t *canvas_hw, int32_t *tmp) {
    if (h <= 0 || w <= 0 || h > kPlanMaxSide / 2 || w > kPlanMaxSide / 2) return PANO_E_ARG;
    int Hm = h, Wm = w;
    int32_t *yM = tmp, *xM = tmp + n, *yF = tmp + 2 * n, *xF = tmp + 3 * n, *padtop = tmp + 4 * n;
    for (int i = 1; i < n; ++i) {
        // run_panorama pads the new frame to the mosaic height first (:374-376)
        const int diff = Hm - h;
        int fh = h, ptop = 0;
        if (diff > 0) { fh = h + diff; ptop = diff; }
        else if (diff < 0) { fh = h - diff; ptop = 0; }
        int32_t g[8];
        double ov;
        // blend_two_images(shift, pair, imgA = mosaic, imgB = frame)
        double sd[2], pd[4];
        shift(i - 1, sd);
        pair(i - 1, pd);
        // a caller's garbage (NaN, inf, offsets beyond any canvas) is refused before it reaches
        // an integer conversion; canvases stay below 2^30 px per side so no int can overflow
        for (int q = 0; q < 2; ++q) if (!(fabs(sd[q]) <= kPlanMaxOffset)) return PANO_E_ARG;
        for (int q = 0; q < 4; ++q) if (!(fabs(pd[q]) <= kPlanMaxOffset)) return PANO_E_ARG;
        int rc = blend_geometry(sd[0], sd[1], pd, Hm, Wm, fh, w, g, &ov);
        if (rc) return rc;
        if (g[4] > kPlanMaxSide || g[5] > kPlanMaxSide) return PANO_E_OVERFLOW;
        const int swapped = g[6];
        // post-swap A is the frame when swapped
        const int ay = g[0], ax = g[1], by = g[2], bx = g[3];
        if (swapped) { yF[i] = ay; xF[i] = ax; yM[i] = by; xM[i] = bx; }
        else { yM[i] = ay; xM[i] = ax; yF[i] = by; xF[i] = bx; }
        padtop[i] = ptop;
        pano_step &s = steps[i - 1];
        s.canvas_h = g[4];
        s.canvas_w = g[5];
        s.frame_is_a = swapped;
        s.pad = 0;
        s.overlap_range = ov;
        Hm = g[4];
        Wm = g[5];
    }
    // origins: the last canvas is the final one; step i's input mosaic sits at (yM, xM)
    int oy = 0, ox = 0;
    for (int i = n - 1; i >= 1; --i) {
        pano_step &s = steps[i - 1];
        s.canvas_y = oy;
        s.canvas_x = ox;
        s.frame_y = oy + yF[i] + padtop[i];
        s.frame_x = ox + xF[i];
        oy += yM[i];
        ox += xM[i];
    }
    first_xy[0] = ox;
    first_xy[1] = oy;
    canvas_hw[0] = Hm;
    canvas_hw[1] = Wm;
    return PANO_OK;
}

// ---- the same plan as per-step constants plus a short serial chain (plan_device's form)
// plan_core's only loop-carried state is the mosaic size (Hm, Wm); everything else a step
// needs is a function of its own shift and pair.  plan_step_const computes that part (in
// parallel, one step per lane), plan_chain_step the rest given (Hm, Wm): the same expressions
// in the same order as plan_core / blend_geometry / pad_place, so the same doubles and ints
// (tools/host_fuzz.cpp checks plan_fast against plan_core on every accepted and refused plan).
struct PlanStepConst {
    double r00, r10;          // ref4[0], ref4[2] after the dx < 0 swap
    int32_t swapped;
    int32_t myA, myB, mxB;    // nearbyint(-dy), nearbyint(dy) (dy after the swap), nearbyint(r00 - r10)
    int32_t bad;              // a shift / pair value NaN, infinite or beyond kPlanMaxOffset
};

static __host__ __device__ inline PlanStepConst plan_step_const(double dx, double dy, const double *ref4) {
    PlanStepConst c{};
    bool bad = !(fabs(dx) <= kPlanMaxOffset) || !(fabs(dy) <= kPlanMaxOffset);
    for (int q = 0; q < 4; ++q) bad = bad || !(fabs(ref4[q]) <= kPlanMaxOffset);
    c.bad = bad;
    if (bad) return c;
    double r00 = ref4[0], r10 = ref4[2];
    c.swapped = dx < 0;
    if (c.swapped) {
        dy = -dy;
        const double t = r00;
        r00 = r10;
        r10 = t;
    }
    c.r00 = r00;
    c.r10 = r10;
    c.myA = (int32_t)(long long)nearbyint(-dy);          // |dy| <= 2^24: exact in int32
    c.myB = (int32_t)(long long)nearbyint(dy);
    c.mxB = (int32_t)(long long)nearbyint(r00 - r10);    // padB_x = r00 - r10
    return c;
}

struct PlanStepOut {
    int32_t H, W;             // the step's canvas (the next Hm, Wm)
    int32_t yM, xM, yF, xF;   // mosaic / frame placement in it
    int32_t ptop;             // run_panorama's top padding of the frame
    int32_t rc;
    double ov;                // overlap_range
};

// The loop-carried part alone: the step's canvas size from the mosaic size.  plan_chain_step
// computes the same H, W (and the placement) with the same expressions; plan_device runs this
// serially over the steps and plan_chain_step afterwards, one step per lane.  |padA_x| < 2^31
// (Wm <= kPlanMaxSide, w <= kPlanMaxSide / 2, |r| <= 2^24), so the int conversion is the
// long long one of pad_place.
static __host__ __device__ inline void plan_chain_hw(const PlanStepConst &c, int Hm, int Wm, int h, int w,
                                                     int &H, int &W) {
    const int diff = Hm - h;
    const int fh = diff > 0 ? h + diff : (diff < 0 ? h - diff : h);
    int hA = Hm, wA = Wm, hB = fh, wB = w;
    if (c.swapped) {
        hA = fh; wA = w; hB = Hm; wB = Wm;
    }
    const int mxA = (int)nearbyint(-(((double)(wB - wA) + c.r00) - c.r10));
    const int hhA = hA + (c.myA >= 0 ? c.myA : -c.myA), hhB = hB + (c.myB >= 0 ? c.myB : -c.myB);
    const int wwA = wA + (mxA >= 0 ? mxA : -mxA), wwB = wB + (c.mxB >= 0 ? c.mxB : -c.mxB);
    H = hhA > hhB ? hhA : hhB;
    W = wwA > wwB ? wwA : wwB;
}

static __host__ __device__ inline PlanStepOut plan_chain_step(const PlanStepConst &c, int Hm, int Wm, int h, int w) {
    PlanStepOut o{};
    const int diff = Hm - h;
    int fh = h, ptop = 0;
    if (diff > 0) { fh = h + diff; ptop = diff; }
    else if (diff < 0) { fh = h - diff; ptop = 0; }
    int hA = Hm, wA = Wm, hB = fh, wB = w;
    if (c.swapped) {
        hA = fh; wA = w; hB = Hm; wB = Wm;
    }
    const double padA_x = ((double)(wB - wA) + c.r00) - c.r10;
    o.ov = (c.r10 - c.r00) + wA;
    const long long mxA = (long long)nearbyint(-padA_x);
    int tA, lA, hhA, wwA, tB, lB, hhB, wwB;
    pad_place(mxA, c.myA, hA, wA, &tA, &lA, &hhA, &wwA);
    pad_place(c.mxB, c.myB, hB, wB, &tB, &lB, &hhB, &wwB);
    plan_chain_hw(c, Hm, Wm, h, w, o.H, o.W);    // = max(hhA, hhB), max(wwA, wwB)
    (void)hhA; (void)hhB; (void)wwA; (void)wwB;
    o.rc = (o.H > kPlanMaxSide || o.W > kPlanMaxSide) ? PANO_E_OVERFLOW : PANO_OK;
    if (c.swapped) { o.yF = tA; o.xF = lA; o.yM = tB; o.xM = lB; }
    else { o.yM = tA; o.xM = lA; o.yF = tB; o.xF = lB; }
    o.ptop = ptop;
    return o;
}

// Host loop form of the above (tools/host_fuzz.cpp compares it with plan_core).
template <typename SH, typename PR>
static __host__ __device__ int plan_fast(SH shift, PR pair, int n, int h, int w, pano_step *steps,
                                         int32_t *first_xy, int32_t *canvas_hw, int32_t *tmp) {
    if (h <= 0 || w <= 0 || h > kPlanMaxSide / 2 || w > kPlanMaxSide / 2) return PANO_E_ARG;
    int Hm = h, Wm = w;
    int32_t *yM = tmp, *xM = tmp + n, *yF = tmp + 2 * n, *xF = tmp + 3 * n, *padtop = tmp + 4 * n;
    for (int i = 1; i < n; ++i) {
        double sd[2], pd[4];
        shift(i - 1, sd);
        pair(i - 1, pd);
        const PlanStepConst c = plan_step_const(sd[0], sd[1], pd);
        if (c.bad) return PANO_E_ARG;
        const PlanStepOut o = plan_chain_step(c, Hm, Wm, h, w);
        if (o.rc) return o.rc;
        yM[i] = o.yM; xM[i] = o.xM; yF[i] = o.yF; xF[i] = o.xF; padtop[i] = o.ptop;
        pano_step &s = steps[i - 1];
        s.canvas_h = o.H;
        s.canvas_w = o.W;
        s.frame_is_a = c.swapped;
        s.pad = 0;
        s.overlap_range = o.ov;
        Hm = o.H;
        Wm = o.W;
    }
    int oy = 0, ox = 0;
    for (int i = n - 1; i >= 1; --i) {
        pano_step &s = steps[i - 1];
        s.canvas_y = oy;
        s.canvas_x = ox;
        s.frame_y = oy + yF[i] + padtop[i];
        s.frame_x = ox + xF[i];
        oy += yM[i];
        ox += xM[i];
    }
    first_xy[0] = ox;
    first_xy[1] = oy;
    canvas_hw[0] = Hm;
    canvas_hw[1] = Wm;
    return PANO_OK;
}

