/*
 * pano.h -- C-ABI of libpano.so, the MI355X (gfx950) panorama-stitching hot path.
 *
 * The reference (sapt36/VFX_Image_Stitching) is Python with no FFI layer; its "operator
 * API" is a set of module-level functions.  Each entry point below replaces one of them
 * (file:line in /root/reference) and is what a ctypes binding of that function calls
 * (see INTEGRATION.md).  Conventions:
 *
 *   - Every pointer named d_* is DEVICE memory (hipMalloc / torch.cuda); h_* is host.
 *   - Calls are asynchronous on the context's stream unless documented otherwise.
 *   - Images are uint8 HWC BGR (row-major, 3 channels), frames of a batch share h, w.
 *   - Return value: PANO_OK (0) or a negative PANO_E_* code; pano_last_error() has the
 *     message.  Nothing throws across the ABI.
 *   - Variable-length outputs use a caller capacity + a device counter; a counter larger
 *     than the capacity means entries were dropped (PANO_E_OVERFLOW after pano_sync()).
 *   - No entry point allocates or synchronises inside the stream order except
 *     pano_ctx_reserve() and pano_sync(), so launch sequences are hipGraph-capturable
 *     after a reserve.
 */
#ifndef PANO_H
#define PANO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PANO_OK            0
#define PANO_E_ARG        -1
#define PANO_E_HIP        -2
#define PANO_E_OVERFLOW   -3
#define PANO_E_NOMATCH    -4
#define PANO_E_UNSUPPORTED -5

#define PANO_DESC_DIM 128

typedef struct pano_ctx pano_ctx;

/* cv2.KeyPoint as the reference fills it (sift_impl.py:206-210, 290-291): float32 fields,
 * octave = octave + 256*layer + 65536*round((u2+0.5)*255), in input-image coordinates
 * after convert_keypoints_to_input_image_size (sift_impl.py:333-343). */
typedef struct pano_kp {
    float x, y, size, angle, response;
    int32_t octave;
} pano_kp;

/* compute_keypoints_and_descriptors kwargs + the hard-coded defaults of the stage
 * functions it chains (sift_impl.py:15, 117, 170, 247, 361-362). */
typedef struct pano_sift_params {
    double sigma;              /* 1.6   */
    int32_t num_intervals;     /* 3     */
    double assumed_blur;       /* 0.5   */
    int32_t border;            /* 5     */
    double contrast_threshold; /* 0.04  */
    double eigen_ratio;        /* 10    */
    int32_t max_iter;          /* 5     */
    double radius_factor;      /* 3     */
    double peak_ratio;         /* 0.8   */
    double scale_factor;       /* 1.5   */
    double scale_multiplier;   /* 3     */
    double descriptor_max;     /* 0.2   */
} pano_sift_params;

/* One per-pair result: ransac()'s best move and best pair (image_stitching_sift.py:86-111)
 * plus bookkeeping.  Coordinates are the float32 keypoint coordinates widened to double. */
typedef struct pano_pair_rec {
    double dx, dy;             /* best move = ptA - ptB                                  */
    double xA, yA, xB, yB;     /* the winning match                                      */
    int32_t n_matches;         /* matches passing the descriptor threshold               */
    int32_t votes;             /* inliers of the winner                                  */
    int32_t best;              /* index of the winning match in match order, -1 if none  */
    int32_t status;            /* PANO_OK, PANO_E_NOMATCH, or PANO_E_OVERFLOW (a frame of
                                  the pair has more keypoints than the capacity: rerun
                                  with a larger cap -- its count is in d_counts)          */
} pano_pair_rec;

/* Placement of one compositing step in the final canvas (computed on the host from the
 * per-pair records by pano_plan_composite; image_stitching_sift.py:156-202, 369-381). */
typedef struct pano_step {
    int32_t frame_x, frame_y;  /* top-left of the new frame's h x w content, final canvas   */
    int32_t canvas_x, canvas_y, canvas_h, canvas_w; /* the step's whole canvas, final coords */
    int32_t frame_is_a;        /* 1: the new frame is imgA of the blend (dx < 0 swap branch) */
    int32_t pad;
    double overlap_range;      /* blend_two_images overlap_range (0 -> alpha = 0)        */
} pano_step;

/* ---------------------------------------------------------------- context */
int pano_ctx_create(int device, void *hip_stream, pano_ctx **out);
int pano_ctx_destroy(pano_ctx *ctx);
int pano_ctx_set_stream(pano_ctx *ctx, void *hip_stream);
/* Scheduling options of this context (bit set; results identical in every setting).
 * PANO_CTX_TAIL_MAIN: the small-octave blur tail on the context's own stream instead of a
 * forked side stream -- fewer cross-stream graph edges, best when other contexts' work fills
 * the device (pipeline.StitchPool); alone, the side stream hides the tail.
 * No reference counterpart. */
#define PANO_CTX_TAIL_MAIN 1
/* PANO_CTX_MATCH_WHOLE: the distance GEMM's query tiles walk every candidate tile themselves
 * (no candidate splits, no partials to fold): fewer, longer workgroups, better when the device
 * is already full (StitchPool), worse for one stitch's latency.  Same results. */
#define PANO_CTX_MATCH_WHOLE 2
int pano_ctx_set_flags(pano_ctx *ctx, int flags);
/* Pre-size scratch for n frames of h x w with cap keypoints per frame (allocates). */
int pano_ctx_reserve(pano_ctx *ctx, int n, int h, int w, int cap);
/* Free every scratch buffer the context grew (after a large batch; the next call re-allocates
 * what it needs).  Waits for the stream; bumps the generation (captured graphs are stale).
 * No reference counterpart: memory management of this library. */
int pano_ctx_release_scratch(pano_ctx *ctx);
int pano_sync(pano_ctx *ctx);
const char *pano_last_error(pano_ctx *ctx);
/* Scratch generation: incremented whenever the context frees and re-allocates scratch
 * (a call needing more than it has).  A hipGraph captured (pano_graph_begin/end) under an
 * older generation references freed scratch and must be re-captured, not replayed. */
uint64_t pano_ctx_generation(pano_ctx *ctx);
const char *pano_version(void);
void pano_sift_default_params(pano_sift_params *p);
/* Host-only helpers (no GPU): the scalar plan of S1/S2 and the f32 Gaussian taps. */
int pano_sift_plan(const pano_sift_params *p, int h, int w, int *n_octaves, int *n_levels,
                   double *sigma_base, double *sigma_levels);
int pano_sift_taps(double sigma, double *taps_out /* >= 64 */, int *n_taps);

/* ---------------------------------------------------------------- C1
 * cylindrical_projection(img_bgr, focal_len)  image_stitching_sift.py:117-136
 * Batched: d_src/d_dst [n][h][w][3]; h_focal[n].  Optional d_colnz [n][w] receives
 * "column has any non-zero byte" flags of each output (used by the compositor). */
int pano_cylindrical(pano_ctx *ctx, const uint8_t *d_src, uint8_t *d_dst, int n, int h, int w,
                     const double *h_focal, uint8_t *d_colnz);

/* ---------------------------------------------------------------- S0..S9
 * compute_keypoints_and_descriptors(image, sigma, num_intervals, assumed_blur,
 * image_border_width)  sift_impl.py:15-39.  Batched over n frames of h x w BGR uint8.
 * d_kps [n][cap], d_desc [n][cap][128] float32 (integer valued), d_counts [n] (may exceed
 * cap on overflow).  Keypoints come out in the reference's sorted, de-duplicated order. */
int pano_sift(pano_ctx *ctx, const uint8_t *d_bgr, int n, int h, int w,
              const pano_sift_params *params, pano_kp *d_kps, float *d_desc, int cap,
              int32_t *d_counts);

/* pano_sift with the descriptors as bytes (the batched Stitcher's form, what the distance GEMM
 * reads): d_desc_u8 [n][cap][128] uint8 (the same integer values) and d_norms [n][cap] int32
 * squared norms (exact).  A quarter of the f32 form's bytes; no repacking before matching. */
int pano_sift_u8(pano_ctx *ctx, const uint8_t *d_bgr, int n, int h, int w,
                 const pano_sift_params *params, pano_kp *d_kps, uint8_t *d_desc_u8,
                 int32_t *d_norms, int cap, int32_t *d_counts);

/* Stage access for the GUI-facing stage functions (sift_impl.py:45-111):
 * after pano_sift_pyramid the Gaussian / DoG pyramid of frame `frame` stays in the
 * context: level 0..num_intervals+2 (Gaussian) / 0..num_intervals+1 (DoG).  After pano_sift
 * every DoG level is there too, but of the Gaussian levels only those the keypoint stages
 * read (levels 1..num_intervals): copying the others returns PANO_E_UNSUPPORTED.
 * Copies one level to d_out (h_o x w_o float32); pano_sift_level_shape reports its size. */
int pano_sift_pyramid(pano_ctx *ctx, const uint8_t *d_bgr, int n, int h, int w,
                      const pano_sift_params *params);
int pano_sift_level_shape(pano_ctx *ctx, int octave, int *h_out, int *w_out, int *n_octaves);
int pano_sift_copy_level(pano_ctx *ctx, int frame, int octave, int level, int dog, float *d_out);

/* Stage functions on caller data (sift_visualizeUI.py:104-115 calls them one by one):
 *
 * pano_sift_base         generate_base_image(image, sigma, assumed_blur)  sift_impl.py:45-56
 *                        d_gray [n][h][w] f32 gray -> d_base [n][2h][2w] f32 (x2 INTER_LINEAR,
 *                        then GaussianBlur sigma_diff).  Exact for integer-valued gray.
 * pano_sift_pyramid_base generate_gaussian_images(base, num_octaves, kernels) + generate_DoG_images
 *                        sift_impl.py:82-111 on ANY f32 base d_base [n][H0][W0]: the base is
 *                        level 0 of octave 0; every Gaussian and DoG level stays resident
 *                        (pano_sift_copy_level reads them back).  The kernels are those of
 *                        params (sigma, num_intervals).
 * pano_sift_pyramid_kernels  the same with the caller's kernel list (any gaussian_kernels, not
 *                        only generate_gaussian_kernels' : sift_impl.py:89-92 blurs level l - 1
 *                        by kernels[l]): n_kernels levels per octave (3..8), each kernel
 *                        cv2.GaussianBlur's float32 one (ksize = round(8 s + 1) | 1, at most 64
 *                        taps: s < 7.9); outside those limits PANO_E_UNSUPPORTED.
 * pano_sift_reserve_levels + pano_sift_set_level
 *                        lay out a resident pyramid for n frames with octave 0 of H0 x W0 and
 *                        upload caller levels into it (Gaussian: dog = 0, DoG: dog = 1), e.g.
 *                        pyramids the caller built or edited; pano_sift_dog recomputes every
 *                        DoG level from the resident Gaussian levels (generate_DoG_images).
 * pano_sift_extrema      find_scale_space_extrema(gaussian_images, dog_images, ...)
 *                        sift_impl.py:117-140 on the resident pyramid: the oriented keypoints
 *                        BEFORE remove_duplicate_keypoints, in the reference's scan order
 *                        (octave, layer, y, x; orientations in peak order), base coordinates.
 *                        d_raw [n][cap], d_counts [n] (> cap: entries dropped; -1: an internal
 *                        scratch capacity overflowed, PANO_E_OVERFLOW from pano_sync).
 * pano_sift_describe     generate_descriptors(keypoints, gaussian_images)  sift_impl.py:361-526
 *                        for caller keypoints (input-image coordinates, converted octave
 *                        field) d_kps [n][cap] / d_counts [n] on the resident pyramid, which
 *                        must hold every Gaussian level (pano_sift_pyramid, _pyramid_base or
 *                        _reserve_levels): d_desc [n][cap][128] f32.  A keypoint whose octave
 *                        or layer lies outside the pyramid gets a zero descriptor. */
/* Per-candidate helpers of find_scale_space_extrema on caller data of ONE octave (the batched
 * kernels' own device code, for callers of the reference's scalar helpers):
 *
 * pano_sift_localize     localize_extremum_via_quadratic_fit(x, y, layer, octave, num_intervals,
 *                        dog_octave, sigma, contrast_threshold, border, eigen_ratio, max_iter)
 *                        sift_impl.py:169-211 for n candidates d_cand [n][3] = (x, y, layer) of
 *                        octave `octave`, whose num_intervals + 2 DoG levels (h x w f32 device
 *                        planes) are h_dog[] (a host array of device pointers).  d_out [n]: the
 *                        keypoint (base-image coordinates, angle -1); d_layer [n]: its final
 *                        layer, -1 when the fit rejects it (the reference's None), -2 when the
 *                        candidate's 3x3x3 cube leaves the levels.
 * pano_sift_orient       compute_keypoints_with_orientations(keypoint, octave, gauss_img)
 *                        sift_impl.py:246-293 for n keypoints d_kps [n] of octave `octave` on its
 *                        Gaussian level d_gauss (h x w f32): d_out [n][PANO_ORI_MAX_PEAKS], the
 *                        oriented copies of keypoint i in peak order, d_counts [n] of them. */
#define PANO_ORI_MAX_PEAKS 18
int pano_sift_localize(pano_ctx *ctx, const pano_sift_params *params, const float *const *h_dog, int n_dog,
                       int h, int w, int octave, const int32_t *d_cand, int n, pano_kp *d_out,
                       int32_t *d_layer);
int pano_sift_orient(pano_ctx *ctx, const pano_sift_params *params, const float *d_gauss, int h, int w,
                     int octave, const pano_kp *d_kps, int n, pano_kp *d_out, int32_t *d_counts);

/* cv2.cvtColor(image, COLOR_BGR2GRAY) on a float32 BGR image (sift_impl.py:27-28, the drop-in's
 * float path): d_bgr [n][h][w][3] f32 -> d_gray [n][h][w] f32, OpenCV's scalar RGB2Gray<float>
 * order b * 0.114f + g * 0.587f + r * 0.299f (parity with its SIMD body unpinned). */
int pano_gray_bgr_f32(pano_ctx *ctx, const float *d_bgr, int n, int h, int w, float *d_gray);

int pano_sift_base(pano_ctx *ctx, const float *d_gray, int n, int h, int w,
                   const pano_sift_params *params, float *d_base);
int pano_sift_pyramid_base(pano_ctx *ctx, const float *d_base, int n, int H0, int W0, int n_octaves,
                           const pano_sift_params *params);
int pano_sift_pyramid_kernels(pano_ctx *ctx, const float *d_base, int n, int H0, int W0, int n_octaves,
                              const double *h_kernels, int n_kernels);
int pano_sift_reserve_levels(pano_ctx *ctx, int n, int H0, int W0, int n_octaves, int n_levels);
int pano_sift_set_level(pano_ctx *ctx, int frame, int octave, int level, int dog, const float *d_in);
int pano_sift_dog(pano_ctx *ctx);
int pano_sift_extrema(pano_ctx *ctx, const pano_sift_params *params, pano_kp *d_raw, int cap,
                      int32_t *d_counts);
int pano_sift_describe(pano_ctx *ctx, const pano_sift_params *params, const pano_kp *d_kps,
                       const int32_t *d_counts, int cap, float *d_desc);

/* ---------------------------------------------------------------- H1..H3
 * compute_keypoints_and_descriptors_harris(img_bgr, max_points)  image_stitching_harris.py:187-214
 * d_xy [n][max_points][2] int32 (x, y), d_desc [n][max_points][128] f32, d_counts [n]. */
int pano_harris(pano_ctx *ctx, const uint8_t *d_bgr, int n, int h, int w, int max_points,
                int32_t *d_xy, float *d_desc, int32_t *d_counts);

/* ---------------------------------------------------------------- M1 / H4
 * Brute-force L2 nearest neighbour of every row of A among rows of B
 * (image_stitching_sift.py:63-79, image_stitching_harris.py:219-240).
 * exact_int == 1: descriptors are integers in [0,255] (SIFT): fp32 MFMA distance GEMM
 *   (v_mfma_f32_32x32x2_f32, LDS-staged), distances exact.
 * exact_int == 2 (the Stitcher default): same inputs, packed once to bf16 rows + norms and
 *   multiplied with v_mfma_f32_32x32x16_bf16 from register-loaded fragments: bit-identical
 *   results (integers <= 255 are exact in bf16; every product and partial sum is an integer
 *   < 2^24, exact in the f32 accumulator).
 * exact_int == 0 (Harris): direct fp32 differences summed in the OpenBLAS sdot order numpy
 *   uses.
 * Batched over pairs: pair p matches frame h_pairs[2p] (A) against h_pairs[2p+1] (B) of a
 * [frames][cap][128] descriptor array with d_counts[frames].
 * Outputs per pair p, row i (< cap): d_best[p][i] (first minimum, -1 if B empty),
 * d_d1[p][i] best distance, d_d2[p][i] second-best distance (Lowe ratio input; with
 * exact_int == 2 d_d2 may be NULL, and the second-best is then not computed). */
int pano_match(pano_ctx *ctx, const float *d_desc, const int32_t *d_counts, int cap,
               const int32_t *h_pairs, int n_pairs, int exact_int,
               int32_t *d_best, float *d_d1, float *d_d2);

/* pano_match on byte descriptors (pano_sift_u8 output): d_desc_u8 [frames][cap][128] and
 * d_norms [frames][cap] their exact squared norms.  bf16 MFMA distance GEMM with each 128-row
 * candidate tile converted once into LDS for 256 query rows; results bit-identical to
 * exact_int 1 / 2 (integers <= 255 exact in bf16, exact f32 accumulation).  d_d2 may be NULL
 * (second-best not computed). */
int pano_match_u8(pano_ctx *ctx, const uint8_t *d_desc_u8, const int32_t *d_norms,
                  const int32_t *d_counts, int cap, const int32_t *h_pairs, int n_pairs,
                  int32_t *d_best, float *d_d1, float *d_d2);

/* The exact squared norms pano_match_u8 reads, for byte descriptors that did not come from
 * pano_sift_u8 (which writes them itself): d_norms[r] = sum of d_desc_u8[r][0..127]^2, rows
 * 16-byte aligned (the `np.dot(d, d)` of image_stitching_sift.py:71 on integer rows). */
int pano_desc_norms_u8(pano_ctx *ctx, const uint8_t *d_desc_u8, int rows, int32_t *d_norms);

/* ---------------------------------------------------------------- R1
 * Match filter (distance < desc_thresh, optional Lowe ratio d1 < ratio*d2 when ratio > 0;
 * d_d2 is read only then and may be NULL otherwise)
 * + ransac(matches, dist_sq_thresh)  image_stitching_sift.py:74-111.
 * Keypoint coordinates come from d_xy_f32 [frames][cap][2] (SIFT: pano_kp x,y are read
 * when d_kps != NULL; Harris: pass d_xy_i32).  Writes d_recs[n_pairs]. */
int pano_pair_shifts(pano_ctx *ctx, const pano_kp *d_kps, const int32_t *d_xy_i32,
                     const int32_t *d_counts, int cap, const int32_t *h_pairs, int n_pairs,
                     const int32_t *d_best, const float *d_d1, const float *d_d2,
                     double desc_thresh, double ratio, double ransac_thr,
                     pano_pair_rec *d_recs);

/* ---------------------------------------------------------------- f3
 * The visualiser's matching + homography (sift_visualizeUI.py:247-266): good matches by the
 * Lowe ratio test on the exact kNN-2 of pano_match / pano_match_u8 (d1 < ratio^2 d2 on the
 * squared distances; FLANN's approximate neighbours are not reproduced) and, optionally,
 * d1 < desc_thresh (<= 0: no threshold); then, for a pair with more than min_good good
 * matches (the visualiser's MIN_MATCH_COUNT = 10), a deterministic homography RANSAC:
 * n_hyp 4-point hypotheses drawn by a counter-based hash of (seed, pair, hypothesis),
 * degenerate samples rejected as cv2's checkSubset does, each scored by the matches whose
 * squared reprojection error is <= reproj_thr^2 (cv2.findHomography(..., cv2.RANSAC, 5.0)),
 * the first best refitted by Hartley-normalised least squares over its inliers.
 * d_recs[n_pairs]; d_mask [n_pairs][cap] (optional) flags the refit's inliers among the pair's
 * good matches, in match order. */
typedef struct pano_homography_rec {
    double H[9];               /* row-major, H[8] = 1 (zeros when status != PANO_OK)        */
    int32_t n_matches;         /* good matches                                              */
    int32_t inliers;           /* inliers of the refitted H                                 */
    int32_t hyp_inliers;       /* inliers of the best hypothesis                            */
    int32_t status;            /* PANO_OK, PANO_E_NOMATCH (too few matches / no model) or
                                  PANO_E_OVERFLOW (a frame's count exceeded cap)             */
} pano_homography_rec;

int pano_pair_homography(pano_ctx *ctx, const pano_kp *d_kps, const int32_t *d_counts, int cap,
                         const int32_t *h_pairs, int n_pairs, const int32_t *d_best,
                         const float *d_d1, const float *d_d2, double desc_thresh, double ratio,
                         double reproj_thr, int n_hyp, uint64_t seed, int min_good,
                         pano_homography_rec *d_recs, uint8_t *d_mask);

/* ransac(matches) on an explicit move list (drop-in for the Python function):
 * d_moves [k][2] double (dx, dy).  d_out[0] = best index (-1 if k == 0), d_out[1] = votes. */
int pano_ransac_translate(pano_ctx *ctx, const double *d_moves, int k, double thr,
                          int32_t *d_out);

/* ---------------------------------------------------------------- B1
 * Host planning of the whole mosaic loop from drift-corrected shifts and best pairs:
 * h_shifts [n-1][2], h_pairs [n-1][4] (xA, yA, xB, yB); every frame h x w.  Fills
 * h_steps[n-1] (step i blends frame i+1), frame 0's placement in h_first and the final
 * canvas size.  Returns PANO_E_UNSUPPORTED if a step would crop (never for pad_image). */
int pano_plan_composite(const double *h_shifts, const double *h_pairs, int n, int h, int w,
                        pano_step *h_steps, int32_t *h_first_xy, int32_t *h_canvas_hw);

/* Run the whole mosaic loop on device: d_frames [n][h][w][3] cylindrical frames,
 * d_colnz [n][w] their column flags, d_canvas [H][W][3] (zeroed here), d_colflags [W]
 * scratch.  Bit-identical to the reference's sequential blend_two_images fold. */
int pano_composite(pano_ctx *ctx, const uint8_t *d_frames, const uint8_t *d_colnz, int n,
                   int h, int w, const pano_step *h_steps, const int32_t *h_first_xy,
                   uint8_t *d_canvas, int H, int W);

/* pano_composite + rectangle_crop's bounding box in the same pass: d_bbox[4] = ymin ymax
 * xmin xmax of gray > black_threshold over the canvas (-1s if none).  When no canvas
 * column is covered by three frames (checked on the host) the fold runs as one parallel
 * pass over the canvas (3 launches); otherwise it is the sequential per-step fold.
 * pano_composite_sequential forces the per-step fold (reference-shaped; used by tests). */
int pano_composite_bbox(pano_ctx *ctx, const uint8_t *d_frames, const uint8_t *d_colnz, int n,
                        int h, int w, const pano_step *h_steps, const int32_t *h_first_xy,
                        uint8_t *d_canvas, int H, int W, int black_threshold, int32_t *d_bbox);
int pano_composite_sequential(pano_ctx *ctx, const uint8_t *d_frames, const uint8_t *d_colnz,
                              int n, int h, int w, const pano_step *h_steps,
                              const int32_t *h_first_xy, uint8_t *d_canvas, int H, int W);

/* Device-planned mosaic loop (the batched Stitcher's single-launch-chain form of
 * run_panorama :336-381): pano_plan_device reads the n-1 pair records on the device, applies
 * run_panorama's record -> shift conversion (int() for Harris: int_shifts = 1), the drift
 * correction and pano_plan_composite's geometry, and writes a plan of pano_plan_device_bytes()
 * bytes to d_plan; pano_composite_planned then composites into d_canvas, a buffer of
 * Hcap x Wcap x 3 bytes laid out as [H][W][3] with the planned H, W.  The plan starts with
 * int32 {status, H, W, n, first_x, first_y}: status PANO_OK, PANO_E_NOMATCH (a pair record
 * is not PANO_OK: no match -- the reference fails there -- or a keypoint-capacity overflow,
 * which the record's own status tells apart), or PANO_E_OVERFLOW (canvas above the capacity or a
 * column covered by three frames: use pano_plan_composite + pano_composite_bbox instead).
 * d_bbox: PANO_BBOX_SLOTS (64) partial boxes {ymin, ymax, xmin, xmax} (int32[256]); the
 * crop box is their elementwise min / max, with ymax < 0 when no pixel passed the threshold
 * (workgroups spread their atomics over the slots instead of serialising on one box).
 * Nothing is read back by either call (graph-capturable).  2 <= n <= 256. */
#define PANO_BBOX_SLOTS 64   /* crop-box partials of pano_composite_planned (one box
                                serialised every workgroup's atomics at L2: 48 us/stitch) */
size_t pano_plan_device_bytes(void);
int pano_plan_device(pano_ctx *ctx, const pano_pair_rec *d_recs, int n, int h, int w,
                     int int_shifts, int Hcap, int Wcap, void *d_plan);
int pano_composite_planned(pano_ctx *ctx, const uint8_t *d_frames, const uint8_t *d_colnz, int n,
                           int h, int w, const void *d_plan, uint8_t *d_canvas, int Hcap,
                           int Wcap, int black_threshold, int32_t *d_bbox);
/* pano_plan_device followed by pano_composite_planned in two launches instead of three (the
 * composite's column tables are built by the plan launch, one workgroup per frame): the same
 * plan, canvas and crop-box partials, byte for byte. */
int pano_plan_composite_device(pano_ctx *ctx, const pano_pair_rec *d_recs, const uint8_t *d_frames,
                               const uint8_t *d_colnz, int n, int h, int w, int int_shifts,
                               void *d_plan, uint8_t *d_canvas, int Hcap, int Wcap,
                               int black_threshold, int32_t *d_bbox);

/* One rank's band of a sharded stitch from the GLOBAL plan of pano_plan_device
 * (built from every rank's gathered records): the rank holds frames f0 .. f0 + n_local - 1
 * (its pairs plus the boundary frame f0) and owns the canvas columns whose last covering
 * frame is one of its frames after f0 (plus frame 0's on the first band).  Writes a local
 * plan (pano_plan_device_bytes) whose canvas is the owned column range -- pass it with the
 * rank's frames to pano_composite_planned, canvas capacity Hcap x Wcap -- and d_band[4] =
 * {status, own_lo, own_hi, global W}: PANO_OK, the global plan's status, PANO_E_UNSUPPORTED
 * (owned columns not contiguous) or PANO_E_OVERFLOW (band wider than Wcap).  Device-only,
 * graph-capturable. */
int pano_band_plan(pano_ctx *ctx, const void *d_plan, int f0, int n_local, int w, int Wcap,
                   void *d_local_plan, int32_t *d_band);
/* The rank's row of the N > 1 layout exchange (distributed.py), on the device: from the global
 * plan, pano_band_plan's d_band and the band's PANO_BBOX_SLOTS crop-box partials, d_row[8]
 * int64 = {ymin, ymax, xmin, xmax} in global columns ({2^30, -1, 2^30, -1} when no pixel
 * passed or the band was refused), own_lo, own_hi, fallback (1: the global or the band plan
 * refused), the global plan's status.  Device-only, graph-capturable. */
int pano_band_layout_row(pano_ctx *ctx, const void *d_plan, const int32_t *d_band,
                         const int32_t *d_bbox, int64_t *d_row);

/* blend_two_images(shift_vec, ref_match, imgA, imgB) for arbitrary inputs
 * image_stitching_sift.py:156-202.  Geometry comes from pano_blend_geometry. */
int pano_blend_geometry(double dx, double dy, const double *h_ref4, int hA, int wA, int hB,
                        int wB, int32_t *h_geom /* [8]: ayA axA ayB axB H W swapped pad */,
                        double *h_overlap);
int pano_blend_two(pano_ctx *ctx, const uint8_t *d_A, int hA, int wA, const uint8_t *d_B,
                   int hB, int wB, const int32_t *h_geom, double overlap_range,
                   uint8_t *d_out);

/* rectangle_crop bbox (image_stitching_sift.py:208-247): d_bbox[4] = ymin ymax xmin xmax of
 * gray > black_threshold (-1s if none). */
int pano_gray_bbox(pano_ctx *ctx, const uint8_t *d_img, int H, int W, int black_threshold,
                   int32_t *d_bbox);

/* ---------------------------------------------------------------- JPEG
 * The reference reads every frame with cv2.imread (image_stitching_sift.py:282,
 * image_stitching_harris.py:394): libjpeg-turbo's default decode.  pano_jpeg_decode runs it on
 * the GPU for a batch of baseline (SOF0/SOF1, Huffman, 8-bit) files of one size, 1 or 3
 * components, 4:4:4 / 4:2:2 / 4:2:0, no restart intervals: islow IDCT, fancy upsampling,
 * fixed-point YCbCr -> RGB, bit-identical to libjpeg-turbo (and PIL / cv2.imread).
 *   h_bufs[i], lens[i]: the files in host memory (read on the host for headers only; the
 *                       entropy-coded bytes are uploaded in one copy);
 *   d_bgr:              device u8 [n][h][w][3] BGR (cv2.imread's channel order);
 *   d_status:           optional device int32 [n]: per-frame PANO_OK, PANO_E_ARG (corrupt or
 *                       truncated scan) or PANO_E_UNSUPPORTED (a marker inside the scan).
 * Header problems (not a JPEG, progressive, arithmetic coding, other sampling, size differs
 * from h x w) fail the call itself.  pano_jpeg_info is host-only. */
int pano_jpeg_info(const uint8_t *h_buf, size_t len, int *h, int *w, int *ncomp);
int pano_jpeg_decode(pano_ctx *ctx, int n, const uint8_t *const *h_bufs, const size_t *lens,
                     uint8_t *d_bgr, int h, int w, int32_t *d_status);
/* Synchronisation statistics of the last pano_jpeg_decode (synchronises the stream): per frame
 * h_stats[4 f + 0] = subsequences the scan was cut into, [4 f + 1] = extra candidates decoded
 * from a predecessor's exit, [4 f + 2] = subsequences decoded serially from their true start
 * (none of their candidates reached), [4 f + 3] = 0.  Diagnostics: the output never depends
 * on them. */
int pano_jpeg_stats(pano_ctx *ctx, int32_t *h_stats, int n);
/* cv2.imwrite(path, panorama) (image_stitching_sift.py:386; OpenCV's default quality 95): the
 * u8 BGR image at d_bgr (h rows of w pixels, row pitch `pitch` bytes -- a crop view of a
 * canvas works as is) encoded on the GPU as a baseline JFIF file, YCbCr 4:2:0, byte-identical
 * to libjpeg-turbo's default encoder (PIL save(quality=q)).  Synchronous: the file is written to
 * h_out (capacity cap) and its length to *out_len; PANO_E_OVERFLOW (with *out_len set) when
 * cap is too small. */
int pano_jpeg_encode(pano_ctx *ctx, const uint8_t *d_bgr, int h, int w, int64_t pitch, int quality,
                     uint8_t *h_out, size_t cap, size_t *out_len);

/* ---------------------------------------------------------------- live kernel timing
 * pano_prof_enable(ctx, k) records a hipEvent pair on the context's stream around every
 * launch of kernel class k (PANO_K_*; PANO_K_ALL = every class; -1 = off).
 * pano_prof_read synchronises the stream and returns launches and elapsed milliseconds of
 * class k since the last read (PANO_K_ALL: all recorded launches), then resets. */
#define PANO_K_CYL_SCATTER 0
#define PANO_K_CYL_GATHER 1
#define PANO_K_BLUR 2
#define PANO_K_EXTREMA 3
#define PANO_K_ORIENT 4
#define PANO_K_SORT 5
#define PANO_K_DESC 6
#define PANO_K_NORMS 7
#define PANO_K_DIST_MFMA 8
#define PANO_K_DIST_DIRECT 9
#define PANO_K_REDUCE 10
#define PANO_K_PAIR_SHIFTS 11
#define PANO_K_COMPOSITE 12
#define PANO_K_BBOX 13
#define PANO_K_H_GRAY 14
#define PANO_K_H_BLUR 15
#define PANO_K_H_RESP 16
#define PANO_K_H_NMS 17
#define PANO_K_H_SELECT 18
#define PANO_K_H_DESC 19
#define PANO_K_JPEG 20
#define PANO_K_ALL 21
int pano_prof_enable(pano_ctx *ctx, int kernel_class);
int pano_prof_read(pano_ctx *ctx, int kernel_class, int *launches, double *total_ms,
                   double *min_ms, double *max_ms);

/* ---------------------------------------------------------------- hipGraph capture
 * Launch-bound sequences (e.g. a whole stitch) can be captured once and replayed:
 * pano_graph_begin(ctx) starts capturing ctx's stream (call the sequence once eagerly first
 * so every scratch buffer has its final size: growth inside a capture fails with
 * PANO_E_UNSUPPORTED); pano_graph_end instantiates it.  pano_graph_launch replays it on
 * ctx's stream with the same device pointers and kernel arguments as captured.  Profiler
 * event pairs recorded during capture (pano_prof_enable) belong to the graph and are
 * re-recorded by every replay: pano_graph_prof reads the last replay (stream synchronised
 * by the caller). */
typedef struct pano_graph pano_graph;
int pano_graph_begin(pano_ctx *ctx);
int pano_graph_end(pano_ctx *ctx, pano_graph **out);
int pano_graph_launch(pano_ctx *ctx, pano_graph *g);
/* Replay g on `hip_stream` (NULL: the context's stream) and wait for it: the batched
 * stitch's whole per-call GPU work as one call (its last node copies the result header to
 * pinned host memory, pano_copy_async). */
int pano_graph_launch_sync(pano_ctx *ctx, pano_graph *g, void *hip_stream);
/* Replay g on `hip_stream` (NULL: the context's stream) without waiting: a caller keeping two
 * stitches in flight (Stitcher.run_sequence) waits on its own event per replay. */
int pano_graph_launch_stream(pano_ctx *ctx, pano_graph *g, void *hip_stream);
/* Copy on the context's stream (device or pinned host pointers; capturable): up to 1 MiB as
 * a copy kernel (the GPU writes pinned host memory directly), larger as hipMemcpyAsync. */
int pano_copy_async(pano_ctx *ctx, void *dst, const void *src, size_t bytes);
int pano_graph_prof(pano_graph *g, int kernel_class, int *launches, double *total_ms);
int pano_graph_destroy(pano_graph *g);

#ifdef __cplusplus
}
#endif
#endif /* PANO_H */
