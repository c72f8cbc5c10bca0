/* OpenCV float32 separable-filter arithmetic, restated in C -- TEST INFRASTRUCTURE.
 *
 * The reference blurs float32 images with cv2.GaussianBlur(img, (0,0), sigma)
 * (/root/reference/sift_impl.py:56,91).  OpenCV routes a float32 Gaussian through
 * sepFilter2D's FilterEngine: a row pass RowFilter<float,float,RowVec_32f> (kernel
 * longer than 5 taps, so not the "small symmetric" row filter) into a float32 row
 * buffer, then a column pass SymmColumnFilter<Cast<float,float>,SymmColumnVec_32f>
 * (the Gaussian kernel is symmetric).  Per output:
 *
 *   row:    s = x[0]*k[0];  s = s + x[i]*k[i]   (i = 1..n-1, in f32; fused with FMA3)
 *   column: s = S[0]*k[0];  s = s + (S[+i] + S[-i])*k[i]   (i = 1..r; the pair sum is
 *           rounded to f32 first; fused with FMA3)
 *
 * numpy cannot express a fused f32 multiply-add, so the variants live here (fmaf from
 * libm is exact).  Modes (oracle/cv2_compat.py selects them, tools/blur_variants.py
 * sweeps them against the author's published panoramas):
 *
 *   row  0: f64 accumulate, tap order, one rounding   (the round-1/2 oracle definition)
 *        1: f32 sequential, fused multiply-add
 *        2: f32 sequential, separate multiply and add
 *   col  0: f64 accumulate, tap order, one rounding
 *        1: f32 symmetric form, fused
 *        2: f32 symmetric form, separate multiply and add
 *        3: f32 sequential over all n taps, fused
 *
 * Borders are BORDER_REFLECT_101 (periodic beyond one reflection), as in cv2_compat.
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, so the compiler adds no fusion).
 */
#include <math.h>
#include <stdlib.h>

static inline int refl101(int i, int n)
{
    if (n == 1) return 0;
    int p = 2 * n - 2;
    i %= p;
    if (i < 0) i += p;
    return i >= n ? p - i : i;
}

static void row_pass(const float* src, float* dst, int h, int w, const float* k, int n, int mode,
                     int* idx)
{
    int r = (n - 1) / 2;
    for (int y = 0; y < h; ++y) {
        const float* s = src + (size_t)y * w;
        float* d = dst + (size_t)y * w;
        for (int x = 0; x < w; ++x) {
            for (int i = 0; i < n; ++i) idx[i] = refl101(x + i - r, w);
            if (mode == 0) {
                double acc = 0.0;
                for (int i = 0; i < n; ++i) acc += (double)k[i] * (double)s[idx[i]];
                d[x] = (float)acc;
            } else if (mode == 1) {
                float acc = s[idx[0]] * k[0];
                for (int i = 1; i < n; ++i) acc = fmaf(s[idx[i]], k[i], acc);
                d[x] = acc;
            } else {
                float acc = s[idx[0]] * k[0];
                for (int i = 1; i < n; ++i) {
                    float p = s[idx[i]] * k[i];
                    acc = acc + p;
                }
                d[x] = acc;
            }
        }
    }
}

static void col_pass(const float* src, float* dst, int h, int w, const float* k, int n, int mode,
                     int* idx)
{
    int r = (n - 1) / 2;
    for (int y = 0; y < h; ++y) {
        for (int i = 0; i < n; ++i) idx[i] = refl101(y + i - r, h);
        float* d = dst + (size_t)y * w;
        for (int x = 0; x < w; ++x) {
            if (mode == 0) {
                double acc = 0.0;
                for (int i = 0; i < n; ++i) acc += (double)k[i] * (double)src[(size_t)idx[i] * w + x];
                d[x] = (float)acc;
            } else if (mode == 3) {
                float acc = src[(size_t)idx[0] * w + x] * k[0];
                for (int i = 1; i < n; ++i) acc = fmaf(src[(size_t)idx[i] * w + x], k[i], acc);
                d[x] = acc;
            } else {
                float acc = src[(size_t)idx[r] * w + x] * k[r];
                for (int i = 1; i <= r; ++i) {
                    float pair = src[(size_t)idx[r + i] * w + x] + src[(size_t)idx[r - i] * w + x];
                    if (mode == 1) {
                        acc = fmaf(pair, k[r + i], acc);
                    } else {
                        float p = pair * k[r + i];
                        acc = acc + p;
                    }
                }
                d[x] = acc;
            }
        }
    }
}

/* dst = column_pass(row_pass(src)); tmp is h*w floats of scratch. Returns 0, or -1 on a
 * bad argument. kx is the n-tap f32 kernel (symmetric for the column modes 1-2). */
int cvb_gaussian_f32(const float* src, float* dst, float* tmp, int h, int w, const float* kx, int n,
                     int row_mode, int col_mode)
{
    if (h <= 0 || w <= 0 || n <= 0 || (n & 1) == 0) return -1;
    if (row_mode < 0 || row_mode > 2 || col_mode < 0 || col_mode > 3) return -1;
    int* idx = (int*)malloc(sizeof(int) * (size_t)n);
    if (!idx) return -1;
    row_pass(src, tmp, h, w, kx, n, row_mode, idx);
    col_pass(tmp, dst, h, w, kx, n, col_mode, idx);
    free(idx);
    return 0;
}
