// Exhaustive device check of the descriptor's fixed-point rounding: for every
// f32 x in [0, 2^31) compare v_cvt_rpi_i32_f32(x) (the PANO_DESC_RPI form, x pre-scaled by
// 2^22) with u32(fma(v, 2^22, 0.5)) for v = x / 2^22 (the unscaled form it replaced).  Counts
// mismatches per binade and prints the first few.
//   hipcc --offload-arch=gfx950 -O2 rpi_check.hip -o rpi_check && ./rpi_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cstdint>

__global__ void check(uint32_t lo, uint32_t n, unsigned long long *bad, uint32_t *first) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const uint32_t u = lo + i;
    const float x = __uint_as_float(u);
    int r;
    asm volatile("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    const float v = x * 2.384185791015625e-07f;                // x / 2^22, exact (power of two)
    const uint32_t f = (uint32_t)fmaf(v, 4194304.0f, 0.5f);
    if ((uint32_t)r != f) {
        const int e = (int)((u >> 23) & 255) - 127;             // binade of x
        atomicAdd(&bad[e < 0 ? 0 : e], 1ull);
        const uint32_t k = atomicAdd(&first[0], 1u);
        if (k < 8) first[1 + k] = u;
    }
}

int main() {
    float a = 0.0f, b = 2147483648.0f;
    uint32_t lo, hi;
    memcpy(&lo, &a, 4);
    memcpy(&hi, &b, 4);
    unsigned long long *bad;
    uint32_t *first;
    hipMalloc(&bad, 64 * 8);
    hipMalloc(&first, 9 * 4);
    hipMemset(bad, 0, 64 * 8);
    hipMemset(first, 0, 9 * 4);
    const uint32_t chunk = 1u << 28;
    for (uint64_t s = lo; s < hi; s += chunk) {
        const uint32_t n = (uint32_t)((hi - s) < chunk ? (hi - s) : chunk);
        check<<<(n + 255) / 256, 256>>>((uint32_t)s, n, bad, first);
    }
    unsigned long long hb[64];
    uint32_t hf[9];
    hipMemcpy(hb, bad, sizeof hb, hipMemcpyDeviceToHost);
    hipMemcpy(hf, first, sizeof hf, hipMemcpyDeviceToHost);
    unsigned long long tot = 0;
    for (int e = 0; e < 64; ++e)
        if (hb[e]) { printf("binade 2^%d: %llu mismatches\n", e, hb[e]); tot += hb[e]; }
    printf("total mismatches over [0, 2^31): %llu\n", tot);
    for (uint32_t k = 0; k < hf[0] && k < 8; ++k) {
        float x;
        memcpy(&x, &hf[1 + k], 4);
        int r = (int)floor((double)x + 0.5);
        printf("  x = %.1f  floor(x + 0.5) = %d  fma form = %u\n", x, r, (uint32_t)fmaf(x / 4194304.0f, 4194304.0f, 0.5f));
    }
    return 0;
}
