// Probe: v_fma_f64 throughput by operand kind (SGPR vs VGPR sources), 16 chains, 8 waves/SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

// MODE 0: acc = fma(acc, s, s)   1: acc = fma(s_tap, v_x[j], acc)   2: acc = fma(v_tap, v_x[j], acc)
template <int MODE>
__global__ void __launch_bounds__(256) k(double *out, double a, double b, int iters) {
    double acc[16], x[16];
    const double vt = a + threadIdx.x * 1e-9;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        acc[j] = (double)(threadIdx.x + j);
        x[j] = b + j * 1e-7 + threadIdx.x * 1e-12;
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (MODE == 0) acc[j] = fma(acc[j], a, b);
            else if (MODE == 1) acc[j] = fma(a, x[j], acc[j]);
            else acc[j] = fma(vt, x[j], acc[j]);
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) asm volatile("" : "+v"(x[j]));
    }
    double s = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += acc[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE>
void run(const char *name) {
    const int blocks = 256 * 8, iters = 4096;
    double *out;
    (void)hipMalloc(&out, sizeof(double) * blocks * 256);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    k<MODE><<<blocks, 256>>>(out, 0.999, 1e-3, iters);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) k<MODE><<<blocks, 256>>>(out, 0.999, 1e-3, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double fmas = 3.0 * blocks * 256.0 * iters * 16;
    printf("%s: %6.2f T FMA/s\n", name, fmas / (ms * 1e-3) / 1e12);
    (void)hipFree(out);
}

int main() {
    run<0>("fma(v_acc, s, s)        ");
    run<1>("fma(s_tap, v_x, v_acc)  ");
    run<2>("fma(v_tap, v_x, v_acc)  ");
    return 0;
}
