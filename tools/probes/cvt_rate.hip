// Probe: v_cvt_f64_f32 throughput next to v_fma_f64 (the blur's widening of staged f32 inputs).
#include <hip/hip_runtime.h>
#include <cstdio>

// per iteration: 16 fma + NC converts
template <int NC>
__global__ void __launch_bounds__(256) k(double *out, double a, int iters) {
    double acc[16];
    float x[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        acc[j] = (double)(threadIdx.x + j);
        x[j] = 1.0f + j * 1e-3f + threadIdx.x * 1e-6f;
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const double v = j < NC ? (double)x[j] : a;
            acc[j] = fma(a, v, acc[j]);
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) asm volatile("" : "+v"(x[j]));
    }
    double s = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += acc[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int NC>
void run() {
    const int blocks = 256 * 8, iters = 4096;
    double *out;
    (void)hipMalloc(&out, sizeof(double) * blocks * 256);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    k<NC><<<blocks, 256>>>(out, 0.999, iters);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) k<NC><<<blocks, 256>>>(out, 0.999, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double it = 3.0 * blocks * 256.0 * iters;
    printf("16 fma + %2d cvt per iter: %6.2f ns per lane-iter x1e3, %6.2f T FMA/s\n", NC,
           ms * 1e-3 / it * 1e12, it * 16 / (ms * 1e-3) / 1e12);
    (void)hipFree(out);
}

int main() {
    run<0>();
    run<4>();
    run<8>();
    run<16>();
    return 0;
}
