// Probe: sustained v_fma_f64 / v_fma_f32 issue rate on this GPU (vector ALU roofline of the
// bit-exact blur), as a function of waves per SIMD and independent chains per thread.
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename T, int CH>
__global__ void __launch_bounds__(256) fma_chain(T *out, T a, T b, int iters) {
    T acc[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) acc[j] = (T)(threadIdx.x + j);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < CH; ++j) acc[j] = fma(acc[j], a, b);
    }
    T s = 0;
#pragma unroll
    for (int j = 0; j < CH; ++j) s += acc[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <typename T, int CH>
void run(const char *name, int wps) {
    const int blocks = 256 * wps, iters = 65536 / CH;
    T *out;
    (void)hipMalloc(&out, sizeof(T) * blocks * 256);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    fma_chain<T, CH><<<blocks, 256>>>(out, (T)0.999, (T)1e-3, iters);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) fma_chain<T, CH><<<blocks, 256>>>(out, (T)0.999, (T)1e-3, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double fmas = 3.0 * blocks * 256.0 * iters * CH;
    printf("%s chains=%2d waves/SIMD=%d: %6.2f T FMA/s\n", name, CH, wps, fmas / (ms * 1e-3) / 1e12);
    (void)hipFree(out);
}

int main() {
    for (int w : {1, 2, 4, 8}) {
        run<double, 4>("f64", w);
        run<double, 8>("f64", w);
        run<double, 16>("f64", w);
    }
    run<float, 16>("f32", 8);
    return 0;
}
