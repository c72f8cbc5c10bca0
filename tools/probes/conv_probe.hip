// Probe: throughput of the blur's inner loop (conv_seg: f32 LDS inputs widened to f64, NT
// taps in SGPRs, SEG accumulators, sequential fma order) with no barriers and no HBM traffic,
// as a function of waves per SIMD, SEG and LDS stride.  Prints T FMA/s (useful FMAs).
#include <hip/hip_runtime.h>
#include <cstdio>

struct Taps { double k[32]; };

template <int NT, int SEG>
__device__ __forceinline__ void conv_seg(const float *__restrict__ p, int stride, const double *__restrict__ k,
                                         double (&acc)[SEG]) {
#pragma unroll
    for (int j = 0; j < SEG; ++j) acc[j] = 0.0;
#pragma unroll
    for (int i = 0; i < SEG + NT - 1; ++i) {
        const double v = (double)p[i * stride];
#pragma unroll
        for (int j = 0; j < SEG; ++j) {
            const int t = i - j;
            if (t >= 0 && t < NT) acc[j] = fma(k[t], v, acc[j]);
        }
    }
}

template <int NT, int SEG, int STRIDE>
__global__ void __launch_bounds__(256) conv_loop(float *out, Taps taps, int iters) {
    __shared__ float lds[96 * 97];
    for (int i = threadIdx.x; i < 96 * 97; i += 256) lds[i] = (float)((i * 37) & 255);
    __syncthreads();
    const int t = threadIdx.x;
    // stride 1: thread = (row t % 64, segment t / 64), pitch 97; stride 97: thread = column
    const float *p = STRIDE == 1 ? lds + (t % 64) * 97 + (t / 64) * SEG : lds + (t / 64) * SEG * 97 + (t % 64);
    float s = 0.f;
    for (int it = 0; it < iters; ++it) {
        double acc[SEG];
        conv_seg<NT, SEG>(p + ((it * 7) & 15) * (STRIDE == 1 ? 97 : 1), STRIDE, taps.k, acc);
#pragma unroll
        for (int j = 0; j < SEG; ++j) s += (float)acc[j];
    }
    out[blockIdx.x * 256 + t] = s;
}

template <int NT, int SEG, int STRIDE>
void run(int wps) {
    const int blocks = 256 * wps, iters = 256;
    float *out;
    (void)hipMalloc(&out, sizeof(float) * blocks * 256);
    Taps tp;
    for (int i = 0; i < 32; ++i) tp.k[i] = 1.0 / (i + 3);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    conv_loop<NT, SEG, STRIDE><<<blocks, 256>>>(out, tp, iters);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) conv_loop<NT, SEG, STRIDE><<<blocks, 256>>>(out, tp, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double fmas = 3.0 * blocks * 256.0 * iters * SEG * NT;
    printf("NT=%2d SEG=%2d stride=%2d waves/SIMD=%d: %6.2f T FMA/s\n", NT, SEG, STRIDE, wps,
           fmas / (ms * 1e-3) / 1e12);
    (void)hipFree(out);
}

int main() {
    for (int w : {2, 4, 6, 8}) {
        run<27, 8, 1>(w);
        run<27, 16, 1>(w);
        run<27, 8, 97>(w);
        run<11, 8, 1>(w);
        run<11, 16, 1>(w);
        run<11, 8, 97>(w);
    }
    return 0;
}
