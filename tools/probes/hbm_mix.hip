// Probe: achievable HBM rate for the blur level's traffic mix (read 1 plane, write 2 planes,
// f32, 14.2 M px = 18 frames x 1024 x 768), float4 per lane, grid-stride.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(256) mix(const float4 *__restrict__ a, float4 *__restrict__ b,
                                           float4 *__restrict__ c, size_t n4, int nw) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        float4 v = a[i];
        if (nw > 0) b[i] = v;
        if (nw > 1) c[i] = make_float4(v.x - 1, v.y - 1, v.z - 1, v.w - 1);
        if (nw == 0 && v.x == 12345.f) b[0] = v;
    }
}

int main() {
    const size_t n = 18ull * 1024 * 768, n4 = n / 4;
    float4 *a, *b, *c;
    (void)hipMalloc(&a, n * 4);
    (void)hipMalloc(&b, n * 4);
    (void)hipMalloc(&c, n * 4);
    (void)hipMemset(a, 0, n * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int nw = 0; nw <= 2; ++nw) {
        for (int blocks : {1024, 2048, 8192}) {
            mix<<<blocks, 256>>>(a, b, c, n4, nw);
            (void)hipEventRecord(e0);
            for (int r = 0; r < 10; ++r) mix<<<blocks, 256>>>(a, b, c, n4, nw);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double bytes = (double)n * 4 * (1 + nw);
            printf("read 1 + write %d planes, %5d blocks: %6.1f us, %5.2f TB/s\n", nw, blocks, ms * 100,
                   bytes / (ms * 1e-4) / 1e12);
        }
    }
    return 0;
}
