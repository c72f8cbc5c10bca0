// Where global_load_lds of 12 / 16 bytes puts each lane's data in LDS (gfx950): each lane loads
// from src + 64 * lane (distinct values), the LDS buffer is dumped after vmcnt(0).
//   hipcc --offload-arch=gfx950 -O2 glds_layout.hip -o glds_layout && ./glds_layout
#include <hip/hip_runtime.h>
#include <cstdio>

#define PROBE(NAME, SIZE)                                                                        \
__global__ void NAME(const float *src, float *out) {                                             \
    __shared__ float lds[64 * 8];                                                                \
    for (int i = threadIdx.x; i < 64 * 8; i += 64) lds[i] = -1.0f;                               \
    __syncthreads();                                                                             \
    const float *q = src + 16 * threadIdx.x;                                                     \
    __builtin_amdgcn_global_load_lds((const void *)q, (__attribute__((address_space(3))) void *)lds, SIZE, 0, 0); \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                             \
    __syncthreads();                                                                             \
    for (int i = threadIdx.x; i < 64 * 8; i += 64) out[i] = lds[i];                              \
}
PROBE(probe12, 12)
PROBE(probe16, 16)
// misaligned source: lane reads from src + 16 lane + 1 (4-byte aligned only)
__global__ void probe16u(const float *src, float *out) {
    __shared__ float lds[64 * 8];
    for (int i = threadIdx.x; i < 64 * 8; i += 64) lds[i] = -1.0f;
    __syncthreads();
    const float *q = src + 16 * threadIdx.x + 1;
    __builtin_amdgcn_global_load_lds((const void *)q, (__attribute__((address_space(3))) void *)lds, 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * 8; i += 64) out[i] = lds[i];
}
__global__ void unused_(const float *src, float *out) {
    __shared__ float lds[64 * 8];
    for (int i = threadIdx.x; i < 64 * 8; i += 64) lds[i] = -1.0f;
    __syncthreads();
    const float *q = src + 16 * threadIdx.x;
    (void)q; (void)lds; (void)out;
}

// 4 waves, the LDS target behind another shared array (nonzero base), per-wave regions
__global__ void probe_multi(const float *src, float *out) {
    __shared__ float pad[4640];
    __shared__ __attribute__((aligned(16))) float ring[4][2][256];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 4640; i += 256) pad[i] = 7.0f;
    for (int i = threadIdx.x; i < 2048; i += 256) (&ring[0][0][0])[i] = -1.0f;
    __syncthreads();
    float *rw = &ring[wv][0][0];
    const float *q = src + 16 * lane + 1;
    __builtin_amdgcn_global_load_lds((const void *)q, (__attribute__((address_space(3))) void *)(rw + 256), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const float4 a = *(const float4 *)(rw + 256 + lane * 4);
    out[threadIdx.x * 4 + 0] = a.x + 1000.0f * wv;
    out[threadIdx.x * 4 + 1] = a.y;
    out[threadIdx.x * 4 + 2] = a.z;
    out[threadIdx.x * 4 + 3] = a.w + pad[threadIdx.x] - 7.0f;
}

int main() {
    float h[64 * 16], *s, *o;
    for (int i = 0; i < 64 * 16; ++i) h[i] = (float)(i / 16) * 100.0f + (float)(i % 16);   // lane*100 + word
    hipMalloc(&s, sizeof h);
    hipMalloc(&o, 64 * 8 * 4);
    hipMemcpy(s, h, sizeof h, hipMemcpyHostToDevice);
    float r[64 * 8];
    probe12<<<1, 64>>>(s, o);
    hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
    printf("size 12, first 24 LDS floats:");
    for (int i = 0; i < 24; ++i) printf(" %g", r[i]);
    printf("\n  floats 186..195:");
    for (int i = 186; i < 196; ++i) printf(" %g", r[i]);
    printf("\n");
    probe16<<<1, 64>>>(s, o);
    hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
    printf("size 16, first 24 LDS floats:");
    for (int i = 0; i < 24; ++i) printf(" %g", r[i]);
    printf("\n");
    probe16u<<<1, 64>>>(s, o);
    hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
    printf("size 16 from a 4-byte aligned source (+1 float), first 12:");
    for (int i = 0; i < 12; ++i) printf(" %g", r[i]);
    printf("\n");
    float *o2;
    hipMalloc(&o2, 1024 * 4);
    float r2[1024];
    probe_multi<<<1, 256>>>(s, o2);
    hipMemcpy(r2, o2, sizeof r2, hipMemcpyDeviceToHost);
    printf("multi-wave, nonzero base: lane 0,1 of wave 0: %g %g %g %g | %g %g %g %g; wave 3 lane 5: %g %g %g %g\n",
           r2[0], r2[1], r2[2], r2[3], r2[4], r2[5], r2[6], r2[7], r2[(192 + 5) * 4], r2[(192 + 5) * 4 + 1],
           r2[(192 + 5) * 4 + 2], r2[(192 + 5) * 4 + 3]);
    return 0;
}
