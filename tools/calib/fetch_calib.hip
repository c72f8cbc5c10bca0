// fetch_calib.hip -- calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE (KB) against known byte
// counts for the access widths libpano uses (MI355X_MICROARCH.md: "other access widths are
// uncalibrated").  Each kernel streams a 512 MiB buffer exactly once, coalesced:
//   read_b32   4 B / lane  (blur staging, extrema staging)
//   read_b96  12 B / lane  (gray_frames)
//   read_b128 16 B / lane
//   write_b32  4 B / lane
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/calib/fetch_calib tools/calib/fetch_calib.hip
// Run:   rocprofv3 --kernel-trace --pmc FETCH_SIZE -- ./tools/calib/fetch_calib   (then WRITE_SIZE)
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void read_b32(const float *__restrict__ p, size_t n, float *out) {
    float s = 0.f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += p[i];
    if (s == 1234.5f) out[0] = s;
}
__global__ void read_b96(const uint8_t *__restrict__ p, size_t n_px, float *out) {
    uint32_t s = 0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n_px / 4; i += (size_t)gridDim.x * 256) {
        const uint32_t *q = (const uint32_t *)(p + i * 12);
        s += q[0] ^ q[1] ^ q[2];
    }
    if (s == 12345u) out[0] = (float)s;
}
__global__ void read_b128(const float4 *__restrict__ p, size_t n, float *out) {
    float s = 0.f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const float4 v = p[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;
}
__global__ void write_b32(float *__restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = 1.0f;
}

int main() {
    const size_t bytes = 512ull << 20;
    float *buf, *out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    if (hipMemset(buf, 0, bytes) != hipSuccess) return 1;
    const int grid = 256 * 32;
    for (int rep = 0; rep < 2; ++rep) {
        read_b32<<<grid, 256>>>(buf, bytes / 4, out);
        read_b96<<<grid, 256>>>((const uint8_t *)buf, bytes / 3, out);
        read_b128<<<grid, 256>>>((const float4 *)buf, bytes / 16, out);
        write_b32<<<grid, 256>>>(buf, bytes / 4);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("streamed %zu bytes per kernel (read_b96: %zu)\n", bytes, (bytes / 3 / 4) * 12);
    return 0;
}
