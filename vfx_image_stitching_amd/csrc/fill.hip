// fill.hip -- small utility kernels.  Stream-ordered byte fill used instead of hipMemsetAsync on every path that may
// be captured into a hipGraph: the fill is an ordinary kernel whose arguments (pointer,
// byte, size) are captured by value, so replays never depend on the runtime's internal
// memset implementation.  16 bytes per thread where alignment allows, bytes at the edges.
#include "pano_internal.h"

namespace {

__global__ void __launch_bounds__(256)
fill_bytes(uint8_t *__restrict__ dst, uint32_t word, size_t head, size_t n16, size_t bytes) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n16) {
        uint4 *p = (uint4 *)(dst + head) + i;
        *p = make_uint4(word, word, word, word);
    }
    // unaligned head and tail bytes (fewer than 16 each), one byte per thread
    const size_t tail0 = head + n16 * 16;
    if (i < head) dst[i] = (uint8_t)word;
    if (i < bytes - tail0) dst[tail0 + i] = (uint8_t)word;
}

}  // namespace

int launch_fill(pano_ctx *ctx, void *dst, uint8_t value, size_t bytes) {
    if (!bytes) return PANO_OK;
    uint8_t *d = (uint8_t *)dst;
    size_t head = (16 - ((uintptr_t)d & 15)) & 15;
    if (head > bytes) head = bytes;
    const size_t n16 = (bytes - head) / 16;
    const uint32_t word = 0x01010101u * value;
    size_t threads = n16 > 16 ? n16 : 16;
    const unsigned blocks = (unsigned)((threads + 255) / 256);
    fill_bytes<<<blocks, 256, 0, ctx->stream>>>(d, word, head, n16, bytes);
    PANO_LAUNCH_CHECK(ctx, "fill_bytes");
    return PANO_OK;
}

// Small copies as a kernel (graph kernel node) instead of a hipMemcpyAsync (a blit / SDMA
// node): the batched stitch's one device -> pinned-host read of its ~1.3 KB result head is
// written by the GPU straight into the mapped host buffer (round 2 timeline: ~30 us around
// the copy node).  Both pointers must be device-addressable (device or pinned host memory).
__global__ void __launch_bounds__(256)
copy_bytes(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst, size_t bytes) {
    const size_t n16 = ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) ? bytes / 16 : 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
        ((uint4 *)dst)[i] = ((const uint4 *)src)[i];
    for (size_t i = n16 * 16 + (size_t)blockIdx.x * 256 + threadIdx.x; i < bytes; i += (size_t)gridDim.x * 256)
        dst[i] = src[i];
}

int launch_copy(pano_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (!bytes) return PANO_OK;
    const size_t items = ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) ? bytes / 16 + 16 : bytes;
    const unsigned blocks = (unsigned)std::min<size_t>((items + 255) / 256, 1024);
    copy_bytes<<<blocks, 256, 0, ctx->stream>>>((const uint8_t *)src, (uint8_t *)dst, bytes);
    PANO_LAUNCH_CHECK(ctx, "copy_bytes");
    return PANO_OK;
}

// S0's float-BGR gray (sift_impl.py:27-28 on a float32 image): cv2.cvtColor(COLOR_BGR2GRAY),
// OpenCV's RGB2Gray<float> scalar body dst = src[0] * 0.114f + src[1] * 0.587f + src[2] *
// 0.299f, left to right, no contraction (the Makefile builds with -ffp-contract=off).  One
// thread per pixel; [n][h][w][3] -> [n][h][w].
__global__ void __launch_bounds__(256)
gray_bgr_f32(const float *__restrict__ bgr, float *__restrict__ gray, size_t px) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= px) return;
    const float *q = bgr + 3 * i;
    gray[i] = (q[0] * 0.114f + q[1] * 0.587f) + q[2] * 0.299f;
}

int pano_gray_bgr_f32(pano_ctx *ctx, const float *bgr, int n, int h, int w, float *gray) {
    if (!ctx || !bgr || !gray || n <= 0 || h <= 0 || w <= 0)
        return ctx ? pano_fail(ctx, PANO_E_ARG, "pano_gray_bgr_f32") : PANO_E_ARG;
    const size_t px = (size_t)n * h * w;
    gray_bgr_f32<<<(unsigned)((px + 255) / 256), 256, 0, ctx->stream>>>(bgr, gray, px);
    PANO_LAUNCH_CHECK(ctx, "gray_bgr_f32");
    return PANO_OK;
}

// Exact squared norms of byte descriptor rows (what pano_match_u8 reads beside the bytes):
// one wave per 8 rows, 8 lanes per row, each lane 16 bytes (v_dot4_u32_u8 on its 4 words),
// then a 3-step shuffle reduction inside the row's lane group.
__global__ void __launch_bounds__(256)
desc_norms_u8(const uint8_t *__restrict__ desc, int32_t *__restrict__ norms, int rows) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    const int r = t >> 3, part = t & 7;
    uint32_t s = 0;
    if (r < rows) {
        const uint4 v = ((const uint4 *)(desc + (size_t)r * 128))[part];
        s = __builtin_amdgcn_udot4(v.x, v.x, 0u, false);
        s = __builtin_amdgcn_udot4(v.y, v.y, s, false);
        s = __builtin_amdgcn_udot4(v.z, v.z, s, false);
        s = __builtin_amdgcn_udot4(v.w, v.w, s, false);
    }
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    s += __shfl_xor(s, 4);
    if (r < rows && part == 0) norms[r] = (int32_t)s;
}

int pano_desc_norms_u8(pano_ctx *ctx, const uint8_t *desc, int rows, int32_t *norms) {
    if (!ctx || rows < 0 || (rows && (!desc || !norms)))
        return ctx ? pano_fail(ctx, PANO_E_ARG, "pano_desc_norms_u8") : PANO_E_ARG;
    if ((uintptr_t)desc & 15)
        return pano_fail(ctx, PANO_E_ARG, "pano_desc_norms_u8: rows must be 16-byte aligned");
    if (!rows) return PANO_OK;
    const size_t threads = (size_t)rows * 8;
    desc_norms_u8<<<(unsigned)((threads + 255) / 256), 256, 0, ctx->stream>>>(desc, norms, rows);
    PANO_LAUNCH_CHECK(ctx, "desc_norms_u8");
    return PANO_OK;
}
