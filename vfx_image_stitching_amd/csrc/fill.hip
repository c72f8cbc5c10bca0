// fill.hip -- stream-ordered byte fill used instead of hipMemsetAsync on every path that may
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
