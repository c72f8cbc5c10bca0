// jpeg_enc.hip -- baseline JPEG encode on the GPU: the reference's
// cv2.imwrite of the cropped panorama (image_stitching_sift.py:386, quality 95), byte-identical
// to libjpeg-turbo with its defaults (what PIL's save(quality=q) writes): YCbCr 4:2:0, islow
// forward DCT, reciprocal quantisation, Annex K Huffman tables, JFIF header.
//
// Five launches:
//   jpeg_enc_blocks   8 threads per 8x8 block (MCU order; row, then column): colour conversion, edge
//                     replication and h2v2 downsampling of its samples, forward DCT,
//                     quantisation (jpeg_core.h enc_samples / enc_transform); the luma blocks
//                     outside the image's block grid take the DC of the block libjpeg copies;
//   jpeg_enc_lengths  the Huffman bit count of every block (its DC difference needs the
//                     previous block of its component) and per-chunk sums;
//   jpeg_enc_emit     each block's bits at its offset (chunk prefix + block scan) into a zeroed
//                     word stream: full words by plain stores, the two shared edge words by
//                     atomic OR;
//   jpeg_enc_ff_count / jpeg_enc_stuff  the bytes with the final ones-padding, a 0x00 after
//                     every 0xFF (a chunked stream expansion), and the total length.
// The host writes the header (jpeg_host.cpp encode_header) and the EOI marker around the
// entropy-coded bytes it copies back.
#include <cstring>

#include "jpeg_core.h"
#include "pano_internal.h"

using namespace pj;

namespace {

constexpr int kEncThreads = 128;
constexpr int kLenChunk = 128;           // blocks per length-prefix chunk: one per thread (a 2.2 Mpx panorama: ~420 workgroups)
constexpr int kByteChunk = 16 * kEncThreads;   // bytes per stuffing chunk: 16 consecutive bytes per thread

struct EncTabs {
    QRecip q[2][64];                     // luma, chroma reciprocals (natural order)
    HuffEnc e[4];                        // DC lum, AC lum, DC chr, AC chr
    uint8_t nat[64];
};

struct EncDev {
    const uint8_t *img;
    EncGeom G;
    int nblk;
    const EncTabs *tabs;
    int16_t *coef;                       // [nblk][64] natural order
    uint32_t *len;                       // [nblk] Huffman bits per block
    uint32_t *chunk_bits;                // [nchunk] bits per kLenChunk blocks
    int nchunk;
    uint32_t *words;                     // bit stream, first bit = MSB of word 0
    uint32_t *ff_cnt;                    // [nbchunk]
    uint8_t *out;                        // stuffed bytes
    uint32_t *total;                     // [0] stream bits, [1] stuffed bytes
};

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
}

// kEncThreads-thread exclusive scan
__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t *wsum, uint32_t *total) {
    constexpr int NW = kEncThreads / 64;
    const uint32_t x = wave_incl_scan(v);
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 63) wsum[wv] = x;
    __syncthreads();
    uint32_t base = 0, tot = 0;
    for (int i = 0; i < NW; ++i) {
        base += i < wv ? wsum[i] : 0;
        tot += wsum[i];
    }
    *total = tot;
    __syncthreads();
    return base + x - v;
}

__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t *wsum) {
    uint32_t t;
    (void)block_exscan(v, wsum, &t);
    return t;
}

// 32 blocks per workgroup, 8 threads per block: thread r samples and transforms row r, then
// (after an LDS transpose) transforms and quantises column r.
__global__ void __launch_bounds__(kEncThreads) jpeg_enc_blocks(EncDev D) {
    __shared__ int32_t ws[kEncThreads / 8][8][9];
    __shared__ QRecip q[2][64];
    for (int i = threadIdx.x; i < 128; i += kEncThreads) q[i >> 6][i & 63] = D.tabs->q[i >> 6][i & 63];
    const int lb = threadIdx.x >> 3, r = threadIdx.x & 7;
    const int b = blockIdx.x * (kEncThreads / 8) + lb;
    const bool live = b < D.nblk;
    int src = live ? enc_dummy_source(D.G, b) : -1;
    const bool dummy = src >= 0;
    if (dummy && enc_dummy_source(D.G, src) >= 0) src = enc_dummy_source(D.G, src);
    const int sb = dummy ? src : b;
    int32_t row[8];
    if (live) {
        enc_sample_row(D.img, D.G, sb, r, row);
        fdct8(row, 1);
        for (int c = 0; c < 8; ++c) ws[lb][r][c] = row[c];
    }
    __syncthreads();
    if (!live) return;
    int32_t col[8];
    for (int i = 0; i < 8; ++i) col[i] = ws[lb][i][r];
    fdct8(col, 2);
    const QRecip *qq = q[(b % 6) < 4 ? 0 : 1];
    int16_t *dst = D.coef + (size_t)b * 64;
    for (int i = 0; i < 8; ++i) {
        const int v = quantize(col[i], qq[i * 8 + r]);
        dst[i * 8 + r] = (int16_t)(dummy && (i | r) ? 0 : v);   // a dummy block keeps the DC only
    }
}

// In-place exclusive scan of v[0 .. n) by one 1024-thread workgroup, 1024 entries per step
// with a running carry: the chunk offsets of jpeg_enc_emit (bits) and jpeg_enc_stuff (0xFF
// bytes).  Each chunk workgroup then reads its own offset -- O(nchunk) in all, where summing
// every earlier chunk per workgroup was O(nchunk^2) (tens of thousands of chunks on a
// config-5-sized canvas).
constexpr int kScanThreads = 1024;
__global__ void __launch_bounds__(kScanThreads) jpeg_enc_exscan(uint32_t *__restrict__ v, int n) {
    __shared__ uint32_t ws[kScanThreads / 64];
    const int wv = threadIdx.x >> 6;
    uint32_t carry = 0;
    for (int base = 0; base < n; base += kScanThreads) {
        const int i = base + (int)threadIdx.x;
        const uint32_t x = i < n ? v[i] : 0u;
        const uint32_t inc = wave_incl_scan(x);
        if ((threadIdx.x & 63) == 63) ws[wv] = inc;
        __syncthreads();
        uint32_t wbase = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < kScanThreads / 64; ++w) {
            const uint32_t t = ws[w];
            wbase += w < wv ? t : 0u;
            tot += t;
        }
        if (i < n) v[i] = carry + wbase + inc - x;
        carry += tot;
        __syncthreads();                 // ws is rewritten by the next step
    }
}

struct CountPut {
    uint32_t n = 0;
    __device__ __forceinline__ void operator()(uint32_t, int len) { n += (uint32_t)len; }
};

__device__ __forceinline__ int dc_diff(const EncDev &D, int b) {
    const int p = enc_prev_same(b);
    return D.coef[(size_t)b * 64] - (p >= 0 ? D.coef[(size_t)p * 64] : 0);
}

__global__ void __launch_bounds__(kEncThreads) jpeg_enc_lengths(EncDev D) {
    __shared__ uint32_t wsum[kEncThreads / 64];
    __shared__ uint32_t acc;
    __shared__ EncTabs T;
    for (int i = threadIdx.x; i < (int)(sizeof(EncTabs) / 4); i += kEncThreads)
        ((uint32_t *)&T)[i] = ((const uint32_t *)D.tabs)[i];
    if (threadIdx.x == 0) acc = 0;
    __syncthreads();
    // one workgroup per chunk of kLenChunk blocks
    const int b0 = blockIdx.x * kLenChunk;
    for (int b = b0 + threadIdx.x; b < b0 + kLenChunk; b += kEncThreads) {
        uint32_t n = 0;
        if (b < D.nblk) {
            const int c = (b % 6) < 4 ? 0 : 1;
            CountPut cp;
            encode_block(D.coef + (size_t)b * 64, dc_diff(D, b), &T.e[2 * c], &T.e[2 * c + 1], T.nat, cp);
            n = cp.n;
            D.len[b] = n;
        }
        const uint32_t s = block_sum(n, wsum);
        if (threadIdx.x == 0) acc += s;
        __syncthreads();
    }
    if (threadIdx.x == 0) D.chunk_bits[blockIdx.x] = acc;
}

// Bits of one block from bit offset `pos`: a 64-bit accumulator flushed a word at a time.
struct EmitPut {
    uint32_t *words;
    uint64_t acc;        // left-aligned pending bits
    int nacc;            // pending bits, counting the `lead` bits of the first word
    uint32_t w;          // word being filled
    bool first;
    __device__ __forceinline__ void flush_word(uint32_t v) {
        if (first) atomicOr(&words[w], v);     // shares its leading bits with the block before
        else words[w] = v;
        first = false;
        ++w;
    }
    __device__ __forceinline__ void operator()(uint32_t v, int len) {
        acc |= (uint64_t)(v & ((1u << len) - 1)) << (64 - nacc - len);
        nacc += len;
        if (nacc >= 32) {
            flush_word((uint32_t)(acc >> 32));
            acc <<= 32;
            nacc -= 32;
        }
    }
    __device__ __forceinline__ void finish() {
        if (nacc > 0) atomicOr(&words[w], (uint32_t)(acc >> 32));   // shared with the next block
    }
};

__global__ void __launch_bounds__(kEncThreads) jpeg_enc_emit(EncDev D) {
    __shared__ uint32_t wsum[kEncThreads / 64];
    __shared__ uint32_t base;
    __shared__ EncTabs T;
    for (int i = threadIdx.x; i < (int)(sizeof(EncTabs) / 4); i += kEncThreads)
        ((uint32_t *)&T)[i] = ((const uint32_t *)D.tabs)[i];
    // bits before this chunk: chunk_bits holds the exclusive prefix (jpeg_enc_exscan)
    if (threadIdx.x == 0) base = D.chunk_bits[blockIdx.x];
    __syncthreads();
    const int b0 = blockIdx.x * kLenChunk;
    for (int b = b0 + threadIdx.x; b < b0 + kLenChunk; b += kEncThreads) {
        const uint32_t n = b < D.nblk ? D.len[b] : 0;
        uint32_t tot;
        const uint32_t off = base + block_exscan(n, wsum, &tot);
        if (b < D.nblk && n) {
            const int c = (b % 6) < 4 ? 0 : 1;
            EmitPut ep;
            ep.words = D.words;
            ep.acc = 0;
            ep.nacc = (int)(off & 31);
            ep.w = off >> 5;
            ep.first = true;
            encode_block(D.coef + (size_t)b * 64, dc_diff(D, b), &T.e[2 * c], &T.e[2 * c + 1], T.nat, ep);
            ep.finish();
        }
        if (b == D.nblk - 1) D.total[0] = off + n;
        __syncthreads();
        if (threadIdx.x == 0) base += tot;
        __syncthreads();
    }
}

// Byte j of the padded stream: bits past the end of the data are ones (jchuff.c flush_bits).
__device__ __forceinline__ uint32_t stream_byte(const uint32_t *words, uint32_t nbits, uint32_t j) {
    uint32_t v = (words[j >> 2] >> (24 - 8 * (j & 3))) & 0xFF;
    const uint32_t bit0 = j * 8;
    if (bit0 + 8 > nbits) {
        const uint32_t valid = nbits > bit0 ? nbits - bit0 : 0;
        v |= 0xFFu >> valid;
    }
    return v;
}

__global__ void __launch_bounds__(kEncThreads) jpeg_enc_ff_count(EncDev D) {
    __shared__ uint32_t wsum[kEncThreads / 64];
    const uint32_t nbits = D.total[0], nbytes = (nbits + 7) / 8;
    const uint32_t j0 = blockIdx.x * kByteChunk;
    uint32_t n = 0;
    for (uint32_t j = j0 + threadIdx.x; j < j0 + kByteChunk && j < nbytes; j += kEncThreads)
        n += stream_byte(D.words, nbits, j) == 0xFF;
    const uint32_t t = block_sum(n, wsum);
    if (threadIdx.x == 0) D.ff_cnt[blockIdx.x] = t;
}

__global__ void __launch_bounds__(kEncThreads) jpeg_enc_stuff(EncDev D) {
    __shared__ uint32_t wsum[kEncThreads / 64];
    __shared__ uint32_t base;
    const uint32_t nbits = D.total[0], nbytes = (nbits + 7) / 8;
    const uint32_t j0 = blockIdx.x * kByteChunk;
    // 0xFF bytes before this chunk: ff_cnt holds the exclusive prefix (jpeg_enc_exscan)
    if (threadIdx.x == 0) base = D.ff_cnt[blockIdx.x] + j0;   // output position of byte j0
    __syncthreads();
    // 16 consecutive bytes per thread (kByteChunk = 16 * kEncThreads)
    const uint32_t jt = j0 + threadIdx.x * 16;
    uint32_t by[16], ff = 0;
    for (int i = 0; i < 16; ++i) {
        const uint32_t j = jt + i;
        by[i] = j < nbytes ? stream_byte(D.words, nbits, j) : 0;
        ff += j < nbytes && by[i] == 0xFF;
    }
    uint32_t tot;
    const uint32_t before = block_exscan(ff, wsum, &tot);
    uint32_t o = base + (jt - j0) + before;
    for (int i = 0; i < 16; ++i) {
        if (jt + i >= nbytes) break;
        D.out[o++] = (uint8_t)by[i];
        if (by[i] == 0xFF) D.out[o++] = 0;
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) D.total[1] = base + (nbytes - j0) + tot;
}

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

}  // namespace

int launch_jpeg_encode(pano_ctx *ctx, const uint8_t *bgr, int h, int w, int64_t pitch, int quality,
                       uint8_t *h_out, size_t cap, size_t *out_len) {
    const EncGeom G = enc_geom(h, w, pitch);
    const int nblk = G.mcus_x * G.mcus_y * 6;
    const int nchunk = (nblk + kLenChunk - 1) / kLenChunk;
    // stream size bound: 64 coefficients x (16-bit code + 11-bit value) per block
    const size_t max_bits = (size_t)nblk * 64 * 27 + 64;
    if (max_bits >= (1ull << 32)) return pano_fail(ctx, PANO_E_UNSUPPORTED, "JPEG encode: image too large");
    const size_t max_bytes = (max_bits + 7) / 8;
    const int nbchunk = (int)((max_bytes + kByteChunk - 1) / kByteChunk);
    uint16_t lum[64], chr[64];
    quant_tables(quality, lum, chr);
    EncTabs tabs;
    memset(&tabs, 0, sizeof(tabs));
    for (int i = 0; i < 64; ++i) {
        tabs.q[0][i] = q_recip(8u * lum[i]);
        tabs.q[1][i] = q_recip(8u * chr[i]);
        tabs.nat[i] = (uint8_t)natural_order(i);
    }
    std_huff_enc(0, 0, &tabs.e[0]);
    std_huff_enc(1, 0, &tabs.e[1]);
    std_huff_enc(0, 1, &tabs.e[2]);
    std_huff_enc(1, 1, &tabs.e[3]);
    const std::vector<uint8_t> hdr = encode_header(h, w, lum, chr);

    size_t dv = 0;
    const size_t o_tabs = dv;   dv = align_up(dv + sizeof(EncTabs), 256);
    const size_t o_coef = dv;   dv = align_up(dv + (size_t)nblk * 128, 256);
    const size_t o_len = dv;    dv = align_up(dv + 4 * (size_t)nblk, 256);
    const size_t o_chunk = dv;  dv = align_up(dv + 4 * (size_t)nchunk, 256);
    const size_t o_words = dv;  dv = align_up(dv + 4 * ((max_bits + 31) / 32 + 2), 256);
    const size_t o_ff = dv;     dv = align_up(dv + 4 * (size_t)nbchunk, 256);
    const size_t o_out = dv;    dv = align_up(dv + 2 * max_bytes + 16, 256);
    const size_t o_total = dv;  dv = align_up(dv + 16, 256);
    // shares the JPEG decoder's scratch (the calls are stream-ordered)
    int rc = pano_grow(ctx, &ctx->jscratch, &ctx->jscratch_bytes, dv);
    if (rc) return rc;
    uint8_t *dev = (uint8_t *)ctx->jscratch;
    // pinned staging (a pageable source or destination makes each copy a staged, blocking
    // one); the previous encode synchronised before returning, so the buffer is free
    constexpr size_t kEpinTot = (sizeof(EncTabs) + 255) / 256 * 256;
    if (!ctx->epin) PANO_HIP(ctx, hipHostMalloc(&ctx->epin, kEpinTot + 256, hipHostMallocDefault));
    memcpy(ctx->epin, &tabs, sizeof(tabs));
    PANO_HIP(ctx, hipMemcpyAsync(dev + o_tabs, ctx->epin, sizeof(tabs), hipMemcpyHostToDevice, ctx->stream));
    EncDev D;
    D.img = bgr;
    D.G = G;
    D.nblk = nblk;
    D.tabs = (const EncTabs *)(dev + o_tabs);
    D.coef = (int16_t *)(dev + o_coef);
    D.len = (uint32_t *)(dev + o_len);
    D.chunk_bits = (uint32_t *)(dev + o_chunk);
    D.nchunk = nchunk;
    D.words = (uint32_t *)(dev + o_words);
    D.ff_cnt = (uint32_t *)(dev + o_ff);
    D.out = dev + o_out;
    D.total = (uint32_t *)(dev + o_total);
    {
        PanoProf prof_(ctx, PK_JPEG);
        rc = launch_fill(ctx, D.words, 0, 4 * ((max_bits + 31) / 32 + 2));
        if (rc) return rc;
        jpeg_enc_blocks<<<(nblk + kEncThreads / 8 - 1) / (kEncThreads / 8), kEncThreads, 0, ctx->stream>>>(D);
        jpeg_enc_lengths<<<nchunk, kEncThreads, 0, ctx->stream>>>(D);
        jpeg_enc_exscan<<<1, kScanThreads, 0, ctx->stream>>>(D.chunk_bits, nchunk);
        jpeg_enc_emit<<<nchunk, kEncThreads, 0, ctx->stream>>>(D);
        jpeg_enc_ff_count<<<nbchunk, kEncThreads, 0, ctx->stream>>>(D);
        jpeg_enc_exscan<<<1, kScanThreads, 0, ctx->stream>>>(D.ff_cnt, nbchunk);
        jpeg_enc_stuff<<<nbchunk, kEncThreads, 0, ctx->stream>>>(D);
        PANO_LAUNCH_CHECK(ctx, "jpeg encode");
    }
    uint32_t *tot = (uint32_t *)((uint8_t *)ctx->epin + kEpinTot);
    PANO_HIP(ctx, hipMemcpyAsync(tot, D.total, 8, hipMemcpyDeviceToHost, ctx->stream));
    PANO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    const size_t need = hdr.size() + tot[1] + 2;
    if (out_len) *out_len = need;
    if (!h_out || cap < need) return pano_fail(ctx, PANO_E_OVERFLOW, "JPEG encode: output buffer too small");
    memcpy(h_out, hdr.data(), hdr.size());
    PANO_HIP(ctx, hipMemcpy(h_out + hdr.size(), D.out, tot[1], hipMemcpyDeviceToHost));
    h_out[hdr.size() + tot[1]] = 0xFF;
    h_out[hdr.size() + tot[1] + 1] = 0xD9;
    return PANO_OK;
}
