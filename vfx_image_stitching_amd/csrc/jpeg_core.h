// jpeg_core.h -- baseline JPEG decode: the per-thread pieces the HIP
// kernels of jpeg.hip run, written once as __host__ __device__ functions so that
// tools/jpeg_sim.cpp can replay the same arithmetic on the CPU while the kernels are developed.
//
// What is being reproduced: the reference reads every frame with cv2.imread
// (image_stitching_sift.py:282, image_stitching_harris.py:394); the harness decodes with
// PIL (vfx_image_stitching_amd/data.py), which SURVEY.md section 8(c) measured pixel-identical
// to cv2.imread on these files.  Both are libjpeg-turbo with its defaults:
//   - Huffman entropy decoding, sequential baseline / extended 8-bit DCT (jdhuff.c),
//   - the accurate integer inverse DCT, JDCT_ISLOW (jidctint.c: 13-bit constants, 2 extra
//     bits after the column pass, range limit through a 1024-entry wrap table),
//   - "fancy" triangular chroma upsampling for h2v1 / h2v2 (jdsample.c) with the context rows
//     of jdmainct.c (rows above the top / below the bottom replicate the edge row),
//   - YCbCr -> RGB with 16-bit fixed-point tables (jdcolor.c).
// Everything here is integer arithmetic and is bit-exact by construction; tests compare the
// GPU output with PIL's decode byte for byte.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

namespace pj {

constexpr int kMaxComp = 3;     // gray or YCbCr
constexpr int kMaxBpm = 10;     // blocks per MCU (JPEG limit)
#ifndef PANO_JPEG_SUB_BITS
#define PANO_JPEG_SUB_BITS 512
#endif
constexpr int kSubBits = PANO_JPEG_SUB_BITS;   // bits per subsequence of the self-synchronising decode
constexpr int kChunk = 4096;    // stuffed bytes per unstuff chunk
constexpr int kStreamPad = 64;  // zero bytes after each unstuffed stream
constexpr int kHuffSub = 16;    // second-level lookup tables per Huffman table

// One Huffman table in decode form (jdhuff.c jpeg_make_d_derived_tbl restated as a two-level
// lookup): the first 9 bits of the stream index lut; codes of up to 9 bits resolve there,
// longer ones through a 128-entry second-level table indexed by the next 7 bits.  An entry
// describes the whole codeword: code length - 1 (bits 0-3), the count s of magnitude bits that
// follow (bits 4-8) and the zig-zag advance - 1 (bits 9-14: 0 for a DC code, the zero run r
// for an AC coefficient, 15 for ZRL, 63 for EOB) -- so a walker moves by length + s bits and
// k + advance positions without decoding the symbol.  lut entries with bit 15 set hold a
// second-level offset; codes the table lacks (reached only off sync) read as a 1-bit code.
// One or two LDS reads per codeword, no search loop.
// Canonical codes longer than 9 bits have contiguous 9-bit prefixes [first_long, first_long +
// nsub), assigned second-level tables 0, 1, ... in that order, so a walker computes the
// second-level index from the bits alone and reads both levels at once (one LDS round trip
// per codeword, not two dependent ones).
struct Huff {
    uint16_t lut[512];
    uint16_t sub[kHuffSub * 128];
    uint32_t first_long;        // 9-bit prefix of the first code longer than 9 bits (512: none)
};

// Everything a kernel needs about one frame (built on the host by jpeg_plan).
struct Frame {
    int32_t h, w, ncomp;
    int32_t hmax, vmax;
    int32_t mcus_x, mcus_y, bpm, total_blocks;
    int32_t comp_h[kMaxComp], comp_v[kMaxComp];     // sampling factors (1/1 for a gray scan)
    int32_t comp_bw[kMaxComp], comp_bh[kMaxComp];   // block grid of each component plane
    int32_t comp_dw[kMaxComp], comp_dh[kMaxComp];   // libjpeg downsampled_width / _height
    int32_t dc_tab[kMaxComp], ac_tab[kMaxComp];     // indices into the batch's table array
    int32_t q_tab[kMaxComp];                        // index into the batch's quant array
    int8_t mcu_comp[kMaxBpm], mcu_bx[kMaxBpm], mcu_by[kMaxBpm];
    int32_t upsample;     // 0: 4:4:4 or gray, 1: h2v1, 2: h2v2
    uint64_t coef_off[kMaxComp];   // int16 element offset of the component's coefficients
    uint64_t samp_off[kMaxComp];   // byte offset of the component's sample plane
    uint64_t src_off;     // stuffed entropy-coded segment: byte offset in the upload
    uint32_t src_len;
    uint32_t chunk0, nchunk;       // unstuff chunks
    uint64_t bits_off;    // unstuffed stream: byte offset (16-aligned) in the stream arena
    uint32_t sub0, nsub;  // subsequences reserved (from the stuffed length, an upper bound)
    uint32_t warm;        // warm-up window (bits) of the subsequence start search
};

// ---------------------------------------------------------------------------------------------
// The stream is read through a window held as 32-bit words in stream order (word i = bytes
// 4i..4i+3, first byte in the top bits): w[j] is stream word woff + j.  Words outside
// [woff, woff + nw) read as zeros (libjpeg pads with zeros after the last marker,
// jdhuff.c jpeg_fill_bit_buffer; the kernels stage every window a walk can reach in LDS).
// The 32 stream bits starting at bit `pos` (a codeword plus its magnitude bits fit in 32).
__host__ __device__ __forceinline__ uint32_t window32(const uint32_t *w, uint32_t woff, uint32_t nw, uint32_t pos) {
    // clamped indices read unconditionally, then selected: no masked (divergent) loads
    const uint32_t i = (pos >> 5) - woff, j = i + 1, last = nw - 1;
    const uint32_t a = w[i < nw ? i : last], b = w[j < nw ? j : last];
    const uint32_t av = i < nw ? a : 0u, bv = j < nw ? b : 0u;
    return (uint32_t)(((((uint64_t)av << 32) | bv) << (pos & 31)) >> 32);
}

// Codeword entry of the table for the bits x (jdhuff.c jpeg_huff_decode): both levels read,
// the second chosen by a select.
__host__ __device__ __forceinline__ uint32_t huff_entry(const Huff *T, uint32_t x) {
    const uint32_t e1 = T->lut[x >> 23];
    const uint32_t e2 = T->sub[((e1 & 0x7FFF) + ((x >> 16) & 127)) & (kHuffSub * 128 - 1)];
    return (e1 & 0x8000) ? e2 : e1;
}
// The same entry with the second-level index taken from the bits (first_long: the table's
// Huff::first_long): the two reads are independent.  For a short code the second read lands
// anywhere inside the table and is discarded.
__host__ __device__ __forceinline__ uint32_t huff_entry_par(const Huff *T, uint32_t x, uint32_t first_long) {
    const uint32_t pre = x >> 23;
    const uint32_t e1 = T->lut[pre];
    const uint32_t e2 = T->sub[(((pre - first_long) & (kHuffSub - 1)) << 7) | ((x >> 16) & 127)];
    return (e1 & 0x8000) ? e2 : e1;
}

// HUFF_EXTEND (jdhuff.h)
__host__ __device__ __forceinline__ int huff_extend(int v, int s) {
    return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v;
}

// Decoder state at a codeword boundary: bit position, block of the MCU, zig-zag index
// (0 = the block's DC code is next).  Two decodes that reach the same state decode the same
// symbols from there on: that is what the self-synchronising passes compare.
__host__ __device__ __forceinline__ uint64_t pack_state(uint32_t pos, int b, int k) {
    return (uint64_t)pos << 16 | (uint64_t)(uint32_t)b << 8 | (uint64_t)(uint32_t)k;
}
__host__ __device__ __forceinline__ uint32_t state_pos(uint64_t s) { return (uint32_t)(s >> 16); }
__host__ __device__ __forceinline__ int state_b(uint64_t s) { return (int)((s >> 8) & 0xFF); }
__host__ __device__ __forceinline__ int state_k(uint64_t s) { return (int)(s & 0xFF); }

// Per-subsequence statistics of a decode: DC codes seen (= blocks started) and the sum of
// the DC differences per component (the DC predictor is a running sum, jdhuff.c decode_mcu).
struct SubStats {
    int32_t blocks;
    int32_t dc[kMaxComp];
};

// Sinks for walk(): what to do with each decoded value.
struct SinkNone {
    static constexpr bool kValues = false;
    __host__ __device__ __forceinline__ bool dc(int, int) { return true; }
    __host__ __device__ __forceinline__ void ac(int, int) {}
    __host__ __device__ __forceinline__ void end_block() {}
};
struct SinkCount {
    static constexpr bool kValues = true;
    // per-component sums kept in three scalars (a dynamically indexed array would live in
    // scratch memory on the GPU)
    int32_t blocks = 0, d0 = 0, d1 = 0, d2 = 0;
    __host__ __device__ __forceinline__ bool dc(int c, int diff) {
        ++blocks;
        d0 += c == 0 ? diff : 0;
        d1 += c == 1 ? diff : 0;
        d2 += c == 2 ? diff : 0;
        return true;
    }
    __host__ __device__ __forceinline__ void ac(int, int) {}
    __host__ __device__ __forceinline__ void end_block() {}
    __host__ __device__ __forceinline__ SubStats stats() const {
        SubStats s;
        s.blocks = blocks; s.dc[0] = d0; s.dc[1] = d1; s.dc[2] = d2;
        return s;
    }
};

// The zig-zag -> natural order map with libjpeg's 16 guard entries (jutils.c
// jpeg_natural_order: a corrupt run past 63 lands on 63).
__host__ __device__ __forceinline__ int natural_order(int k) {
    // Row-major position of the k-th zig-zag coefficient, computed (no table) from the
    // anti-diagonal it lies on: diagonal d holds k in [d(d+1)/2 ...) for d < 8 and mirrors
    // for the lower-right half.
    if (k > 63) return 63;
    int d, i;
    if (k < 36) {                       // upper-left triangle, diagonals 0..7
        d = 0; while ((d + 1) * (d + 2) / 2 <= k) ++d;
        i = k - d * (d + 1) / 2;        // index along the diagonal
        const int r = (d & 1) ? i : d - i;
        return r * 8 + (d - r);
    }
    const int kk = 63 - k;              // mirror: lower-right triangle
    d = 0; while ((d + 1) * (d + 2) / 2 <= kk) ++d;
    i = kk - d * (d + 1) / 2;
    const int r = (d & 1) ? i : d - i;  // position in the mirrored block
    return 63 - (r * 8 + (d - r));
}

// Walk the codewords that start in [start, end): from state `start` decode until the bit
// position reaches `end`; returns the state at the first boundary >= end.  The sink sees
// every DC difference (dc returns false to stop early) and AC coefficient.  T: the DC tables
// of components 0..2 followed by their AC tables (T[c], T[3 + c]).  Every codeword takes one
// instruction path (selects, not branches) up to the sink calls, so the lanes of a wave, each
// at its own decoder state, do not serialise on divergent paths.
template <class Sink>
__host__ __device__ __forceinline__ uint64_t walk(const uint32_t *words, uint32_t woff, uint32_t nwords,
                                                  uint64_t start, uint32_t end, const Huff *T,
                                                  const int8_t *mcu_comp, int bpm, Sink &sink) {
    uint32_t pos = state_pos(start);
    int b = state_b(start), k = state_k(start);
    // the MCU layout as 2 bits per block in a register (no memory read per block)
    uint32_t layout = 0;
    for (int i = 0; i < bpm; ++i) layout |= (uint32_t)(mcu_comp[i] & 3) << (2 * i);
    // each table's first long prefix, 10 bits apiece (tables 0..5: DC of components 0..2,
    // then their AC tables)
    uint64_t flpack = 0;
    for (int i = 0; i < 6; ++i) flpack |= (uint64_t)(T[i].first_long & 1023) << (10 * i);
    int c = (int)(layout >> (2 * b)) & 3;
    // bit buffer: buf holds stream bits [pos, pos + cnt) left-aligned, cnt >= 32 at the top of
    // every iteration; nxt is the next stream word, loaded an iteration before it is needed, so
    // the only reads on a codeword's critical path are its table entries
    const uint32_t last = nwords - 1;
    auto rd = [&](uint32_t wi) -> uint32_t {
        const uint32_t j = wi - woff;
        const uint32_t v = words[j < nwords ? j : last];
        return j < nwords ? v : 0u;
    };
    uint32_t wi = pos >> 5;
    uint64_t buf = (((uint64_t)rd(wi) << 32) | rd(wi + 1)) << (pos & 31);
    int cnt = 64 - (int)(pos & 31);
    wi += 2;
    uint32_t nxt = rd(wi);
    uint32_t guard = end - pos + 64;   // every codeword consumes >= 1 bit
    while (pos < end && guard--) {
        const bool need = cnt < 32;
        buf |= need ? (uint64_t)nxt << ((32 - cnt) & 63) : 0ull;
        cnt += need ? 32 : 0;
        wi += need ? 1u : 0u;
        nxt = rd(wi);
        const uint32_t x = (uint32_t)(buf >> 32);
        const bool isdc = k == 0;
        const int tix = isdc ? c : 3 + c;
        const uint32_t e = huff_entry_par(T + tix, x, (uint32_t)(flpack >> (10 * tix)) & 1023);
        const int cl = (int)(e & 15) + 1;
        const int s = (int)((e >> 4) & 31);
        const int adv = (int)((e >> 9) & 63) + 1;
        const int used = cl + s;
        pos += (uint32_t)used;
        buf = used < 64 ? buf << used : 0ull;
        cnt -= used;
        if (Sink::kValues) {
            const uint32_t raw = s ? (x << cl) >> (32 - s) : 0u;
            const int v = s ? huff_extend((int)raw, s) : 0;
            if (isdc) {
                if (!sink.dc(c, v)) break;
            } else if (s) {
                sink.ac(k + adv - 1, v);
            }
        }
        const int kn = k + adv;
        const bool eob = kn >= 64;
        b = eob ? (b + 1 == bpm ? 0 : b + 1) : b;
        k = eob ? 0 : kn;
        c = (int)(layout >> (2 * b)) & 3;
        if (Sink::kValues && eob) sink.end_block();
    }
    return pack_state(pos, b, k);
}

// Block index (MCU order) -> coefficient block address (int16 elements).
__host__ __device__ __forceinline__ uint64_t block_addr(const Frame &F, int32_t blk) {
    const int32_t m = blk / F.bpm, bb = blk - m * F.bpm;
    const int32_t mx = m % F.mcus_x, my = m / F.mcus_x;
    const int c = F.mcu_comp[bb];
    const int32_t bx = mx * F.comp_h[c] + F.mcu_bx[bb];
    const int32_t by = my * F.comp_v[c] + F.mcu_by[bb];
    return F.coef_off[c] + ((uint64_t)by * F.comp_bw[c] + bx) * 64;
}

// Writes coefficients of the blocks a subsequence decodes (natural order, DC predicted).  The
// block position advances incrementally (block of the MCU, MCU column, MCU row): no division
// per block.
struct SinkWrite {
    static constexpr bool kValues = true;
    int16_t *coef;
    const Frame *F;
    const uint8_t *nat;           // natural_order(k) for k < 80 (a table in LDS / host memory)
    int32_t blk;                  // current block index (MCU order)
    int32_t bb, mx, my;           // its block of the MCU, MCU column and row
    int32_t p0, p1, p2;           // DC predictors of components 0..2
    uint64_t addr;                // current block's address
    bool live;
    __host__ __device__ __forceinline__ void seek(int32_t b) {     // position of block b
        blk = b;
        const int32_t m = b / F->bpm;
        bb = b - m * F->bpm;
        mx = m % F->mcus_x;
        my = m / F->mcus_x;
    }
    __host__ __device__ __forceinline__ uint64_t address() const {
        const int c = F->mcu_comp[bb];
        return F->coef_off[c] + ((uint64_t)(my * F->comp_v[c] + F->mcu_by[bb]) * F->comp_bw[c] +
                                 mx * F->comp_h[c] + F->mcu_bx[bb]) * 64;
    }
    __host__ __device__ __forceinline__ bool dc(int c, int diff) {
        if (blk >= F->total_blocks) return false;
        p0 += c == 0 ? diff : 0;
        p1 += c == 1 ? diff : 0;
        p2 += c == 2 ? diff : 0;
        addr = address();
        live = true;
        coef[addr] = (int16_t)(c == 0 ? p0 : (c == 1 ? p1 : p2));
        return true;
    }
    __host__ __device__ __forceinline__ void ac(int k, int v) {
        if (live) coef[addr + nat[k < 80 ? k : 79]] = (int16_t)v;
    }
    __host__ __device__ __forceinline__ void end_block() {
        ++blk;
        live = false;
        if (++bb == F->bpm) {
            bb = 0;
            if (++mx == F->mcus_x) { mx = 0; ++my; }
        }
    }
};

// ---------------------------------------------------------------------------------------------
// Inverse DCT: jidctint.c jpeg_idct_islow (CONST_BITS 13, PASS1_BITS 2), 64-bit JLONG math.
__host__ __device__ __forceinline__ int range_limit_idct(int64_t x) {
    // sample_range_limit + CENTERJSAMPLE indexed by (x & RANGE_MASK) (jdmaster.c
    // prepare_range_limit_table): [0,128) -> x+128, [128,512) -> 255, [512,896) -> 0,
    // [896,1024) -> x-896 (i.e. x+128 for x in [-128,0)).
    const int i = (int)x & 1023;
    if (i < 128) return i + 128;
    if (i < 512) return 255;
    if (i < 896) return 0;
    return i - 896;
}

// One 8-point pass.  in[0..7] (stride s), out8: the 8 results before descale.
__host__ __device__ __forceinline__ void idct8(const int64_t *z, int64_t *o) {
    const int64_t F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373,
                  F1175 = 9633, F1501 = 12299, F1847 = 15137, F1961 = 16069, F2053 = 16819,
                  F2562 = 20995, F3072 = 25172;
    // even part
    int64_t z2 = z[2], z3 = z[6];
    int64_t z1 = (z2 + z3) * F0541;
    int64_t tmp2 = z1 + z3 * (-F1847);
    int64_t tmp3 = z1 + z2 * F0765;
    int64_t tmp0 = (z[0] + z[4]) * 8192;
    int64_t tmp1 = (z[0] - z[4]) * 8192;
    const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    // odd part
    tmp0 = z[7]; tmp1 = z[5]; tmp2 = z[3]; tmp3 = z[1];
    z1 = tmp0 + tmp3; z2 = tmp1 + tmp2; z3 = tmp0 + tmp2;
    int64_t z4 = tmp1 + tmp3;
    const int64_t z5 = (z3 + z4) * F1175;
    tmp0 *= F0298; tmp1 *= F2053; tmp2 *= F3072; tmp3 *= F1501;
    z1 *= -F0899; z2 *= -F2562; z3 *= -F1961; z4 *= -F0390;
    z3 += z5; z4 += z5;
    tmp0 += z1 + z3; tmp1 += z2 + z4; tmp2 += z2 + z3; tmp3 += z1 + z4;
    o[0] = tmp10 + tmp3; o[7] = tmp10 - tmp3;
    o[1] = tmp11 + tmp2; o[6] = tmp11 - tmp2;
    o[2] = tmp12 + tmp1; o[5] = tmp12 - tmp1;
    o[3] = tmp13 + tmp0; o[4] = tmp13 - tmp0;
}

__host__ __device__ __forceinline__ int64_t descale(int64_t x, int n) {
    return (x + ((int64_t)1 << (n - 1))) >> n;
}

// Column pass of one column: coef column c (natural order) x quant -> ws column (int).
__host__ __device__ __forceinline__ void idct_col(const int16_t *blk, const uint16_t *q, int c, int32_t *ws) {
    int64_t z[8], o[8];
    for (int r = 0; r < 8; ++r) z[r] = (int64_t)((int32_t)blk[r * 8 + c] * (int32_t)q[r * 8 + c]);
    idct8(z, o);
    for (int r = 0; r < 8; ++r) ws[r * 8 + c] = (int32_t)descale(o[r], 11);
}
// Row pass of one row: ws row r -> 8 samples.
__host__ __device__ __forceinline__ void idct_row(const int32_t *ws, int r, uint8_t *out) {
    int64_t z[8], o[8];
    for (int c = 0; c < 8; ++c) z[c] = ws[r * 8 + c];
    idct8(z, o);
    for (int c = 0; c < 8; ++c) out[c] = (uint8_t)range_limit_idct(descale(o[c], 18));
}

// ---------------------------------------------------------------------------------------------
// Upsampling (jdsample.c) and colour conversion (jdcolor.c), per output pixel.
// Chroma sample at output (x, y) of a component plane p (pitch ppitch) with downsampled size
// (dw, dh).  mode 0: full size; 1: h2v1 fancy; 2: h2v2 fancy.
__host__ __device__ __forceinline__ int chroma_at(const uint8_t *p, int ppitch, int dw, int dh, int mode, int x, int y) {
    if (mode == 0) return p[(size_t)y * ppitch + x];
    if (mode == 1) {
        // h2v1_fancy_upsample: first output = in[0], last output = in[dw-1]; else 3/4 nearer
        // + 1/4 farther, biased +1 (left) / +2 (right).
        const uint8_t *row = p + (size_t)y * ppitch;
        const int j = x >> 1;
        if ((x & 1) == 0) {
            if (j == 0) return row[0];
            return (row[j] * 3 + row[j - 1] + 1) >> 2;
        }
        if (j == dw - 1) return row[j];
        return (row[j] * 3 + row[j + 1] + 2) >> 2;
    }
    // h2v2_fancy_upsample: colsum = 3 * nearer row + farther row (rows outside replicate the
    // edge row, jdmainct.c context pointers); output = (3 * this + neighbour colsum + 8 | 7) >> 4.
    const int i = y >> 1;
    int i1 = (y & 1) ? i + 1 : i - 1;
    if (i1 < 0) i1 = 0;
    if (i1 > dh - 1) i1 = dh - 1;
    const uint8_t *r0 = p + (size_t)i * ppitch, *r1 = p + (size_t)i1 * ppitch;
    const int j = x >> 1;
    const int cs = r0[j] * 3 + r1[j];
    if ((x & 1) == 0) {
        if (j == 0) return (cs * 4 + 8) >> 4;
        return (cs * 3 + (r0[j - 1] * 3 + r1[j - 1]) + 8) >> 4;
    }
    if (j == dw - 1) return (cs * 4 + 7) >> 4;
    return (cs * 3 + (r0[j + 1] * 3 + r1[j + 1]) + 7) >> 4;
}

__host__ __device__ __forceinline__ int clamp255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

// ycc_rgb_convert (jdcolor.c build_ycc_rgb_table, SCALEBITS 16) -> B, G, R.
__host__ __device__ __forceinline__ void ycc_to_bgr(int y, int cb, int cr, uint8_t *bgr) {
    const int x_cb = cb - 128, x_cr = cr - 128;
    const int cr_r = (91881 * x_cr + 32768) >> 16;
    const int cb_b = (116130 * x_cb + 32768) >> 16;
    const int g = (-22554 * x_cb + 32768 + (-46802) * x_cr) >> 16;
    bgr[0] = (uint8_t)clamp255(y + cb_b);
    bgr[1] = (uint8_t)clamp255(y + g);
    bgr[2] = (uint8_t)clamp255(y + cr_r);
}

// ---------------------------------------------------------------------------------------------
// Encoder (cv2.imwrite / PIL save, quality 95: libjpeg-turbo's defaults).
// RGB -> YCbCr, jccolor.c rgb_ycc_convert (SCALEBITS 16, FIX(x) = (int)(x * 65536 + 0.5)).
__host__ __device__ __forceinline__ void rgb_to_ycc(int r, int g, int b, int &y, int &cb, int &cr) {
    const int F0299 = 19595, F0587 = 38470, F0114 = 7471, F016874 = 11059, F033126 = 21709,
              F05 = 32768, F041869 = 27439, F008131 = 5329;
    const int half = 1 << 15, off = 128 << 16;
    y = (F0299 * r + F0587 * g + F0114 * b + half) >> 16;
    cb = (-F016874 * r - F033126 * g + F05 * b + off + half - 1) >> 16;
    cr = (F05 * r - F041869 * g - F008131 * b + off + half - 1) >> 16;
}

// jfdctint.c jpeg_fdct_islow on one 8-point line (pass 1 when pass == 1: rows, descale
// CONST_BITS - PASS1_BITS; pass 2: columns, descale by PASS1_BITS / CONST_BITS + PASS1_BITS).
// d: 8 inputs (stride 1), written back in place; values are 16-bit DCTELEMs.
__host__ __device__ __forceinline__ void fdct8(int32_t *d, int pass) {
    const int64_t F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373,
                  F1175 = 9633, F1501 = 12299, F1847 = 15137, F1961 = 16069, F2053 = 16819,
                  F2562 = 20995, F3072 = 25172;
    const int64_t tmp0 = d[0] + d[7], tmp7 = d[0] - d[7], tmp1 = d[1] + d[6], tmp6 = d[1] - d[6];
    const int64_t tmp2 = d[2] + d[5], tmp5 = d[2] - d[5], tmp3 = d[3] + d[4], tmp4 = d[3] - d[4];
    const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    const int sh = pass == 1 ? 11 : 15;           // CONST_BITS -/+ PASS1_BITS
    if (pass == 1) {
        d[0] = (int16_t)((tmp10 + tmp11) * 4);
        d[4] = (int16_t)((tmp10 - tmp11) * 4);
    } else {
        d[0] = (int16_t)descale(tmp10 + tmp11, 2);
        d[4] = (int16_t)descale(tmp10 - tmp11, 2);
    }
    int64_t z1 = (tmp12 + tmp13) * F0541;
    d[2] = (int16_t)descale(z1 + tmp13 * F0765, sh);
    d[6] = (int16_t)descale(z1 + tmp12 * (-F1847), sh);
    z1 = tmp4 + tmp7;
    int64_t z2 = tmp5 + tmp6, z3 = tmp4 + tmp6, z4 = tmp5 + tmp7;
    const int64_t z5 = (z3 + z4) * F1175;
    const int64_t t4 = tmp4 * F0298, t5 = tmp5 * F2053, t6 = tmp6 * F3072, t7 = tmp7 * F1501;
    z1 *= -F0899; z2 *= -F2562; z3 *= -F1961; z4 *= -F0390;
    z3 += z5; z4 += z5;
    d[7] = (int16_t)descale(t4 + z1 + z3, sh);
    d[5] = (int16_t)descale(t5 + z2 + z4, sh);
    d[3] = (int16_t)descale(t6 + z2 + z3, sh);
    d[1] = (int16_t)descale(t7 + z1 + z4, sh);
}

// jcdctmgr.c: quantisation by reciprocal multiplication (compute_reciprocal + quantize, 16-bit
// DCTELEM), identical to libjpeg-turbo's C and SIMD paths.  q8 = quantval << 3.
struct QRecip {
    uint16_t recip, corr;
    int16_t shift;           // total right shift of the product
};
__host__ __device__ __forceinline__ QRecip q_recip(uint32_t q8) {
    QRecip r;
    if (q8 == 1) { r.recip = 1; r.corr = 0; r.shift = 0; return r; }
    int b = 0;
    while ((1u << (b + 1)) <= q8) ++b;             // floor(log2(q8))
    int rr = 16 + b;
    uint32_t fq = (uint32_t)((1ull << rr) / q8), fr = (uint32_t)((1ull << rr) % q8);
    uint32_t c = q8 / 2;
    if (fr == 0) { fq >>= 1; --rr; }
    else if (fr <= q8 / 2u) ++c;
    else ++fq;
    r.recip = (uint16_t)fq;
    r.corr = (uint16_t)c;
    r.shift = (int16_t)rr;
    return r;
}
__host__ __device__ __forceinline__ int quantize(int v, QRecip q) {
    const uint32_t a = (uint32_t)(v < 0 ? -v : v);
    const uint32_t p = ((a + q.corr) & 0xFFFF) * (uint32_t)q.recip;   // UDCTELEM2 product
    const int r = (int)(p >> q.shift);
    return v < 0 ? -r : r;
}

__host__ __device__ __forceinline__ int imin(int a, int b) { return a < b ? a : b; }

// Encoder geometry: 3 components, 4:2:0 (libjpeg's default for YCbCr), MCU = Y0 Y1 Y2 Y3 Cb Cr.
struct EncGeom {
    int32_t h, w, mcus_x, mcus_y;
    int32_t ybw, ybh;            // luma blocks holding image data: ceil(w / 8), ceil(h / 8)
    int64_t pitch;               // image row pitch in bytes (BGR rows)
};
__host__ __device__ __forceinline__ EncGeom enc_geom(int h, int w, int64_t pitch) {
    EncGeom G;
    G.h = h; G.w = w; G.pitch = pitch;
    G.mcus_x = (w + 15) / 16; G.mcus_y = (h + 15) / 16;
    G.ybw = (w + 7) / 8; G.ybh = (h + 7) / 8;
    return G;
}

// Level-shifted samples of row r of one block (MCU order index blk), 8 values: the
// pre-processing chain of jcprepct.c / jcsample.c -- colour conversion, right-edge and
// bottom-edge replication, h2v2 downsampling with the 1,2,1,2 bias -- for a real block.
__host__ __device__ __forceinline__ void enc_sample_row(const uint8_t *img, const EncGeom &G, int blk, int r,
                                                        int32_t *s8) {
    const int m = blk / 6, b = blk - 6 * (blk / 6);
    const int mx = m % G.mcus_x, my = m / G.mcus_x;
    if (b < 4) {
        const int bx = 2 * mx + (b & 1), by = 2 * my + (b >> 1);
        const uint8_t *row = img + (int64_t)imin(by * 8 + r, G.h - 1) * G.pitch;
        for (int c = 0; c < 8; ++c) {
            const uint8_t *p = row + 3 * imin(bx * 8 + c, G.w - 1);
            int Y, cb, cr;
            rgb_to_ycc(p[2], p[1], p[0], Y, cb, cr);
            s8[c] = Y - 128;
        }
        return;
    }
    const int hc = (G.h + 1) / 2;          // chroma rows holding data
    const int cy = imin(my * 8 + r, hc - 1);
    const uint8_t *r0 = img + (int64_t)(2 * cy) * G.pitch;
    const uint8_t *r1 = img + (int64_t)imin(2 * cy + 1, G.h - 1) * G.pitch;
    for (int c = 0; c < 8; ++c) {
        const int cx = mx * 8 + c;
        const int x0 = 3 * imin(2 * cx, G.w - 1), x1 = 3 * imin(2 * cx + 1, G.w - 1);
        int Y, cb0, cr0, cb1, cr1, cb2, cr2, cb3, cr3;
        rgb_to_ycc(r0[x0 + 2], r0[x0 + 1], r0[x0], Y, cb0, cr0);
        rgb_to_ycc(r0[x1 + 2], r0[x1 + 1], r0[x1], Y, cb1, cr1);
        rgb_to_ycc(r1[x0 + 2], r1[x0 + 1], r1[x0], Y, cb2, cr2);
        rgb_to_ycc(r1[x1 + 2], r1[x1 + 1], r1[x1], Y, cb3, cr3);
        const int bias = (cx & 1) ? 2 : 1;
        const int v = b == 4 ? (cb0 + cb1 + cb2 + cb3 + bias) >> 2 : (cr0 + cr1 + cr2 + cr3 + bias) >> 2;
        s8[c] = v - 128;
    }
}
__host__ __device__ __forceinline__ void enc_samples(const uint8_t *img, const EncGeom &G, int blk, int32_t *s) {
    for (int r = 0; r < 8; ++r) enc_sample_row(img, G, blk, r, s + 8 * r);
}

// Forward DCT (rows, then columns) and quantisation of 64 level-shifted samples -> coef
// (natural order).  q: reciprocals of the component's table.
__host__ __device__ __forceinline__ void enc_transform(int32_t *s, const QRecip *q, int16_t *coef) {
    for (int r = 0; r < 8; ++r) fdct8(s + r * 8, 1);
    for (int c = 0; c < 8; ++c) {
        int32_t col[8];
        for (int r = 0; r < 8; ++r) col[r] = s[r * 8 + c];
        fdct8(col, 2);
        for (int r = 0; r < 8; ++r) s[r * 8 + c] = col[r];
    }
    for (int i = 0; i < 64; ++i) coef[i] = (int16_t)quantize(s[i], q[i]);
}

// jccoefct.c compress_data dummy blocks: a luma block outside the image's block grid has
// zero AC and the DC of the block it copies -- the left neighbour (right edge) or the MCU's
// block 1 (bottom edge, which may itself copy block 0).  Returns the MCU-order index of the
// real block whose DC it takes, or -1 for a real block.
__host__ __device__ __forceinline__ int enc_dummy_source(const EncGeom &G, int blk) {
    const int m = blk / 6, b = blk - 6 * (blk / 6);
    if (b >= 4) return -1;
    const int mx = m % G.mcus_x, my = m / G.mcus_x;
    const int bx = 2 * mx + (b & 1), by = 2 * my + (b >> 1);
    if (bx < G.ybw && by < G.ybh) return -1;
    if (by >= G.ybh) return 6 * m + ((2 * mx + 1) < G.ybw ? 1 : 0);
    return blk - 1;
}

// MCU-order index of the previous block of the same component (DC predictor), -1 at the start.
__host__ __device__ __forceinline__ int enc_prev_same(int blk) {
    const int m = blk / 6, b = blk - 6 * (blk / 6);
    if (b >= 1 && b <= 3) return blk - 1;
    if (m == 0) return -1;
    return b == 0 ? blk - 3 : blk - 6;
}

// Huffman encode tables (jchuff.c jpeg_make_c_derived_tbl): code and length per symbol.
struct HuffEnc {
    uint16_t code[256];
    uint8_t len[256];
};

// Bit count of |v| (jchuff.c: nbits of the magnitude).
__host__ __device__ __forceinline__ int nbits_of(int v) {
    uint32_t a = (uint32_t)(v < 0 ? -v : v);
    int n = 0;
    while (a) { ++n; a >>= 1; }
    return n;
}

// One block's Huffman bits (jchuff.c encode_one_block): calls put(code, len) in stream order.
// blk: quantised coefficients in natural order; nat: zig-zag -> natural.
template <class Put>
__host__ __device__ __forceinline__ void encode_block(const int16_t *blk, int dc_diff, const HuffEnc *dct,
                                                      const HuffEnc *act, const uint8_t *nat, Put &put) {
    int t2 = dc_diff < 0 ? dc_diff - 1 : dc_diff;
    int nb = nbits_of(dc_diff);
    put(dct->code[nb], dct->len[nb]);
    if (nb) put((uint32_t)t2 & ((1u << nb) - 1), nb);
    int r = 0;
    for (int k = 1; k < 64; ++k) {
        const int v = blk[nat[k]];
        if (v == 0) { ++r; continue; }
        while (r > 15) { put(act->code[0xF0], act->len[0xF0]); r -= 16; }
        nb = nbits_of(v);
        const int sym = (r << 4) + nb;
        put(act->code[sym], act->len[sym]);
        put((uint32_t)(v < 0 ? v - 1 : v) & ((1u << nb) - 1), nb);
        r = 0;
    }
    if (r > 0) put(act->code[0], act->len[0]);
}

// ---------------------------------------------------------------------------------------------
// Host side: marker parsing (jdmarker.c restated for the markers a baseline file carries) and
// the decode-form tables.
struct Parsed {
    int h = 0, w = 0, ncomp = 0, restart = 0, sof = 0;
    int comp_id[kMaxComp] = {0}, comp_h[kMaxComp] = {0}, comp_v[kMaxComp] = {0}, comp_q[kMaxComp] = {0};
    int comp_dc[kMaxComp] = {0}, comp_ac[kMaxComp] = {0};
    uint16_t qt[4][64];            // natural order
    bool qt_ok[4] = {false, false, false, false};
    uint8_t hbits[2][4][17];       // [class][id][length 1..16]
    uint8_t hvals[2][4][256];
    bool h_ok[2][4] = {{false, false, false, false}, {false, false, false, false}};
    const uint8_t *ecs = nullptr;  // entropy-coded segment (stuffed bytes)
    size_t ecs_len = 0;
};

// Standard tables of JPEG Annex K.3 (libjpeg uses them when a file has no DHT).
void std_huff(int cls, int id, uint8_t *bits17, uint8_t *vals256);
// Returns 0 or a PANO_E_* code; *err gets a message.
int parse(const uint8_t *buf, size_t len, Parsed *out, std::string *err);
// Builds the decode form of a (bits, vals) table of class cls (0 DC, 1 AC): PANO_OK, PANO_E_ARG
// (invalid code lengths) or PANO_E_UNSUPPORTED (long codes spread over more than kHuffSub 9-bit
// prefixes).
int make_huff(int cls, const uint8_t *bits17, const uint8_t *vals, Huff *out);
// Frame geometry (MCU layout, component planes, upsampling mode) of a parsed file; the
// arena offsets and table indices are filled in by the caller.
int plan_frame(const Parsed &P, Frame *F, std::string *err);
// Encoder side: jcparam.c jpeg_set_quality tables (natural order) and the Annex K encode
// tables; the file header libjpeg-turbo writes for a 3-component 4:2:0 baseline image
// (SOI, JFIF APP0 1.01, DQT x2, SOF0, DHT x4, SOS), as PIL's save(quality=q) does.
void quant_tables(int quality, uint16_t *lum64, uint16_t *chr64);
void std_huff_enc(int cls, int id, HuffEnc *out);
std::vector<uint8_t> encode_header(int h, int w, const uint16_t *lum64, const uint16_t *chr64);

}  // namespace pj
