// jpeg.hip -- baseline JPEG decode on the GPU: the reference's
// cv2.imread of every frame (image_stitching_sift.py:282, image_stitching_harris.py:394),
// bit-identical to libjpeg-turbo's default decode (what cv2.imread and PIL run).
//
// A batch of files is decoded by ten launches, all frames at once:
//   jpeg_unstuff_count / jpeg_unstuff_write  remove the 0x00 stuffed after 0xFF bytes of the
//        entropy-coded segments (a chunked stream compaction);
//   jpeg_sync_warm   the Huffman stream has no restart markers, so it is cut into subsequences
//        of kSubBits bits and the decoder state at each subsequence start is found by
//        self-synchronisation: one thread per (chain of kChain subsequences, MCU-phase
//        hypothesis) decodes a warm-up window before its chain from a guessed state, which
//        converges on the true codeword boundaries, then walks its subsequences with counting,
//        recording at each one's start a candidate state and its exit state, blocks started
//        and DC difference sums;
//   jpeg_sync_fix    where an exit of subsequence t-1 matches none of t's candidates, t is
//        decoded from that exit as an extra candidate (all such (t, exit) pairs in parallel);
//   jpeg_sync_fix2   the same once more from the extra candidates' exits (one more slot per
//        subsequence): a region where every warm chain failed is bridged in two rounds;
//   jpeg_sync_resolve  one workgroup per frame chains the candidates: the true start of
//        subsequence t is the exit of t-1's chosen candidate, found by a composition scan of
//        the per-subsequence candidate maps; a subsequence whose candidates all missed is
//        decoded again from the true start (rare, in the same kernel).  The same pass emits
//        the exclusive prefix of the statistics: first block index and DC predictors;
//   jpeg_write       one thread per subsequence decodes its range from the true start and
//        writes coefficients in natural order with the DC predicted;
//   jpeg_idct        islow inverse DCT per 8x8 block into the component sample planes;
//   jpeg_color       fancy chroma upsampling + YCbCr -> BGR, u8 [n][h][w][3].
// Every walk reads its bits from a window of the stream staged in LDS, and its Huffman tables
// from LDS (two-level lookup, jpeg_core.h).  The host parses headers only (jpeg_host.cpp) and
// uploads tables + entropy bytes once.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "jpeg_core.h"
#include "pano_internal.h"

using namespace pj;

namespace {

struct Dev {
    const Frame *frames;
    const Huff *tabs;
    const uint16_t *quant;      // [Q][64] natural order
    const uint32_t *chunk_frame;
    const uint8_t *src;
    uint8_t *stream;
    int16_t *coef;
    uint8_t *samp;
    uint32_t *chunk_cnt;
    uint32_t *nbits;
    int32_t *flags;
    int32_t *stats;             // [n][4]: subsequences, fix candidates, serial decodes, 0
    int32_t *status;            // caller's, may be null
    uint64_t *cand;             // [S][nps]: warm slots [0, np), fix slots [np, 2 np), fix2 slot 2 np
    uint64_t *cexit;            // [S][nps]
    SubStats *cstats;           // [S][nps]
    uint64_t *start;            // [S]
    SubStats *scan;             // [S] exclusive prefix
    uint64_t *maps;             // [S] candidate map of subsequence t >= 1: slot of t-1 -> slot of t
    int n, np, nps;             // candidate slots: np phases (max bpm), nps = 2 np + 1
    int chain;                  // subsequences per warm chain (<= kChain)
};

constexpr uint64_t kNoCand = ~0ull;
constexpr int kMargin = 8;      // words staged past a window's last bit (the 32-bit peek of its last code)

// ---------------------------------------------------------------------------------------- LDS
// A frame's decode tables in LDS: DC / AC per component + the MCU layout.
struct LdsTabs {
    Huff T[2 * kMaxComp];       // DC tables of components 0..2, then their AC tables
    int8_t mcu_comp[kMaxBpm];
    uint8_t nat[80];
};

__device__ __forceinline__ void stage_tabs(const Dev &D, const Frame &F, LdsTabs &L) {
    const int nt = blockDim.x;
    constexpr int HW = sizeof(Huff) / 4;
    for (int c = 0; c < F.ncomp; ++c) {
        const uint32_t *sd = (const uint32_t *)&D.tabs[F.dc_tab[c]];
        const uint32_t *sa = (const uint32_t *)&D.tabs[F.ac_tab[c]];
        uint32_t *dd = (uint32_t *)&L.T[c], *da = (uint32_t *)&L.T[kMaxComp + c];
        for (int i = threadIdx.x; i < HW; i += nt) {
            dd[i] = sd[i];
            da[i] = sa[i];
        }
    }
    if (threadIdx.x < kMaxBpm) L.mcu_comp[threadIdx.x] = F.mcu_comp[threadIdx.x];
    if (threadIdx.x < 80) L.nat[threadIdx.x] = (uint8_t)natural_order(threadIdx.x);
}

__device__ __forceinline__ uint32_t frame_nsub(const Frame &F, uint32_t nb) {
    const uint32_t s = (nb + kSubBits - 1) / kSubBits;
    return s < F.nsub ? s : F.nsub;
}

__device__ __forceinline__ uint32_t stream_words(const Frame &F, uint32_t nb) {
    return (nb / 8 + kStreamPad) / 4;
}

// Stage stream words [w0, w0 + n) of a frame into LDS in stream order (first byte in the top
// bits); words past the frame's stream read as zero.
__device__ __forceinline__ void stage_window(const Dev &D, const Frame &F, uint32_t nb, uint32_t w0, uint32_t n,
                                             uint32_t *win) {
    const uint32_t *src = (const uint32_t *)(D.stream + F.bits_off);
    const uint32_t nw = stream_words(F, nb);
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t j = w0 + i;
        win[i] = j < nw ? __builtin_bswap32(src[j]) : 0u;
    }
}

// 256-thread block exclusive scan of a u32 (4 waves of 64).
__device__ __forceinline__ uint32_t block_exscan256(uint32_t v, uint32_t *wsum, uint32_t *total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    uint32_t base = 0;
    for (int i = 0; i < wv; ++i) base += wsum[i];
    *total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
    return base + x - v;
}

// ---------------------------------------------------------------------------------- unstuff
__global__ void __launch_bounds__(256) jpeg_unstuff_count(Dev D) {
    __shared__ uint32_t wsum[4];
    const uint32_t c = blockIdx.x;
    const uint32_t f = D.chunk_frame[c];
    const Frame &F = D.frames[f];
    const uint32_t b0 = (c - F.chunk0) * kChunk + threadIdx.x * 16;
    const uint8_t *src = D.src + F.src_off;
    uint32_t cnt = 0, mk = 0;
    if (b0 < F.src_len) {
        const uint4 q = *(const uint4 *)(src + b0);   // the upload pads every segment by 16
        const uint8_t *by = (const uint8_t *)&q;
        uint32_t prev = b0 ? src[b0 - 1] : 0;
        const uint32_t m = F.src_len - b0 < 16 ? F.src_len - b0 : 16;
        for (uint32_t i = 0; i < m; ++i) {
            const uint32_t b = by[i];
            const bool ff = prev == 0xFF;
            cnt += !(ff && b == 0);
            mk |= ff && b != 0;
            prev = b;
        }
    }
    uint32_t total;
    (void)block_exscan256(cnt, wsum, &total);
    if (threadIdx.x == 0) D.chunk_cnt[c] = total;
    if (mk) atomicOr(&D.flags[f], 1);
}

__global__ void __launch_bounds__(256) jpeg_unstuff_write(Dev D) {
    __shared__ uint32_t wsum[4];
    __shared__ uint32_t red[256];
    const uint32_t c = blockIdx.x;
    const uint32_t f = D.chunk_frame[c];
    const Frame &F = D.frames[f];
    // prefix of kept bytes over the frame's earlier chunks
    uint32_t p = 0;
    for (uint32_t i = F.chunk0 + threadIdx.x; i < c; i += 256) p += D.chunk_cnt[i];
    red[threadIdx.x] = p;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    const uint32_t prefix = red[0];
    const uint32_t b0 = (c - F.chunk0) * kChunk + threadIdx.x * 16;
    const uint8_t *src = D.src + F.src_off;
    uint8_t keep[16];
    uint32_t cnt = 0, m = 0;
    if (b0 < F.src_len) {
        const uint4 q = *(const uint4 *)(src + b0);
        const uint8_t *by = (const uint8_t *)&q;
        uint32_t prev = b0 ? src[b0 - 1] : 0;
        m = F.src_len - b0 < 16 ? F.src_len - b0 : 16;
        for (uint32_t i = 0; i < 16; ++i) {
            const uint32_t b = by[i];
            if (i < m && !(prev == 0xFF && b == 0)) keep[cnt++] = (uint8_t)b;
            prev = b;
        }
    }
    uint32_t total;
    const uint32_t off = block_exscan256(cnt, wsum, &total);
    uint8_t *dst = D.stream + F.bits_off;
    for (uint32_t i = 0; i < cnt; ++i) dst[prefix + off + i] = keep[i];
    if (c == F.chunk0 + F.nchunk - 1) {
        const uint32_t end = prefix + total;
        if (threadIdx.x == 0) D.nbits[f] = end * 8;
        if (threadIdx.x < kStreamPad) dst[end + threadIdx.x] = 0;
    }
}

// ------------------------------------------------------------------------------------ sync
// Launch shapes: warm runs kSyncThreads threads = chains x np phase slots (the tail threads
// idle), at most kChainsPerBlock chains; fix runs kSyncThreads = subsequences x np slots.  The
// window is every bit those walks can reach.
constexpr int kWarmMax = 16384;                     // cap of Frame::warm (bits)
constexpr int kSyncThreads = 256;
constexpr int kChain = 4;                           // subsequences per warm chain
constexpr int kChainsPerBlock = 42;
constexpr int kWinWords = (kWarmMax + kChainsPerBlock * kChain * kSubBits) / 32 + 2 * kMargin;
__host__ __device__ __forceinline__ int chains_per_block(int np) {
    return kSyncThreads / np < kChainsPerBlock ? kSyncThreads / np : kChainsPerBlock;
}

__global__ void __launch_bounds__(kSyncThreads) jpeg_sync_warm(Dev D) {
    __shared__ LdsTabs L;
    __shared__ uint32_t win[kWinWords];
    const int f = blockIdx.y;
    const Frame &F = D.frames[f];
    const uint32_t nb = D.nbits[f];
    const uint32_t nsub = frame_nsub(F, nb);
    const int np = D.np, cpb = chains_per_block(np);
    const int G = D.chain;
    const uint32_t t0 = blockIdx.x * cpb * G;        // first subsequence of the block
    if (t0 >= nsub) return;                          // whole block past the frame's stream
    const uint32_t W = F.warm;
    const uint32_t b0 = t0 * kSubBits > W ? t0 * kSubBits - W : 0;      // first bit any walk reads
    const uint32_t w0 = b0 >> 5;
    const uint32_t b1 = (t0 + cpb * G) * kSubBits;
    const uint32_t nwin = (b1 >> 5) - w0 + kMargin;
    stage_tabs(D, F, L);
    stage_window(D, F, nb, w0, nwin, win);
    __syncthreads();
    const int ch = threadIdx.x / np, j = threadIdx.x % np;
    const uint32_t ta = t0 + ch * G;                 // the chain's first subsequence
    if (ch >= cpb || ta >= nsub) return;
    if (j >= F.bpm) {                                // phase slot this frame's MCU lacks
        for (uint32_t t = ta; t < ta + G && t < nsub; ++t) D.cand[(size_t)(F.sub0 + t) * D.nps + j] = kNoCand;
        return;
    }
    const uint32_t p0 = ta * kSubBits;
    SinkNone sn;
    uint64_t st = p0 <= W ? walk(win, w0, nwin, pack_state(0, 0, 0), p0, L.T, L.mcu_comp, F.bpm, sn)
                          : walk(win, w0, nwin, pack_state(p0 - W, j, 0), p0, L.T, L.mcu_comp, F.bpm, sn);
    for (uint32_t t = ta; t < ta + G && t < nsub; ++t) {
        const uint32_t end = (t + 1) * kSubBits < nb ? (t + 1) * kSubBits : nb;
        SinkCount sc;
        const uint64_t x = walk(win, w0, nwin, st, end, L.T, L.mcu_comp, F.bpm, sc);
        const size_t q = (size_t)(F.sub0 + t) * D.nps + j;
        D.cand[q] = st;
        D.cexit[q] = x;
        D.cstats[q] = sc.stats();
        st = x;
    }
}

// Extra candidates: for subsequence t >= 1 and warm slot i of t-1 whose exit starts none of
// t's warm candidates, t decoded from that exit (slot np + i); else the slot is empty.
__global__ void __launch_bounds__(kSyncThreads) jpeg_sync_fix(Dev D) {
    __shared__ LdsTabs L;
    __shared__ uint32_t win[(kSyncThreads * kSubBits) / 32 + 2 * kMargin];
    __shared__ int any;
    const int f = blockIdx.y;
    const Frame &F = D.frames[f];
    const uint32_t nb = D.nbits[f];
    const uint32_t nsub = frame_nsub(F, nb);
    const int np = D.np, nps = D.nps, spb = kSyncThreads / np;
    const uint32_t t0 = blockIdx.x * spb;
    if (t0 >= nsub) return;
    const uint32_t t = t0 + threadIdx.x / np, i = threadIdx.x % np;   // subsequence, predecessor slot
    bool need = false;
    uint64_t e = kNoCand;
    const bool slot = (int)(threadIdx.x / np) < spb && t < nsub;
    const bool mine = slot && (int)i < F.bpm;
    if (threadIdx.x == 0) any = 0;
    __syncthreads();
    if (mine && t >= 1) {
        const size_t qp = (size_t)(F.sub0 + t - 1) * nps + i, qt = (size_t)(F.sub0 + t) * nps;
        e = D.cexit[qp];
        need = true;
        for (int j = 0; j < F.bpm; ++j) need &= D.cand[qt + j] != e;
        if (need) {
            any = 1;
            atomicAdd(&D.stats[4 * f + 1], 1);
        }
    }
    if (slot) D.cand[(size_t)(F.sub0 + t) * nps + np + i] = kNoCand;
    __syncthreads();
    if (!any) return;                                // uniform: no walk in this block
    const uint32_t w0 = (t0 * kSubBits) >> 5;
    const uint32_t nwin = (uint32_t)(spb * kSubBits) / 32 + kMargin;
    stage_tabs(D, F, L);
    stage_window(D, F, nb, w0, nwin, win);
    __syncthreads();
    if (!need) return;
    const uint32_t p0 = t * kSubBits;
    const uint32_t end = p0 + kSubBits < nb ? p0 + kSubBits : nb;
    SinkCount sc;
    const uint64_t x = walk(win, w0, nwin, e, end, L.T, L.mcu_comp, F.bpm, sc);
    const size_t q = (size_t)(F.sub0 + t) * nps + np + i;
    D.cand[q] = e;
    D.cexit[q] = x;
    D.cstats[q] = sc.stats();
}

// Second round: for subsequence t >= 1 and fix slot np + i of t-1 whose exit starts none of
// t's candidates, t decoded from that exit into slot 2 np (the first such i; the others fall to
// the serial fallback of the resolve).
__global__ void __launch_bounds__(kSyncThreads) jpeg_sync_fix2(Dev D) {
    __shared__ LdsTabs L;
    __shared__ uint32_t win[(kSyncThreads * kSubBits) / 32 + 2 * kMargin];
    __shared__ int pick[kSyncThreads];
    __shared__ int any;
    const int f = blockIdx.y;
    const Frame &F = D.frames[f];
    const uint32_t nb = D.nbits[f];
    const uint32_t nsub = frame_nsub(F, nb);
    const int np = D.np, nps = D.nps, spb = kSyncThreads / np;
    const uint32_t t0 = blockIdx.x * spb;
    if (t0 >= nsub) return;
    const int tl = threadIdx.x / np, i = threadIdx.x % np;
    const uint32_t t = t0 + tl;
    const bool slot = tl < spb && t < nsub;
    const bool mine = slot && i < F.bpm;
    if (threadIdx.x == 0) any = 0;
    pick[threadIdx.x] = np;
    __syncthreads();
    uint64_t e = kNoCand;
    bool need = false;
    if (mine && t >= 1) {
        const size_t qp = (size_t)(F.sub0 + t - 1) * nps + np + i, qt = (size_t)(F.sub0 + t) * nps;
        if (D.cand[qp] != kNoCand) {
            e = D.cexit[qp];
            need = true;
            for (int j = 0; j < 2 * np; ++j) need &= D.cand[qt + j] != e;
            if (need) atomicMin(&pick[tl], i);
        }
    }
    __syncthreads();
    if (slot && i == 0) D.cand[(size_t)(F.sub0 + t) * nps + 2 * np] = kNoCand;
    need = need && pick[tl] == i;
    if (need) any = 1;
    __syncthreads();
    if (!any) return;
    const uint32_t w0 = (t0 * kSubBits) >> 5;
    const uint32_t nwin = (uint32_t)(spb * kSubBits) / 32 + kMargin;
    stage_tabs(D, F, L);
    stage_window(D, F, nb, w0, nwin, win);
    __syncthreads();
    if (!need) return;
    atomicAdd(&D.stats[4 * f + 1], 1);
    const uint32_t end = (t + 1) * kSubBits < nb ? (t + 1) * kSubBits : nb;
    SinkCount sc;
    const uint64_t x = walk(win, w0, nwin, e, end, L.T, L.mcu_comp, F.bpm, sc);
    const size_t q = (size_t)(F.sub0 + t) * nps + 2 * np;
    D.cand[q] = e;
    D.cexit[q] = x;
    D.cstats[q] = sc.stats();
}

// Candidate map of subsequence t: for each slot i of t-1, the first slot of t whose start
// equals i's exit (15 = none), 4 bits per entry (nps <= 13).
constexpr uint64_t kNone = 15;
__device__ __forceinline__ uint64_t map_get(uint64_t m, int i) { return (m >> (4 * i)) & 15; }
// (second after first): entry i -> second[first[i]]
__device__ __forceinline__ uint64_t map_then(uint64_t first, uint64_t second, int nps) {
    uint64_t r = 0;
    for (int i = 0; i < nps; ++i) {
        const uint64_t a = map_get(first, i);
        r |= (a == kNone ? kNone : map_get(second, (int)a)) << (4 * i);
    }
    return r;
}
__device__ __forceinline__ uint64_t map_const(uint64_t v, int nps) {
    uint64_t r = 0;
    for (int i = 0; i < nps; ++i) r |= v << (4 * i);
    return r;
}
// first slot of t (candidates ct[0..nps)) starting at e
__device__ __forceinline__ uint64_t find_slot(const uint64_t *ct, int nps, uint64_t e) {
    uint64_t jj = kNone;
    if (e == kNoCand) return jj;
    for (int j = nps - 1; j >= 0; --j) if (ct[j] == e) jj = (uint64_t)j;
    return jj;
}

// The candidate map of every subsequence t >= 1 of every frame, all in parallel (one thread
// per subsequence): entry i is the slot of t that slot i of t-1 exits into (kNone if none).
// jpeg_sync_resolve composes them per frame.  The candidate and exit records are loaded up
// front (kMapSlots at a time, predicated) so their loads are in flight together.
constexpr int kMapSlots = 2 * 6 + 1;    // nps at 6 blocks per MCU (4:2:0), the most the parser accepts
__global__ void __launch_bounds__(256) jpeg_sync_maps(Dev D) {
    const int f = blockIdx.y;
    const Frame &F = D.frames[f];
    const uint32_t nsub = frame_nsub(F, D.nbits[f]);
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t == 0 || t >= nsub) return;
    const int nps = D.nps;
    const size_t S = F.sub0 + t;
    uint64_t ct[kMapSlots], xp[kMapSlots], cp[kMapSlots];
#pragma unroll
    for (int i = 0; i < kMapSlots; ++i) {
        const bool in = i < nps;
        ct[i] = in ? D.cand[S * nps + i] : kNoCand;
        xp[i] = in ? D.cexit[(S - 1) * nps + i] : kNoCand;
        cp[i] = in ? D.cand[(S - 1) * nps + i] : kNoCand;
    }
    uint64_t m = 0;
#pragma unroll
    for (int i = 0; i < kMapSlots; ++i) {
        uint64_t jj = kNone;
        if (cp[i] != kNoCand && xp[i] != kNoCand) {
#pragma unroll
            for (int j = kMapSlots - 1; j >= 0; --j)
                if (j < nps && ct[j] == xp[i]) jj = (uint64_t)j;
        }
        if (i < nps) m |= jj << (4 * i);
    }
    D.maps[S] = m;
}

constexpr int kResolveThreads = 512;
constexpr int kFixRun = 16;      // subsequences one serial fallback may decode in a row

__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t *wsum, uint32_t *total) {
    // kResolveThreads-thread exclusive scan (waves of 64)
    constexpr int NW = kResolveThreads / 64;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wv] = x;
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

__global__ void __launch_bounds__(kResolveThreads) jpeg_sync_resolve(Dev D) {
    __shared__ LdsTabs L;
    __shared__ uint64_t maps[kResolveThreads];
    __shared__ uint32_t wsum[kResolveThreads / 64];
    __shared__ uint32_t win[kFixRun * kSubBits / 32 + 2 * kMargin];
    __shared__ int s_fail;
    __shared__ uint32_t s_next;
    __shared__ uint64_t s_exit;
    __shared__ SubStats s_acc;
    constexpr int NT = kResolveThreads;
    const int f = blockIdx.x;
    const Frame &F = D.frames[f];
    stage_tabs(D, F, L);
    const uint32_t nb = D.nbits[f];
    const uint32_t nsub = frame_nsub(F, nb);
    const int nps = D.nps;
    const size_t S0 = F.sub0;
    if (threadIdx.x == 0 && nsub > 0) {
        // subsequence 0 decodes from the exact start: every warm candidate is the same
        D.start[S0] = D.cand[S0 * nps];
        SubStats z = {0, {0, 0, 0}};
        D.scan[S0] = z;
        s_acc = D.cstats[S0 * nps];
        s_exit = D.cexit[S0 * nps];
    }
    __syncthreads();
    uint32_t base = 1;
    uint32_t guard = nsub + 8;
    while (base < nsub && guard--) {
        const uint32_t t = base + threadIdx.x;
        const bool in = t < nsub;
        // map of t: from the known exit (t == base) or from t-1's slots
        uint64_t m = map_const(kNone, nps);
        if (in) {
            const uint64_t *ct = D.cand + (S0 + t) * nps;
            if (threadIdx.x == 0) m = map_const(find_slot(ct, nps, s_exit), nps);
            else m = D.maps[S0 + t];                       // jpeg_sync_maps
        }
        maps[threadIdx.x] = m;
        if (threadIdx.x == 0) s_fail = NT;
        __syncthreads();
        // inclusive scan by composition: maps[t] = M_t after ... after M_base
        for (int o = 1; o < NT; o <<= 1) {
            uint64_t prev = 0;
            if ((int)threadIdx.x >= o) prev = maps[threadIdx.x - o];
            __syncthreads();
            if ((int)threadIdx.x >= o) maps[threadIdx.x] = map_then(prev, maps[threadIdx.x], nps);
            __syncthreads();
        }
        // chosen slot of t (the composed map is constant: its first map is)
        const uint32_t J = (uint32_t)map_get(maps[threadIdx.x], 0);
        if (in && J == kNone) atomicMin(&s_fail, (int)threadIdx.x);
        __syncthreads();
        const int nres = min(s_fail, (int)min((uint32_t)NT, nsub - base));   // resolved in this chunk
        SubStats st = {0, {0, 0, 0}};
        if ((int)threadIdx.x < nres) st = D.cstats[(S0 + t) * nps + J];
        // exclusive prefix of the statistics over the resolved run
        uint32_t tb;
        const uint32_t pb = block_exscan((uint32_t)st.blocks, wsum, &tb);
        uint32_t pd[kMaxComp], td[kMaxComp];
        for (int c = 0; c < kMaxComp; ++c) pd[c] = block_exscan((uint32_t)st.dc[c], wsum, &td[c]);
        if ((int)threadIdx.x < nres) {
            D.start[S0 + t] = D.cand[(S0 + t) * nps + J];
            SubStats sc;
            sc.blocks = s_acc.blocks + (int32_t)pb;
            for (int c = 0; c < kMaxComp; ++c) sc.dc[c] = s_acc.dc[c] + (int32_t)pd[c];
            D.scan[S0 + t] = sc;
            if ((int)threadIdx.x == nres - 1) s_exit = D.cexit[(S0 + t) * nps + J];
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            s_acc.blocks += (int32_t)tb;
            for (int c = 0; c < kMaxComp; ++c) s_acc.dc[c] += (int32_t)td[c];
        }
        base += nres;
        __syncthreads();
        if (nres < NT && base < nsub) {
            // every candidate of `base` missed: decode it from the true start (one thread), and
            // its successors while their candidates miss too (a run of such subsequences is
            // typical: the warm chains of one region failed together)
            const uint32_t w0 = (base * kSubBits) >> 5, nwin = (kFixRun * kSubBits) / 32 + kMargin;
            stage_window(D, F, nb, w0, nwin, win);
            __syncthreads();
            if (threadIdx.x == 0) {
                uint64_t e = s_exit;
                uint32_t t = base;
                for (int r = 0; r < kFixRun && t < nsub; ++r) {
                    const uint32_t end = (t + 1) * kSubBits < nb ? (t + 1) * kSubBits : nb;
                    SinkCount sc;
                    const uint64_t x = walk(win, w0, nwin, e, end, L.T, L.mcu_comp, F.bpm, sc);
                    D.start[S0 + t] = e;
                    D.scan[S0 + t] = s_acc;
                    s_acc.blocks += sc.blocks;
                    s_acc.dc[0] += sc.d0;
                    s_acc.dc[1] += sc.d1;
                    s_acc.dc[2] += sc.d2;
                    D.stats[4 * f + 2] += 1;
                    e = x;
                    ++t;
                    if (t >= nsub || find_slot(D.cand + (S0 + t) * nps, nps, x) != kNone) break;
                }
                s_exit = e;
                s_next = t;
            }
            __syncthreads();
            base = s_next;
            __syncthreads();
        }
    }
    if (threadIdx.x == 0) {
        int st = PANO_OK;
        if (D.flags[f] & 1) st = PANO_E_UNSUPPORTED;            // a marker inside the scan
        else if (s_acc.blocks < F.total_blocks || nsub == 0) st = PANO_E_ARG;   // truncated
        D.flags[f] = st;
        D.stats[4 * f] = (int32_t)nsub;
        if (D.status) D.status[f] = st;
    }
}

// ----------------------------------------------------------------------------------- write
constexpr int kWriteThreads = 128;
__global__ void __launch_bounds__(kWriteThreads) jpeg_write(Dev D) {
    __shared__ LdsTabs L;
    __shared__ Frame Fs;
    __shared__ uint32_t win[(kWriteThreads * kSubBits) / 32 + 2 * kMargin];
    const int f = blockIdx.y;
    const Frame &F = D.frames[f];
    const uint32_t nb = D.nbits[f];
    const uint32_t nsub = frame_nsub(F, nb);
    const uint32_t t0 = blockIdx.x * kWriteThreads;
    if (t0 >= nsub || D.flags[f] != PANO_OK) return;
    const uint32_t w0 = (t0 * kSubBits) >> 5;
    const uint32_t nwin = (uint32_t)(kWriteThreads * kSubBits) / 32 + kMargin;
    stage_tabs(D, F, L);
    stage_window(D, F, nb, w0, nwin, win);
    for (int i = threadIdx.x; i < (int)(sizeof(Frame) / 4); i += kWriteThreads)
        ((uint32_t *)&Fs)[i] = ((const uint32_t *)&F)[i];
    __syncthreads();
    const uint32_t t = t0 + threadIdx.x;
    if (t >= nsub) return;
    const uint64_t s0 = D.start[F.sub0 + t];
    const SubStats sc = D.scan[F.sub0 + t];
    SinkWrite w;
    w.coef = D.coef;
    w.F = &Fs;
    w.nat = L.nat;
    const int k0 = state_k(s0);
    const int32_t b0 = sc.blocks - (k0 > 0 ? 1 : 0);
    w.seek(b0 > 0 ? b0 : 0);
    w.blk = b0;
    w.p0 = sc.dc[0];
    w.p1 = sc.dc[1];
    w.p2 = sc.dc[2];
    w.live = k0 > 0 && b0 >= 0 && b0 < Fs.total_blocks;
    w.addr = w.live ? w.address() : 0;
    const uint32_t end = (t + 1) * kSubBits < nb ? (t + 1) * kSubBits : nb;
    walk(win, w0, nwin, s0, end, L.T, L.mcu_comp, Fs.bpm, w);
}

// ------------------------------------------------------------------------------------ IDCT
// 32 blocks per workgroup, 8 threads per block: column pass (thread = column), row pass
// (thread = row, 8 bytes out).
__global__ void __launch_bounds__(256) jpeg_idct(Dev D) {
    __shared__ __align__(16) int16_t cf[32][64];
    __shared__ int32_t ws[32][65];
    __shared__ uint16_t q[64];
    const int f = blockIdx.y / kMaxComp, c = blockIdx.y % kMaxComp;
    const Frame &F = D.frames[f];
    if (c >= F.ncomp || D.flags[f] != PANO_OK) return;
    const int bw = F.comp_bw[c], nblk = bw * F.comp_bh[c];
    if (threadIdx.x < 64) q[threadIdx.x] = D.quant[(size_t)F.q_tab[c] * 64 + threadIdx.x];
    const int lb = threadIdx.x >> 3, r = threadIdx.x & 7;
    const int blk = blockIdx.x * 32 + lb;
    const bool live = blk < nblk;
    const int16_t *src = D.coef + F.coef_off[c] + (size_t)blk * 64;
    if (live) *(uint4 *)&cf[lb][r * 8] = *(const uint4 *)(src + r * 8);
    __syncthreads();
    if (live) idct_col(cf[lb], q, r, ws[lb]);
    __syncthreads();
    if (live) {
        union { uint8_t b[8]; uint2 v; } o;
        idct_row(ws[lb], r, o.b);
        const int bx = blk % bw, by = blk / bw;
        uint8_t *dst = D.samp + F.samp_off[c] + (size_t)(by * 8 + r) * (bw * 8) + bx * 8;
        *(uint2 *)dst = o.v;
    }
}

// ----------------------------------------------------------------------------------- colour
// One thread per output pixel, grid (pixel blocks, frame).
__global__ void __launch_bounds__(256) jpeg_color(Dev D, uint8_t *out, int h, int w) {
    const int f = blockIdx.y;
    const Frame &F = D.frames[f];
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= (uint32_t)(h * w)) return;
    const int y = i / w, x = i - y * w;
    uint8_t *o = out + ((size_t)f * h * w + i) * 3;
    if (D.flags[f] != PANO_OK) {
        o[0] = o[1] = o[2] = 0;
        return;
    }
    const uint8_t *py = D.samp + F.samp_off[0];
    const int Y = py[(size_t)y * F.comp_bw[0] * 8 + x];
    if (F.ncomp == 1) {
        o[0] = o[1] = o[2] = (uint8_t)Y;
        return;
    }
    const int cb = chroma_at(D.samp + F.samp_off[1], F.comp_bw[1] * 8, F.comp_dw[1], F.comp_dh[1], F.upsample, x, y);
    const int cr = chroma_at(D.samp + F.samp_off[2], F.comp_bw[2] * 8, F.comp_dw[2], F.comp_dh[2], F.upsample, x, y);
    uint8_t bgr[3];
    ycc_to_bgr(Y, cb, cr, bgr);
    o[0] = bgr[0];
    o[1] = bgr[1];
    o[2] = bgr[2];
}

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

}  // namespace

int jpeg_last_stats(pano_ctx *ctx, int32_t *h, int n) {
    if (!ctx->jstats || n > ctx->jstats_n) return pano_fail(ctx, PANO_E_ARG, "no JPEG decode with that many frames");
    PANO_HIP(ctx, hipStreamSynchronize(ctx->stream));
    PANO_HIP(ctx, hipMemcpy(h, ctx->jstats, 16 * (size_t)n, hipMemcpyDeviceToHost));
    return PANO_OK;
}

// PANO_JPEG_HOST_TIMING=1 (diagnostics): host microseconds of the call's phases on stderr
struct HostClock {
    bool on = false;
    std::chrono::steady_clock::time_point t0;
    HostClock() {
        const char *e = getenv("PANO_JPEG_HOST_TIMING");
        on = e && atoi(e) != 0;
        t0 = std::chrono::steady_clock::now();
    }
    void mark(const char *what) {
        if (!on) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[jpeg host] %s %.1f us\n", what, std::chrono::duration<double, std::micro>(t - t0).count());
        t0 = t;
    }
};

int launch_jpeg_decode(pano_ctx *ctx, int n, const uint8_t *const *bufs, const size_t *lens, uint8_t *bgr,
                       int h, int w, int32_t *status) {
    HostClock hc;
    // ---- host: parse, plan, tables
    std::vector<Parsed> ps((size_t)n);
    std::vector<Frame> fr((size_t)n);
    std::vector<Huff> tabs;
    std::vector<std::vector<uint8_t>> tab_keys;      // (bits, vals) bytes of each table
    std::vector<uint16_t> quant;
    std::vector<uint32_t> chunk_frame;
    for (int f = 0; f < n; ++f) {
        std::string err;
        int rc = parse(bufs[f], lens[f], &ps[f], &err);
        if (!rc) rc = plan_frame(ps[f], &fr[f], &err);
        if (rc) return pano_fail(ctx, rc, "frame " + std::to_string(f) + ": " + err);
        if (ps[f].h != h || ps[f].w != w)
            return pano_fail(ctx, PANO_E_ARG, "frame " + std::to_string(f) + ": size differs from the batch's");
        if (ps[f].ecs_len == 0) return pano_fail(ctx, PANO_E_ARG, "frame " + std::to_string(f) + ": empty scan");
        if (ps[f].ecs_len >= (1u << 28)) return pano_fail(ctx, PANO_E_UNSUPPORTED, "JPEG scan larger than 256 MiB");
        Frame &F = fr[f];
        for (int c = 0; c < F.ncomp; ++c) {
            for (int cls = 0; cls < 2; ++cls) {
                const int id = cls ? ps[f].comp_ac[c] : ps[f].comp_dc[c];
                uint8_t bits[17], vals[256];
                if (ps[f].h_ok[cls][id]) {
                    memcpy(bits, ps[f].hbits[cls][id], 17);
                    memcpy(vals, ps[f].hvals[cls][id], 256);
                } else {
                    std_huff(cls, id, bits, vals);   // libjpeg-turbo's default tables
                }
                std::vector<uint8_t> key(bits, bits + 17);
                key.insert(key.end(), vals, vals + 256);
                int ti = -1;
                for (size_t k = 0; k < tab_keys.size(); ++k)
                    if (tab_keys[k] == key) { ti = (int)k; break; }
                if (ti < 0) {
                    Huff T;
                    const int hr = make_huff(cls, bits, vals, &T);
                    if (hr) return pano_fail(ctx, hr, "frame " + std::to_string(f) + ": unsupported Huffman table");
                    ti = (int)tabs.size();
                    tabs.push_back(T);
                    tab_keys.push_back(key);
                }
                (cls ? F.ac_tab[c] : F.dc_tab[c]) = ti;
            }
            F.q_tab[c] = (int)(quant.size() / 64);
            quant.insert(quant.end(), ps[f].qt[ps[f].comp_q[c]], ps[f].qt[ps[f].comp_q[c]] + 64);
        }
        for (int c = F.ncomp; c < kMaxComp; ++c) { F.dc_tab[c] = F.dc_tab[0]; F.ac_tab[c] = F.ac_tab[0]; }
    }
    hc.mark("parse + tables");
    // ---- layout: upload (frames, tables, quant, chunk map, entropy bytes) and device arenas
    size_t src_total = 0, stream_total = 0, coef_total = 0, samp_total = 0;
    uint32_t chunks = 0, subs = 0, nsub_max = 0, max_blocks = 0;
    int np = 1;
    for (int f = 0; f < n; ++f) {
        Frame &F = fr[f];
        F.src_off = src_total;
        F.src_len = (uint32_t)ps[f].ecs_len;
        src_total += align_up(F.src_len + 16, 16);
        F.chunk0 = chunks;
        F.nchunk = (F.src_len + kChunk - 1) / kChunk;
        for (uint32_t k = 0; k < F.nchunk; ++k) chunk_frame.push_back((uint32_t)f);
        chunks += F.nchunk;
        F.bits_off = stream_total;
        stream_total += align_up(F.src_len + kStreamPad + 16, 256);
        F.sub0 = subs;
        F.nsub = (uint32_t)(((uint64_t)F.src_len * 8 + kSubBits - 1) / kSubBits);
        subs += F.nsub;
        nsub_max = std::max(nsub_max, F.nsub);
        np = std::max(np, F.bpm);
        if (F.bpm > 6) return pano_fail(ctx, PANO_E_UNSUPPORTED, "JPEG with more than 6 blocks per MCU");
        for (int c = 0; c < F.ncomp; ++c) {
            const size_t nbk = (size_t)F.comp_bw[c] * F.comp_bh[c];
            F.coef_off[c] = coef_total;
            coef_total += nbk * 64;
            F.samp_off[c] = samp_total;
            samp_total += align_up(nbk * 64, 256);
            max_blocks = std::max(max_blocks, (uint32_t)nbk);
        }
    }
    size_t up = 0;
    const size_t o_frames = up;  up = align_up(up + sizeof(Frame) * n, 256);
    const size_t o_tabs = up;    up = align_up(up + sizeof(Huff) * tabs.size(), 256);
    const size_t o_quant = up;   up = align_up(up + 2 * quant.size(), 256);
    const size_t o_chunks = up;  up = align_up(up + 4 * chunk_frame.size(), 256);
    const size_t o_src = up;     up = align_up(up + src_total, 256);
    const size_t up_bytes = up;
    const int nps = 2 * np + 1;
    size_t dv = align_up(up_bytes, 256);
    const size_t o_stream = dv;  dv = align_up(dv + stream_total, 256);
    const size_t o_coef = dv;    dv = align_up(dv + 2 * coef_total, 256);
    const size_t o_samp = dv;    dv = align_up(dv + samp_total, 256);
    const size_t o_ccnt = dv;    dv = align_up(dv + 4 * (size_t)chunks, 256);
    const size_t o_nbits = dv;   dv = align_up(dv + 4 * (size_t)n, 256);
    const size_t o_flags = dv;   dv = align_up(dv + 4 * (size_t)n, 256);
    const size_t o_stats = dv;   dv = align_up(dv + 16 * (size_t)n, 256);
    const size_t o_cand = dv;    dv = align_up(dv + 8 * (size_t)subs * nps, 256);
    const size_t o_cexit = dv;   dv = align_up(dv + 8 * (size_t)subs * nps, 256);
    const size_t o_cstats = dv;  dv = align_up(dv + sizeof(SubStats) * (size_t)subs * nps, 256);
    const size_t o_start = dv;   dv = align_up(dv + 8 * (size_t)subs, 256);
    const size_t o_scan = dv;    dv = align_up(dv + sizeof(SubStats) * (size_t)subs, 256);
    const size_t o_maps = dv;    dv = align_up(dv + 8 * (size_t)subs, 256);
    const size_t dev_bytes = dv;

    hc.mark("layout");
    int rc = pano_grow(ctx, &ctx->jscratch, &ctx->jscratch_bytes, dev_bytes);
    if (rc) return rc;
    // pinned staging, two buffers in turn: wait until the upload out of this one (two calls
    // ago) has completed, fill it, upload
    const int slot = ctx->jslot;
    ctx->jslot ^= 1;
    if (!ctx->jev[slot]) PANO_HIP(ctx, hipEventCreateWithFlags(&ctx->jev[slot], hipEventDisableTiming));
    else PANO_HIP(ctx, hipEventSynchronize(ctx->jev[slot]));
    if (ctx->jpin_bytes[slot] < up_bytes) {
        if (ctx->jpin[slot]) (void)hipHostFree(ctx->jpin[slot]);
        ctx->jpin[slot] = nullptr;
        ctx->jpin_bytes[slot] = 0;
        const size_t sz = up_bytes + up_bytes / 4 + 65536;
        PANO_HIP(ctx, hipHostMalloc(&ctx->jpin[slot], sz, hipHostMallocDefault));
        ctx->jpin_bytes[slot] = sz;
    }
    hc.mark("grow + staging wait");
    uint8_t *pin = (uint8_t *)ctx->jpin[slot];
    memcpy(pin + o_frames, fr.data(), sizeof(Frame) * n);
    if (!tabs.empty()) memcpy(pin + o_tabs, tabs.data(), sizeof(Huff) * tabs.size());
    memcpy(pin + o_quant, quant.data(), 2 * quant.size());
    memcpy(pin + o_chunks, chunk_frame.data(), 4 * chunk_frame.size());
    for (int f = 0; f < n; ++f) {
        memcpy(pin + o_src + fr[f].src_off, ps[f].ecs, fr[f].src_len);
        memset(pin + o_src + fr[f].src_off + fr[f].src_len, 0, 16);
    }
    hc.mark("pinned memcpy");
    uint8_t *dev = (uint8_t *)ctx->jscratch;
    PANO_HIP(ctx, hipMemcpyAsync(dev, pin, up_bytes, hipMemcpyHostToDevice, ctx->stream));
    PANO_HIP(ctx, hipEventRecord(ctx->jev[slot], ctx->stream));
    hc.mark("upload enqueue");

    Dev D;
    D.frames = (const Frame *)(dev + o_frames);
    D.tabs = (const Huff *)(dev + o_tabs);
    D.quant = (const uint16_t *)(dev + o_quant);
    D.chunk_frame = (const uint32_t *)(dev + o_chunks);
    D.src = dev + o_src;
    D.stream = dev + o_stream;
    D.coef = (int16_t *)(dev + o_coef);
    D.samp = dev + o_samp;
    D.chunk_cnt = (uint32_t *)(dev + o_ccnt);
    D.nbits = (uint32_t *)(dev + o_nbits);
    D.flags = (int32_t *)(dev + o_flags);
    D.stats = (int32_t *)(dev + o_stats);
    ctx->jstats = D.stats;
    ctx->jstats_n = n;
    D.status = status;
    D.cand = (uint64_t *)(dev + o_cand);
    D.cexit = (uint64_t *)(dev + o_cexit);
    D.cstats = (SubStats *)(dev + o_cstats);
    D.start = (uint64_t *)(dev + o_start);
    D.scan = (SubStats *)(dev + o_scan);
    D.maps = (uint64_t *)(dev + o_maps);
    D.n = n;
    D.np = np;
    D.nps = nps;
    {
        // subsequences per warm chain (PANO_JPEG_CHAIN, 1..kChain; speed only)
        const char *env = getenv("PANO_JPEG_CHAIN");
        const int g = env ? atoi(env) : 1;
        D.chain = g < 1 ? 1 : (g > kChain ? kChain : g);
    }

    PanoProf prof_(ctx, PK_JPEG);
    rc = launch_fill(ctx, dev + o_coef, 0, 2 * coef_total);
    if (!rc) rc = launch_fill(ctx, dev + o_flags, 0, 4 * (size_t)n);
    if (!rc) rc = launch_fill(ctx, dev + o_stats, 0, 16 * (size_t)n);
    if (rc) return rc;
    jpeg_unstuff_count<<<chunks, 256, 0, ctx->stream>>>(D);
    jpeg_unstuff_write<<<chunks, 256, 0, ctx->stream>>>(D);
    {
        const uint32_t per = (uint32_t)(chains_per_block(np) * D.chain);
        jpeg_sync_warm<<<dim3((nsub_max + per - 1) / per, n), kSyncThreads, 0, ctx->stream>>>(D);
        const uint32_t spb = kSyncThreads / np;
        jpeg_sync_fix<<<dim3((nsub_max + spb - 1) / spb, n), kSyncThreads, 0, ctx->stream>>>(D);
        jpeg_sync_fix2<<<dim3((nsub_max + spb - 1) / spb, n), kSyncThreads, 0, ctx->stream>>>(D);
    }
    jpeg_sync_maps<<<dim3((nsub_max + 255) / 256, n), 256, 0, ctx->stream>>>(D);
    jpeg_sync_resolve<<<n, kResolveThreads, 0, ctx->stream>>>(D);
    jpeg_write<<<dim3((nsub_max + kWriteThreads - 1) / kWriteThreads, n), kWriteThreads, 0, ctx->stream>>>(D);
    jpeg_idct<<<dim3((max_blocks + 31) / 32, n * kMaxComp), 256, 0, ctx->stream>>>(D);
    jpeg_color<<<dim3((unsigned)(((size_t)h * w + 255) / 256), n), 256, 0, ctx->stream>>>(D, bgr, h, w);
    PANO_LAUNCH_CHECK(ctx, "jpeg decode");
    hc.mark("launches");
    return PANO_OK;
}
