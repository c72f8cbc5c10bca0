// jpeg_sim.cpp -- CPU replay of the GPU JPEG decoder's passes (vfx_image_stitching_amd/csrc/
// jpeg.hip) through the same __host__ __device__ functions (jpeg_core.h), one "thread" at a
// time.  Development and test tool: tests/test_jpeg.py compares its output with PIL's decode
// on the CPU, so the decode logic (parse, tables, self-synchronising walk, DC prediction,
// islow IDCT, fancy upsampling, colour conversion) is checked without a GPU; the -m gpu tests
// check the kernels themselves.
//
//   jpeg_sim [-L bits] in.jpg out.bgr   -> raw u8 BGR [h][w][3]; stats on stdout (JSON)
//   jpeg_sim [-L bits] --batch f1 f2 ...  -> one stats line per file, no pixels
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../include/pano.h"
#include "../vfx_image_stitching_amd/csrc/jpeg_core.h"

using namespace pj;

static std::vector<uint8_t> read_file(const char *path, bool *ok) {
    std::vector<uint8_t> buf;
    FILE *fp = fopen(path, "rb");
    *ok = fp != nullptr;
    if (!fp) return buf;
    uint8_t tmp[65536];
    size_t r;
    while ((r = fread(tmp, 1, sizeof tmp, fp)) > 0) buf.insert(buf.end(), tmp, tmp + r);
    fclose(fp);
    return buf;
}

// The whole decode of one file; the status line (JSON) goes to stdout, the pixels to *out.
// Returns 0 on success.
static int decode_one(const std::vector<uint8_t> &buf, int L, std::vector<uint8_t> *out_px) {
    Parsed P;
    std::string err;
    int rc = parse(buf.data(), buf.size(), &P, &err);
    Frame F;
    if (rc == 0) rc = plan_frame(P, &F, &err);
    if (rc == 0 && P.ecs_len == 0) { rc = PANO_E_ARG; err = "empty scan"; }   // as pano_jpeg_decode
    if (rc) { printf("{\"status\": %d, \"error\": \"%s\"}\n", rc, err.c_str()); return 1; }

    // tables (std tables where the file has none, as libjpeg-turbo does): T[c] DC, T[3 + c] AC
    Huff T[2 * kMaxComp];
    for (int c = 0; c < P.ncomp; ++c)
        for (int cls = 0; cls < 2; ++cls) {
            uint8_t bits[17], vals[256];
            const int id = cls ? P.comp_ac[c] : P.comp_dc[c];
            if (P.h_ok[cls][id]) { memcpy(bits, P.hbits[cls][id], 17); memcpy(vals, P.hvals[cls][id], 256); }
            else std_huff(cls, id, bits, vals);
            const int hr = make_huff(cls, bits, vals, &T[cls * 3 + c]);
            if (hr) { printf("{\"status\": %d, \"error\": \"huffman table\"}\n", hr); return 1; }
        }

    // unstuff (jpeg_unstuff_* kernels): drop the 0x00 after every 0xFF
    std::vector<uint8_t> st;
    int markers = 0;
    for (size_t i = 0; i < P.ecs_len; ++i) {
        const uint8_t b = P.ecs[i];
        if (i > 0 && P.ecs[i - 1] == 0xFF) {
            if (b == 0) continue;
            ++markers;
        }
        st.push_back(b);
    }
    const uint32_t nbits = (uint32_t)st.size() * 8;
    st.resize(st.size() + kStreamPad, 0);
    while (st.size() % 4) st.push_back(0);
    std::vector<uint32_t> wv(st.size() / 4);     // stream-order words, as the kernels stage them
    for (size_t i = 0; i < wv.size(); ++i)
        wv[i] = (uint32_t)st[4 * i] << 24 | (uint32_t)st[4 * i + 1] << 16 | (uint32_t)st[4 * i + 2] << 8 | st[4 * i + 3];
    const uint32_t *words = wv.data();
    const uint32_t nw = (uint32_t)wv.size();
    const uint32_t nsub = (nbits + L - 1) / L;

    // jpeg_sync_warm: for every subsequence t and MCU phase hypothesis j < bpm, a warm-up
    // window of W bits before t is decoded from (t*L - W, block j, DC next) to a candidate start
    // c[t][j] (subsequences within W of the stream start decode from the exact start, bit 0);
    // each candidate is then decoded over t with counting: exit x[t][j] and statistics.  A
    // decode from a wrong bit position re-synchronises with the true decode only when it also
    // lands in the right block of the MCU; trying every phase makes one of them land early.
    const uint32_t W = getenv("JPEG_SIM_W") ? (uint32_t)atoi(getenv("JPEG_SIM_W")) : F.warm;
    const int NP = F.bpm, NS = 2 * F.bpm + 1;      // warm slots, fix slots, fix2 slot
    const uint64_t kNoCand = ~0ull;
    std::vector<uint64_t> cand((size_t)nsub * NS, kNoCand), ex((size_t)nsub * NS, kNoCand);
    std::vector<SubStats> cstats((size_t)nsub * NS);
    auto end_of = [&](uint32_t t) { uint32_t e = (t + 1) * (uint32_t)L; return e < nbits ? e : nbits; };
    long decoded = 0;
    const uint32_t G = getenv("JPEG_SIM_CHAIN") ? (uint32_t)atoi(getenv("JPEG_SIM_CHAIN")) : 1;
    for (uint32_t ta = 0; ta < nsub; ta += G)          // chains of G subsequences
        for (int j = 0; j < NP; ++j) {
            const uint32_t p0 = ta * (uint32_t)L;
            SinkNone sn;
            uint64_t stt = p0 <= W ? walk(words, 0, nw, pack_state(0, 0, 0), p0, T, F.mcu_comp, F.bpm, sn)
                                   : walk(words, 0, nw, pack_state(p0 - W, j, 0), p0, T, F.mcu_comp, F.bpm, sn);
            for (uint32_t t = ta; t < ta + G && t < nsub; ++t) {
                const size_t q = (size_t)t * NS + j;
                SinkCount sc;
                cand[q] = stt;
                ex[q] = walk(words, 0, nw, stt, end_of(t), T, F.mcu_comp, F.bpm, sc);
                cstats[q] = sc.stats();
                stt = ex[q];
                ++decoded;
            }
        }
    // jpeg_sync_fix: where a warm exit of t-1 matches no warm candidate of t, decode t from that
    // exit as an extra candidate (slot bpm + i)
    int fix_slots = 0;
    for (uint32_t t = 1; t < nsub; ++t)
        for (int i = 0; i < NP; ++i) {
            const uint64_t e = ex[(size_t)(t - 1) * NS + i];
            bool hit = false;
            for (int j = 0; j < NP; ++j) hit |= cand[(size_t)t * NS + j] == e;
            if (hit) continue;
            const size_t q = (size_t)t * NS + NP + i;
            SinkCount sc;
            cand[q] = e;
            ex[q] = walk(words, 0, nw, e, end_of(t), T, F.mcu_comp, F.bpm, sc);
            cstats[q] = sc.stats();
            ++fix_slots;
        }
    // jpeg_sync_fix2: the same from the fix slots' exits, into slot 2 np (first such one)
    for (uint32_t t = nsub; t-- > 1;)                 // reads t-1's fix slots only: any order
        for (int i = 0; i < NP; ++i) {
            const size_t qp = (size_t)(t - 1) * NS + NP + i;
            if (cand[qp] == kNoCand) continue;
            const uint64_t e = ex[qp];
            bool hit = false;
            for (int j = 0; j < 2 * NP; ++j) hit |= cand[(size_t)t * NS + j] == e;
            if (hit) continue;
            const size_t q = (size_t)t * NS + 2 * NP;
            SinkCount sc;
            cand[q] = e;
            ex[q] = walk(words, 0, nw, e, end_of(t), T, F.mcu_comp, F.bpm, sc);
            cstats[q] = sc.stats();
            ++fix_slots;
            break;
        }
    // jpeg_sync_resolve: J_t = the first candidate of t equal to the true exit of t-1 (t = 0
    // exact); none -> decode t from that exit (serial fallback)
    std::vector<uint64_t> start(nsub);
    std::vector<SubStats> stats(nsub);
    int fails = 0;
    start[0] = cand[0]; stats[0] = cstats[0];
    uint64_t prev_exit = ex[0];
    for (uint32_t t = 1; t < nsub; ++t) {
        int jj = -1;
        for (int j = 0; j < NS; ++j) if (cand[(size_t)t * NS + j] == prev_exit) { jj = j; break; }
        if (jj < 0) {
            ++fails;
            SinkCount sc;
            start[t] = prev_exit;
            prev_exit = walk(words, 0, nw, start[t], end_of(t), T, F.mcu_comp, F.bpm, sc);
            stats[t] = sc.stats();
        } else {
            start[t] = cand[(size_t)t * NS + jj];
            stats[t] = cstats[(size_t)t * NS + jj];
            prev_exit = ex[(size_t)t * NS + jj];
        }
    }
    const int fixes = fails, serial_fixes = fails;
    // scan
    std::vector<SubStats> scan(nsub);
    SubStats acc = {0, {0, 0, 0}};
    for (uint32_t t = 0; t < nsub; ++t) {
        scan[t] = acc;
        acc.blocks += stats[t].blocks;
        for (int c = 0; c < kMaxComp; ++c) acc.dc[c] += stats[t].dc[c];
    }
    if (acc.blocks < F.total_blocks) { printf("{\"status\": -1, \"error\": \"truncated: %d of %d blocks\"}\n", acc.blocks, F.total_blocks); return 1; }
    // write
    size_t ncoef = 0;
    for (int c = 0; c < F.ncomp; ++c) { F.coef_off[c] = ncoef; ncoef += (size_t)F.comp_bw[c] * F.comp_bh[c] * 64; }
    std::vector<int16_t> coef(ncoef, 0);
    uint8_t nat[80];
    for (int k = 0; k < 80; ++k) nat[k] = (uint8_t)natural_order(k);
    for (uint32_t t = 0; t < nsub; ++t) {
        SinkWrite w;
        w.coef = coef.data(); w.F = &F; w.nat = nat;
        const int k0 = state_k(start[t]);
        const int32_t b0 = scan[t].blocks - (k0 > 0 ? 1 : 0);
        w.seek(b0 > 0 ? b0 : 0);
        w.blk = b0;
        w.p0 = scan[t].dc[0]; w.p1 = scan[t].dc[1]; w.p2 = scan[t].dc[2];
        w.live = k0 > 0 && b0 >= 0 && b0 < F.total_blocks;
        w.addr = w.live ? w.address() : 0;
        walk(words, 0, nw, start[t], end_of(t), T, F.mcu_comp, F.bpm, w);
    }
    // IDCT
    std::vector<std::vector<uint8_t>> samp(F.ncomp);
    for (int c = 0; c < F.ncomp; ++c) {
        const int pw = F.comp_bw[c] * 8;
        samp[c].assign((size_t)pw * F.comp_bh[c] * 8, 0);
        const uint16_t *q = P.qt[P.comp_q[c]];
        for (int by = 0; by < F.comp_bh[c]; ++by)
            for (int bx = 0; bx < F.comp_bw[c]; ++bx) {
                const int16_t *blk = &coef[F.coef_off[c] + ((size_t)by * F.comp_bw[c] + bx) * 64];
                int32_t ws[64];
                for (int cc = 0; cc < 8; ++cc) idct_col(blk, q, cc, ws);
                for (int rr = 0; rr < 8; ++rr) idct_row(ws, rr, &samp[c][(size_t)(by * 8 + rr) * pw + bx * 8]);
            }
    }
    // upsample + colour
    std::vector<uint8_t> out((size_t)F.h * F.w * 3);
    for (int y = 0; y < F.h; ++y)
        for (int x = 0; x < F.w; ++x) {
            uint8_t *o = &out[((size_t)y * F.w + x) * 3];
            const int Y = samp[0][(size_t)y * F.comp_bw[0] * 8 + x];
            if (F.ncomp == 1) { o[0] = o[1] = o[2] = (uint8_t)Y; continue; }
            const int cb = chroma_at(samp[1].data(), F.comp_bw[1] * 8, F.comp_dw[1], F.comp_dh[1], F.upsample, x, y);
            const int cr = chroma_at(samp[2].data(), F.comp_bw[2] * 8, F.comp_dw[2], F.comp_dh[2], F.upsample, x, y);
            ycc_to_bgr(Y, cb, cr, o);
        }
    printf("{\"status\": 0, \"h\": %d, \"w\": %d, \"ncomp\": %d, \"upsample\": %d, \"nbits\": %u, \"nsub\": %u, "
           "\"fix_slots\": %d, \"fixes\": %d, \"serial_fixes\": %d, \"walks\": %ld, \"blocks\": %d, \"total_blocks\": %d, "
           "\"markers\": %d}\n",
           F.h, F.w, F.ncomp, F.upsample, nbits, nsub, fix_slots, fixes, serial_fixes, decoded,
           acc.blocks, F.total_blocks, markers);
    out_px->swap(out);
    return 0;
}

int main(int argc, char **argv) {
    int L = kSubBits, a = 1;
    if (argc > 2 && !strcmp(argv[1], "-L")) { L = atoi(argv[2]); a = 3; }
    if (argc - a >= 1 && !strcmp(argv[a], "--batch")) {
        // --batch f1 f2 ...: decode every file, one status line each, no pixels written (the
        // sanitizer corpus run, tools/host_sanitize.sh)
        for (int i = a + 1; i < argc; ++i) {
            bool ok;
            const std::vector<uint8_t> buf = read_file(argv[i], &ok);
            if (!ok) { perror(argv[i]); return 2; }
            std::vector<uint8_t> px;
            decode_one(buf, L, &px);
        }
        return 0;
    }
    if (argc - a != 2) { fprintf(stderr, "usage: jpeg_sim [-L bits] in.jpg out.bgr | jpeg_sim --batch f...\n"); return 2; }
    bool ok;
    const std::vector<uint8_t> buf = read_file(argv[a], &ok);
    if (!ok) { perror("open"); return 2; }
    std::vector<uint8_t> out;
    const int rc = decode_one(buf, L, &out);
    if (rc) return rc;
    FILE *fo = fopen(argv[a + 1], "wb");
    if (!fo) { perror("out"); return 2; }
    fwrite(out.data(), 1, out.size(), fo);
    fclose(fo);
    return 0;
}
