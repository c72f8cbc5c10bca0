// jpeg_sim.cpp -- CPU replay of the GPU JPEG decoder's passes (vfx_image_stitching_amd/csrc/
// jpeg.hip) through the same __host__ __device__ functions (jpeg_core.h), one "thread" at a
// time.  Development and test tool: tests/test_jpeg.py compares its output with PIL's decode
// on the CPU, so the decode logic (parse, tables, self-synchronising walk, DC prediction,
// islow IDCT, fancy upsampling, colour conversion) is checked without a GPU; the -m gpu tests
// check the kernels themselves.
//
//   jpeg_sim [-L bits] in.jpg out.bgr   -> raw u8 BGR [h][w][3]; stats on stdout (JSON)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../vfx_image_stitching_amd/csrc/jpeg_core.h"

using namespace pj;

int main(int argc, char **argv) {
    int L = kSubBits, a = 1;
    if (argc > 2 && !strcmp(argv[1], "-L")) { L = atoi(argv[2]); a = 3; }
    if (argc - a != 2) { fprintf(stderr, "usage: jpeg_sim [-L bits] in.jpg out.bgr\n"); return 2; }
    FILE *fp = fopen(argv[a], "rb");
    if (!fp) { perror("open"); return 2; }
    std::vector<uint8_t> buf;
    uint8_t tmp[65536];
    size_t r;
    while ((r = fread(tmp, 1, sizeof tmp, fp)) > 0) buf.insert(buf.end(), tmp, tmp + r);
    fclose(fp);

    Parsed P;
    std::string err;
    int rc = parse(buf.data(), buf.size(), &P, &err);
    Frame F;
    if (rc == 0) rc = plan_frame(P, &F, &err);
    if (rc) { printf("{\"status\": %d, \"error\": \"%s\"}\n", rc, err.c_str()); return 1; }

    // tables (std tables where the file has none, as libjpeg-turbo does)
    Huff dcT[kMaxComp], acT[kMaxComp];
    for (int c = 0; c < P.ncomp; ++c) {
        uint8_t bits[17], vals[256];
        const int d = P.comp_dc[c], q = P.comp_ac[c];
        if (P.h_ok[0][d]) make_huff(P.hbits[0][d], P.hvals[0][d], &dcT[c]); else { std_huff(0, d, bits, vals); make_huff(bits, vals, &dcT[c]); }
        if (P.h_ok[1][q]) make_huff(P.hbits[1][q], P.hvals[1][q], &acT[c]); else { std_huff(1, q, bits, vals); make_huff(bits, vals, &acT[c]); }
    }
    const Huff *dcp = dcT, *acp = acT;

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
    const uint32_t *words = (const uint32_t *)st.data();
    const uint32_t nw = (uint32_t)(st.size() / 4);
    const uint32_t nsub = (nbits + L - 1) / L;

    // pass A (jpeg_sync_warm): for every subsequence t and every MCU phase hypothesis j, a
    // warm-up window of W bits before t is decoded from (t*L - W, block j, DC next) to find a
    // candidate start c[t][j]; subsequences within W of the stream start decode from the exact
    // start (bit 0).  Each candidate is then decoded over t with counting: exit x[t][j] and
    // statistics.  A decode from a wrong bit position re-synchronises with the true decode
    // only when it also lands in the right MCU phase; trying every phase makes one of them
    // land in it early (the phase, not the bit alignment, dominates the sync distance).
    const uint32_t W = getenv("JPEG_SIM_W") ? (uint32_t)atoi(getenv("JPEG_SIM_W")) : F.warm;
    const int NP = F.bpm;
    std::vector<uint64_t> cand((size_t)nsub * NP), ex((size_t)nsub * NP);
    std::vector<SubStats> cstats((size_t)nsub * NP);
    auto end_of = [&](uint32_t t) { uint32_t e = (t + 1) * (uint32_t)L; return e < nbits ? e : nbits; };
    long decoded = 0;
    for (uint32_t t = 0; t < nsub; ++t)
        for (int j = 0; j < NP; ++j) {
            const uint32_t p0 = t * (uint32_t)L;
            SinkNone sn;
            const size_t q = (size_t)t * NP + j;
            cand[q] = p0 <= W ? walk(words, nw, pack_state(0, 0, 0), p0, dcp, acp, F.mcu_comp, F.bpm, sn)
                              : walk(words, nw, pack_state(p0 - W, j, 0), p0, dcp, acp, F.mcu_comp, F.bpm, sn);
            SinkCount sc;
            ex[q] = walk(words, nw, cand[q], end_of(t), dcp, acp, F.mcu_comp, F.bpm, sc);
            cstats[q] = sc.stats();
            ++decoded;
        }
    // resolve (jpeg_sync_resolve): the chain J_t = index of the candidate of t equal to the
    // true exit of t-1, starting from the exact t = 0; no match -> decode t from that exit.
    std::vector<uint64_t> start(nsub);
    std::vector<SubStats> stats(nsub);
    int fails = 0, rounds = 0, fixes = 0, serial_fixes = 0;
    int J = 0;
    start[0] = cand[0]; stats[0] = cstats[0];
    uint64_t prev_exit = ex[0];
    for (uint32_t t = 1; t < nsub; ++t) {
        int jj = -1;
        for (int j = 0; j < NP; ++j) if (cand[(size_t)t * NP + j] == prev_exit) { jj = j; break; }
        if (jj < 0) {
            ++fails;
            SinkCount sc;
            start[t] = prev_exit;
            prev_exit = walk(words, nw, start[t], end_of(t), dcp, acp, F.mcu_comp, F.bpm, sc);
            stats[t] = sc.stats();
        } else {
            start[t] = cand[(size_t)t * NP + jj];
            stats[t] = cstats[(size_t)t * NP + jj];
            prev_exit = ex[(size_t)t * NP + jj];
        }
        J = jj;
    }
    (void)J; fixes = fails;
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
        w.blk = scan[t].blocks - (k0 > 0 ? 1 : 0);
        w.p0 = scan[t].dc[0]; w.p1 = scan[t].dc[1]; w.p2 = scan[t].dc[2];
        w.live = k0 > 0 && w.blk >= 0 && w.blk < F.total_blocks;
        w.addr = w.live ? block_addr(F, w.blk) : 0;
        walk(words, nw, start[t], end_of(t), dcp, acp, F.mcu_comp, F.bpm, w);
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
    FILE *fo = fopen(argv[a + 1], "wb");
    if (!fo) { perror("out"); return 2; }
    fwrite(out.data(), 1, out.size(), fo);
    fclose(fo);
    printf("{\"status\": 0, \"h\": %d, \"w\": %d, \"ncomp\": %d, \"upsample\": %d, \"nbits\": %u, \"nsub\": %u, "
           "\"rounds\": %d, \"fixes\": %d, \"serial_fixes\": %d, \"walks\": %ld, \"blocks\": %d, \"total_blocks\": %d, "
           "\"markers\": %d}\n",
           F.h, F.w, F.ncomp, F.upsample, nbits, nsub, rounds, fixes, serial_fixes, decoded,
           acc.blocks, F.total_blocks, markers);
    return 0;
}
