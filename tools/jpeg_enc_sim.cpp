// jpeg_enc_sim.cpp -- CPU replay of the GPU JPEG encoder's per-block functions (jpeg_core.h:
// enc_samples, enc_transform, encode_block; jpeg_enc.hip runs them one block per thread).
// Development and test tool: tests/test_jpeg.py compares its file with PIL's
// save(quality=q) byte for byte.
//
//   jpeg_enc_sim in.bgr h w quality out.jpg
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../vfx_image_stitching_amd/csrc/jpeg_core.h"

using namespace pj;

int main(int argc, char **argv) {
    if (argc != 6) { fprintf(stderr, "usage: jpeg_enc_sim in.bgr h w quality out.jpg\n"); return 2; }
    const int h = atoi(argv[2]), w = atoi(argv[3]), q = atoi(argv[4]);
    std::vector<uint8_t> img((size_t)h * w * 3);
    FILE *f = fopen(argv[1], "rb");
    if (!f || fread(img.data(), 1, img.size(), f) != img.size()) { perror("in"); return 2; }
    fclose(f);
    uint16_t lum[64], chr[64];
    quant_tables(q, lum, chr);
    QRecip ql[64], qc[64];
    for (int i = 0; i < 64; ++i) { ql[i] = q_recip(8u * lum[i]); qc[i] = q_recip(8u * chr[i]); }
    HuffEnc E[4];            // DC lum, AC lum, DC chr, AC chr
    std_huff_enc(0, 0, &E[0]); std_huff_enc(1, 0, &E[1]); std_huff_enc(0, 1, &E[2]); std_huff_enc(1, 1, &E[3]);
    uint8_t nat[64];
    for (int k = 0; k < 64; ++k) nat[k] = (uint8_t)natural_order(k);
    const EncGeom G = enc_geom(h, w, (int64_t)w * 3);
    const int nblk = G.mcus_x * G.mcus_y * 6;
    std::vector<int16_t> coef((size_t)nblk * 64);
    for (int b = 0; b < nblk; ++b) {
        int32_t s[64];
        const int src = enc_dummy_source(G, b);
        const QRecip *qq = (b % 6) < 4 ? ql : qc;
        if (src < 0) {
            enc_samples(img.data(), G, b, s);
            enc_transform(s, qq, &coef[(size_t)b * 64]);
        } else {
            int16_t tmp[64];
            int sb = src;
            while (enc_dummy_source(G, sb) >= 0) sb = enc_dummy_source(G, sb);
            enc_samples(img.data(), G, sb, s);
            enc_transform(s, qq, tmp);
            for (int i = 0; i < 64; ++i) coef[(size_t)b * 64 + i] = 0;
            coef[(size_t)b * 64] = tmp[0];
        }
    }
    std::vector<uint8_t> out = encode_header(h, w, lum, chr);
    uint64_t acc = 0;
    int nacc = 0;
    auto byte_out = [&](uint8_t v) { out.push_back(v); if (v == 0xFF) out.push_back(0); };
    struct Put {
        uint64_t *acc; int *nacc; decltype(byte_out) *bo;
        void operator()(uint32_t v, int len) {
            *acc = (*acc << len) | (v & ((1u << len) - 1));
            *nacc += len;
            while (*nacc >= 8) { (*bo)((uint8_t)(*acc >> (*nacc - 8))); *nacc -= 8; }
        }
    } put{&acc, &nacc, &byte_out};
    for (int b = 0; b < nblk; ++b) {
        const int p = enc_prev_same(b);
        const int diff = coef[(size_t)b * 64] - (p >= 0 ? coef[(size_t)p * 64] : 0);
        const int c = (b % 6) < 4 ? 0 : 1;
        encode_block(&coef[(size_t)b * 64], diff, &E[2 * c], &E[2 * c + 1], nat, put);
    }
    if (nacc) put(0x7F, 8 - nacc);            // jchuff.c flush_bits: pad with ones
    out.push_back(0xFF); out.push_back(0xD9);
    FILE *o = fopen(argv[5], "wb");
    if (!o) { perror("out"); return 2; }
    fwrite(out.data(), 1, out.size(), o);
    fclose(o);
    printf("{\"bytes\": %zu, \"blocks\": %d}\n", out.size(), nblk);
    return 0;
}
