// jpeg_host.cpp -- host half of the baseline JPEG decoder: marker parsing (the subset of
// libjpeg's jdmarker.c a sequential file needs), Huffman decode tables (jdhuff.c
// jpeg_make_d_derived_tbl restated) and the Annex K.3 standard tables.  Everything that
// touches pixels runs on the GPU (jpeg.hip); this file only reads headers.
#include <stdlib.h>
#include <string.h>

#include "../../include/pano.h"
#include "jpeg_core.h"

namespace pj {

namespace {

// Annex K.3 (ITU-T T.81): code-length counts (lengths 1..16) and symbols of the four tables
// libjpeg installs by default (jstdhuff.c) and PIL's encoder writes.
const uint8_t kDcLumBits[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
const uint8_t kDcChrBits[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
const uint8_t kAcLumBits[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
const uint8_t kAcChrBits[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
const uint8_t kAcLumVals[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61,
    0x07, 0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52,
    0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25,
    0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45,
    0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64,
    0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99,
    0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6,
    0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3,
    0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8,
    0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
const uint8_t kAcChrVals[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61,
    0x71, 0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33,
    0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18,
    0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44,
    0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63,
    0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97,
    0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4,
    0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca,
    0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7,
    0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};

int fail(std::string *err, int code, const char *msg) {
    if (err) *err = msg;
    return code;
}

}  // namespace

void std_huff(int cls, int id, uint8_t *bits17, uint8_t *vals256) {
    const bool lum = id == 0;
    const uint8_t *bits = cls == 0 ? (lum ? kDcLumBits : kDcChrBits) : (lum ? kAcLumBits : kAcChrBits);
    bits17[0] = 0;
    int total = 0;
    for (int l = 0; l < 16; ++l) { bits17[l + 1] = bits[l]; total += bits[l]; }
    memset(vals256, 0, 256);
    if (cls == 0) {
        for (int i = 0; i < total; ++i) vals256[i] = (uint8_t)i;
    } else {
        memcpy(vals256, lum ? kAcLumVals : kAcChrVals, (size_t)total);
    }
}

void std_huff_enc(int cls, int id, HuffEnc *E) {
    // jchuff.c jpeg_make_c_derived_tbl over the Annex K table: canonical codes by length
    uint8_t bits[17], vals[256];
    std_huff(cls, id, bits, vals);
    memset(E, 0, sizeof(*E));
    int code = 0, p = 0;
    for (int l = 1; l <= 16; ++l) {
        for (int i = 0; i < bits[l]; ++i, ++p) {
            E->code[vals[p]] = (uint16_t)code++;
            E->len[vals[p]] = (uint8_t)l;
        }
        code <<= 1;
    }
}

void quant_tables(int quality, uint16_t *lum, uint16_t *chr) {
    // jcparam.c: Annex K.1 tables (natural order) scaled by jpeg_quality_scaling, clamped to
    // [1, 255] (force_baseline), as jpeg_set_quality(cinfo, quality, TRUE)
    static const uint16_t kLum[64] = {
        16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55,
        14, 13, 16, 24, 40, 57, 69, 56, 14, 17, 22, 29, 51, 87, 80, 62,
        18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
        49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
    static const uint16_t kChr[64] = {
        17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
        24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
        99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
        99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
    if (quality <= 0) quality = 1;
    if (quality > 100) quality = 100;
    const long scale = quality < 50 ? 5000 / quality : 200 - quality * 2;
    for (int i = 0; i < 64; ++i) {
        long a = ((long)kLum[i] * scale + 50) / 100, b = ((long)kChr[i] * scale + 50) / 100;
        lum[i] = (uint16_t)(a < 1 ? 1 : (a > 255 ? 255 : a));
        chr[i] = (uint16_t)(b < 1 ? 1 : (b > 255 ? 255 : b));
    }
}

std::vector<uint8_t> encode_header(int h, int w, const uint16_t *lum, const uint16_t *chr) {
    // jcmarker.c write_file_header / write_frame_header / write_scan_header for a baseline
    // 3-component 4:2:0 image with the default JFIF header and the Annex K Huffman tables
    std::vector<uint8_t> o = {0xFF, 0xD8, 0xFF, 0xE0, 0x00, 0x10, 'J', 'F', 'I', 'F', 0x00, 0x01, 0x01,
                              0x00, 0x00, 0x01, 0x00, 0x01, 0x00, 0x00};
    for (int t = 0; t < 2; ++t) {
        const uint16_t *q = t ? chr : lum;
        o.insert(o.end(), {0xFF, 0xDB, 0x00, 0x43, (uint8_t)t});
        for (int k = 0; k < 64; ++k) o.push_back((uint8_t)q[natural_order(k)]);
    }
    o.insert(o.end(), {0xFF, 0xC0, 0x00, 0x11, 0x08, (uint8_t)(h >> 8), (uint8_t)h, (uint8_t)(w >> 8), (uint8_t)w,
                       0x03, 0x01, 0x22, 0x00, 0x02, 0x11, 0x01, 0x03, 0x11, 0x01});
    for (int id = 0; id < 2; ++id)
        for (int cls = 0; cls < 2; ++cls) {
            uint8_t bits[17], vals[256];
            std_huff(cls, id, bits, vals);
            int total = 0;
            for (int l = 1; l <= 16; ++l) total += bits[l];
            const int len = 2 + 1 + 16 + total;
            o.insert(o.end(), {0xFF, 0xC4, (uint8_t)(len >> 8), (uint8_t)len, (uint8_t)(cls << 4 | id)});
            o.insert(o.end(), bits + 1, bits + 17);
            o.insert(o.end(), vals, vals + total);
        }
    o.insert(o.end(), {0xFF, 0xDA, 0x00, 0x0C, 0x03, 0x01, 0x00, 0x02, 0x11, 0x03, 0x11, 0x00, 0x3F, 0x00});
    return o;
}

int make_huff(int cls, const uint8_t *bits17, const uint8_t *vals, Huff *T) {
    // jdhuff.c jpeg_make_d_derived_tbl: code lengths -> canonical codes; then the two-level
    // lookup of jpeg_core.h (9 bits, then 7 more for the longer codes).
    int size[257], code[257];
    int p = 0;
    for (int l = 1; l <= 16; ++l) {
        if (p + bits17[l] > 256) return PANO_E_ARG;
        for (int i = 0; i < bits17[l]; ++i) size[p++] = l;
    }
    size[p] = 0;
    const int total = p;
    int c = 0, si = total ? size[0] : 0;
    p = 0;
    while (size[p]) {
        while (size[p] == si) code[p++] = c++;
        if (c >= (1 << si)) return PANO_E_ARG;     // JERR_BAD_HUFF_TABLE
        c <<= 1;
        ++si;
    }
    memset(T, 0, sizeof(*T));
    T->first_long = 512;
    int nsub = 0;
    for (int i = 0; i < total; ++i) {
        const int l = size[i];
        // length - 1 | magnitude bits << 4 | (zig-zag advance - 1) << 9 (jpeg_core.h Huff):
        // DC advance 1; AC s > 0: run + 1; ZRL 16; EOB (s = 0, any other run) to the end
        const int sym = vals[i];
        const int sbits = cls ? (sym & 15) : (sym > 16 ? 16 : sym);
        const int advm1 = !cls ? 0 : (sbits ? sym >> 4 : ((sym >> 4) == 15 ? 15 : 63));
        const uint16_t e = (uint16_t)((l - 1) | sbits << 4 | advm1 << 9);
        if (l <= 9) {
            const int lo = code[i] << (9 - l), hi = (code[i] + 1) << (9 - l);
            for (int q = lo; q < hi; ++q) T->lut[q] = e;
            continue;
        }
        const int pre = code[i] >> (l - 9);             // first 9 bits of the code
        if (!(T->lut[pre] & 0x8000)) {
            if (T->lut[pre] != 0) return PANO_E_ARG;    // a shorter code is its prefix
            if (nsub == kHuffSub) return PANO_E_UNSUPPORTED;
            if (nsub == 0) T->first_long = (uint32_t)pre;
            // canonical codes: the long prefixes are contiguous and in order (jpeg_core.h Huff)
            if ((uint32_t)pre != T->first_long + (uint32_t)nsub) return PANO_E_ARG;
            T->lut[pre] = (uint16_t)(0x8000 | nsub * 128);
            ++nsub;
        }
        uint16_t *sub = T->sub + (T->lut[pre] & 0x7FFF);
        const int rest = code[i] & ((1 << (l - 9)) - 1);    // the code's bits after the first 9
        const int lo = rest << (16 - l), hi = (rest + 1) << (16 - l);
        for (int q = lo; q < hi; ++q) sub[q] = e;
    }
    return PANO_OK;
}

int parse(const uint8_t *buf, size_t len, Parsed *P, std::string *err) {
    if (!buf || len < 4 || buf[0] != 0xFF || buf[1] != 0xD8) return fail(err, PANO_E_ARG, "not a JPEG (no SOI)");
    size_t i = 2;
    bool have_sof = false;
    for (;;) {
        if (i >= len) return fail(err, PANO_E_ARG, "truncated JPEG: no SOS");
        if (buf[i] != 0xFF) return fail(err, PANO_E_ARG, "corrupt JPEG: marker expected");
        while (i < len && buf[i] == 0xFF) ++i;           // fill bytes
        if (i >= len) return fail(err, PANO_E_ARG, "truncated JPEG");
        const int m = buf[i++];
        if (m == 0xD8 || m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;
        if (m == 0xD9) return fail(err, PANO_E_ARG, "JPEG has no scan (EOI before SOS)");
        if (i + 2 > len) return fail(err, PANO_E_ARG, "truncated JPEG segment");
        const size_t seglen = (size_t)buf[i] << 8 | buf[i + 1];
        if (seglen < 2 || i + seglen > len) return fail(err, PANO_E_ARG, "truncated JPEG segment");
        const uint8_t *s = buf + i + 2;
        const size_t sl = seglen - 2;
        switch (m) {
        case 0xC0: case 0xC1: {
            if (sl < 6) return fail(err, PANO_E_ARG, "bad SOF");
            if (s[0] != 8) return fail(err, PANO_E_UNSUPPORTED, "JPEG sample precision other than 8 bits");
            P->sof = m;
            P->h = s[1] << 8 | s[2];
            P->w = s[3] << 8 | s[4];
            P->ncomp = s[5];
            if (P->ncomp != 1 && P->ncomp != 3) return fail(err, PANO_E_UNSUPPORTED, "JPEG with other than 1 or 3 components");
            if (sl < 6 + 3 * (size_t)P->ncomp) return fail(err, PANO_E_ARG, "bad SOF");
            if (P->h <= 0 || P->w <= 0) return fail(err, PANO_E_UNSUPPORTED, "JPEG with DNL height or zero size");
            for (int c = 0; c < P->ncomp; ++c) {
                P->comp_id[c] = s[6 + 3 * c];
                P->comp_h[c] = s[7 + 3 * c] >> 4;
                P->comp_v[c] = s[7 + 3 * c] & 15;
                P->comp_q[c] = s[8 + 3 * c];
                if (P->comp_h[c] < 1 || P->comp_h[c] > 4 || P->comp_v[c] < 1 || P->comp_v[c] > 4 || P->comp_q[c] > 3)
                    return fail(err, PANO_E_ARG, "bad SOF component");
            }
            have_sof = true;
            break;
        }
        case 0xC2: case 0xC6: case 0xCA: case 0xCE:
            return fail(err, PANO_E_UNSUPPORTED, "progressive JPEG");
        case 0xC3: case 0xC5: case 0xC7: case 0xC9: case 0xCB: case 0xCD: case 0xCF:
            return fail(err, PANO_E_UNSUPPORTED, "lossless / hierarchical / arithmetic-coded JPEG");
        case 0xC4: {
            size_t j = 0;
            while (j < sl) {
                if (j + 17 > sl) return fail(err, PANO_E_ARG, "bad DHT");
                const int cls = s[j] >> 4, id = s[j] & 15;
                if (cls > 1 || id > 3) return fail(err, PANO_E_ARG, "bad DHT table id");
                int total = 0;
                P->hbits[cls][id][0] = 0;
                for (int l = 1; l <= 16; ++l) { P->hbits[cls][id][l] = s[j + l]; total += s[j + l]; }
                if (total > 256 || j + 17 + total > sl) return fail(err, PANO_E_ARG, "bad DHT");
                memset(P->hvals[cls][id], 0, 256);
                memcpy(P->hvals[cls][id], s + j + 17, (size_t)total);
                P->h_ok[cls][id] = true;
                j += 17 + total;
            }
            break;
        }
        case 0xDB: {
            size_t j = 0;
            while (j < sl) {
                const int pq = s[j] >> 4, tq = s[j] & 15;
                if (tq > 3 || pq > 1 || j + 1 + 64 * (pq + 1) > sl) return fail(err, PANO_E_ARG, "bad DQT");
                for (int k = 0; k < 64; ++k) {
                    const int v = pq ? (s[j + 1 + 2 * k] << 8 | s[j + 2 + 2 * k]) : s[j + 1 + k];
                    P->qt[tq][natural_order(k)] = (uint16_t)v;   // the file stores zig-zag order
                }
                P->qt_ok[tq] = true;
                j += 1 + 64 * (pq + 1);
            }
            break;
        }
        case 0xDD:
            if (sl < 2) return fail(err, PANO_E_ARG, "bad DRI");
            P->restart = s[0] << 8 | s[1];
            break;
        case 0xDA: {
            if (!have_sof) return fail(err, PANO_E_ARG, "SOS before SOF");
            const int ns = sl ? s[0] : 0;
            if (ns != P->ncomp) return fail(err, PANO_E_UNSUPPORTED, "multi-scan (non-interleaved) sequential JPEG");
            if (sl < 1 + 2 * (size_t)ns + 3) return fail(err, PANO_E_ARG, "bad SOS");
            int order[kMaxComp];
            for (int q = 0; q < ns; ++q) {
                const int cs = s[1 + 2 * q];
                int c = -1;
                for (int t = 0; t < P->ncomp; ++t) if (P->comp_id[t] == cs) c = t;
                if (c < 0) return fail(err, PANO_E_ARG, "SOS names an unknown component");
                order[q] = c;
                P->comp_dc[c] = s[2 + 2 * q] >> 4;
                P->comp_ac[c] = s[2 + 2 * q] & 15;
                if (P->comp_dc[c] > 3 || P->comp_ac[c] > 3) return fail(err, PANO_E_ARG, "bad SOS table id");
            }
            for (int q = 0; q < ns; ++q)
                if (order[q] != q) return fail(err, PANO_E_UNSUPPORTED, "scan order differs from frame order");
            const uint8_t *t = s + 1 + 2 * ns;
            if (t[0] != 0 || t[1] != 63 || t[2] != 0) return fail(err, PANO_E_UNSUPPORTED, "JPEG scan is not sequential DCT");
            // Entropy-coded segment: from here up to the first marker that is neither a stuffed
            // 0xFF00 nor an RSTn (fill bytes 0xFF before it included), as libjpeg's
            // next_marker() finds it.  Whatever follows EOI (MPF secondary images, gain maps,
            // appended thumbnails) is never part of the scan.
            const size_t e0 = i + seglen;
            size_t e1 = len;
            for (size_t q = e0; q + 1 < len;) {
                // the next 0xFF (memchr: vectorised, ~1 in 256 entropy bytes is one)
                const void *hit = memchr(buf + q, 0xFF, len - 1 - q);
                if (!hit) break;
                q = (size_t)((const uint8_t *)hit - buf);
                const uint8_t nx = buf[q + 1];
                if (nx == 0x00 || (nx >= 0xD0 && nx <= 0xD7)) { q += 2; continue; }
                e1 = q;
                break;
            }
            while (e1 > e0 && buf[e1 - 1] == 0xFF) --e1;
            P->ecs = buf + e0;
            P->ecs_len = e1 - e0;
            for (int c = 0; c < P->ncomp; ++c)
                if (!P->qt_ok[P->comp_q[c]]) return fail(err, PANO_E_ARG, "JPEG component without a quantisation table");
            return PANO_OK;
        }
        default:
            break;   // APPn, COM, DNL-free others: skipped as libjpeg skips them
        }
        i += seglen;
    }
}

int plan_frame(const Parsed &P, Frame *F, std::string *err) {
    memset(F, 0, sizeof(*F));
    F->h = P.h;
    F->w = P.w;
    F->ncomp = P.ncomp;
    if (P.ncomp == 1) {
        // A single-component scan is non-interleaved: one block per MCU over the component's
        // own block grid, whatever sampling factors the SOF declares (jdinput.c).
        F->hmax = F->vmax = 1;
        F->comp_h[0] = F->comp_v[0] = 1;
        F->mcus_x = (P.w + 7) / 8;
        F->mcus_y = (P.h + 7) / 8;
        F->bpm = 1;
        F->comp_bw[0] = F->mcus_x;
        F->comp_bh[0] = F->mcus_y;
        F->comp_dw[0] = P.w;
        F->comp_dh[0] = P.h;
        F->upsample = 0;
    } else {
        int hmax = 1, vmax = 1;
        for (int c = 0; c < P.ncomp; ++c) {
            hmax = P.comp_h[c] > hmax ? P.comp_h[c] : hmax;
            vmax = P.comp_v[c] > vmax ? P.comp_v[c] : vmax;
        }
        F->hmax = hmax;
        F->vmax = vmax;
        F->mcus_x = (P.w + 8 * hmax - 1) / (8 * hmax);
        F->mcus_y = (P.h + 8 * vmax - 1) / (8 * vmax);
        int b = 0;
        for (int c = 0; c < P.ncomp; ++c) {
            F->comp_h[c] = P.comp_h[c];
            F->comp_v[c] = P.comp_v[c];
            F->comp_bw[c] = F->mcus_x * P.comp_h[c];
            F->comp_bh[c] = F->mcus_y * P.comp_v[c];
            F->comp_dw[c] = (P.w * P.comp_h[c] + hmax - 1) / hmax;
            F->comp_dh[c] = (P.h * P.comp_v[c] + vmax - 1) / vmax;
            for (int by = 0; by < P.comp_v[c]; ++by)
                for (int bx = 0; bx < P.comp_h[c]; ++bx) {
                    if (b >= kMaxBpm) return fail(err, PANO_E_ARG, "JPEG MCU has more than 10 blocks");
                    F->mcu_comp[b] = (int8_t)c;
                    F->mcu_bx[b] = (int8_t)bx;
                    F->mcu_by[b] = (int8_t)by;
                    ++b;
                }
        }
        F->bpm = b;
        // Luma at the maximum sampling, both chroma planes at one ratio of it: 1x1 (4:4:4),
        // 2x1 (4:2:2, h2v1 fancy) or 2x2 (4:2:0, h2v2 fancy) -- jdsample.c jinit_upsampler.
        if (P.comp_h[0] != hmax || P.comp_v[0] != vmax || P.comp_h[1] != P.comp_h[2] || P.comp_v[1] != P.comp_v[2])
            return fail(err, PANO_E_UNSUPPORTED, "JPEG chroma sampling other than 4:4:4, 4:2:2 or 4:2:0");
        const int rh = hmax / P.comp_h[1], rv = vmax / P.comp_v[1];
        if (rh * P.comp_h[1] != hmax || rv * P.comp_v[1] != vmax)
            return fail(err, PANO_E_UNSUPPORTED, "JPEG chroma sampling other than 4:4:4, 4:2:2 or 4:2:0");
        if (rh == 1 && rv == 1) F->upsample = 0;
        else if (rh == 2 && rv == 1) F->upsample = 1;
        else if (rh == 2 && rv == 2) F->upsample = 2;
        else return fail(err, PANO_E_UNSUPPORTED, "JPEG chroma sampling other than 4:4:4, 4:2:2 or 4:2:0");
        // libjpeg switches to box upsampling when the chroma plane is <= 2 samples wide.
        if (F->upsample && F->comp_dw[1] <= 2) return fail(err, PANO_E_UNSUPPORTED, "JPEG narrower than 5 pixels");
    }
    F->total_blocks = F->mcus_x * F->mcus_y * F->bpm;
    // Warm-up window of the start search (jpeg.hip jpeg_sync_warm): ~3 MCUs' worth of bits
    // (PANO_JPEG_WARM_MCUS), in [2048, 16384].  A decode started at a wrong bit position
    // re-synchronises only when it also lands in the right block of the MCU, so the distance
    // scales with the bits per MCU.
    {
        const char *env = getenv("PANO_JPEG_WARM_MCUS");
        const uint64_t m = env && atoi(env) > 0 ? (uint64_t)atoi(env) : 3;   // measured: 3 MCUs 0.69 ms, 4 0.76, 2 0.72
        const uint64_t mcus = (uint64_t)F->mcus_x * F->mcus_y;
        const uint64_t wb = m * (uint64_t)P.ecs_len * 8 / (mcus ? mcus : 1);
        const uint64_t wr = (wb + kSubBits - 1) / kSubBits * kSubBits;
        F->warm = (uint32_t)(wr < 2048 ? 2048 : (wr > 16384 ? 16384 : wr));
    }
    if (P.restart > 0 && P.restart < F->mcus_x * F->mcus_y)
        return fail(err, PANO_E_UNSUPPORTED, "JPEG with restart intervals");
    return PANO_OK;
}

}  // namespace pj
