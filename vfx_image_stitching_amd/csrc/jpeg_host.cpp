// jpeg_host.cpp -- host half of the baseline JPEG decoder: marker parsing (the subset of
// libjpeg's jdmarker.c a sequential file needs), Huffman decode tables (jdhuff.c
// jpeg_make_d_derived_tbl restated) and the Annex K.3 standard tables.  Everything that
// touches pixels runs on the GPU (jpeg.hip); this file only reads headers.
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

bool make_huff(const uint8_t *bits17, const uint8_t *vals, Huff *T) {
    // jdhuff.c jpeg_make_d_derived_tbl: code lengths -> canonical codes, per-length maxcode and
    // value offsets, then the 9-bit lookahead table.
    int size[257], code[257];
    int p = 0;
    for (int l = 1; l <= 16; ++l) {
        if (p + bits17[l] > 256) return false;
        for (int i = 0; i < bits17[l]; ++i) size[p++] = l;
    }
    size[p] = 0;
    const int total = p;
    int c = 0, si = total ? size[0] : 0;
    p = 0;
    while (size[p]) {
        while (size[p] == si) code[p++] = c++;
        if (c >= (1 << si)) return false;     // JERR_BAD_HUFF_TABLE
        c <<= 1;
        ++si;
    }
    memset(T, 0, sizeof(*T));
    p = 0;
    for (int l = 1; l <= 16; ++l) {
        if (bits17[l]) {
            T->valoff[l] = p - code[p];
            p += bits17[l];
            T->maxcode[l] = code[p - 1];
        } else {
            T->maxcode[l] = -1;
        }
    }
    T->maxcode[17] = 0x7FFFFFFF;
    memcpy(T->vals, vals, (size_t)total);
    for (int i = 0; i < total; ++i) {
        const int l = size[i];
        if (l > 9) continue;
        const int lo = code[i] << (9 - l), hi = (code[i] + 1) << (9 - l);
        for (int e = lo; e < hi; ++e) T->lut[e] = (uint16_t)(l << 8 | vals[i]);
    }
    return true;
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
            // Entropy-coded segment: from here to the last EOI, without trailing fill bytes.
            const size_t e0 = i + seglen;
            size_t e1 = len;
            for (size_t q = len; q >= e0 + 2; --q)
                if (buf[q - 2] == 0xFF && buf[q - 1] == 0xD9) { e1 = q - 2; break; }
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
    // Warm-up window of the start search (jpeg.hip jpeg_sync_warm): ~8 MCUs' worth of bits,
    // in [4096, 32768].  A decode started at a wrong bit position re-synchronises only when it
    // also lands in the right block of the MCU, so the distance scales with the MCU size
    // (measured on the reference's frames: 0.1 % of subsequences need the fallback).
    {
        const uint64_t mcus = (uint64_t)F->mcus_x * F->mcus_y;
        const uint64_t w8 = 8 * (uint64_t)P.ecs_len * 8 / (mcus ? mcus : 1);
        const uint64_t wr = (w8 + kSubBits - 1) / kSubBits * kSubBits;
        F->warm = (uint32_t)(wr < 4096 ? 4096 : (wr > 32768 ? 32768 : wr));
    }
    if (P.restart > 0 && P.restart < F->mcus_x * F->mcus_y)
        return fail(err, PANO_E_UNSUPPORTED, "JPEG with restart intervals");
    return PANO_OK;
}

}  // namespace pj
