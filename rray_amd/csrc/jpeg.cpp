// jpeg.cpp — baseline (sequential Huffman) JPEG decoder for image textures (texture.rs:15-19:
// Texture::new decodes any image file, then to_rgba8).
//
// The reference decodes through the image crate 0.25 (its JPEG decoder is zune-jpeg, not vendored
// here); this decoder follows ITU-T T.81 with libjpeg's conventions for every step whose rounding is
// implementation-defined, so its texels are the libjpeg-turbo (PIL) decode bit for bit: the integer
// "islow" inverse DCT (13-bit constants, 2 extra pass-1 bits, the post-IDCT range-limit table),
// YCbCr -> RGB with 16-bit fixed-point tables, and the triangle ("fancy") chroma upsampling for
// h2v1 / h2v2 sampling (replication where the chroma row is 1-2 samples wide).  tests/test_jpeg.py pins it against PIL on the reference's own texture and
// on synthetic files (4:4:4 / 4:2:2 / 4:2:0 / grey, restart intervals, progressive, odd sizes).
//
// Scope: 8-bit Huffman-coded baseline, extended-sequential and progressive frames (SOF0 / SOF1 /
// SOF2), one or several scans, restart intervals, 1 (grey) or 3 components, sampling 1x1 for chroma
// with luma 1x1, 2x1 or 2x2.  Arithmetic-coded, lossless, hierarchical, 12-bit, CMYK and other
// sampling layouts return RR_E_LIMIT.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rray/rray.h"
#include "png.hpp"

namespace rr {
namespace {

const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Huff {
    bool present = false;
    // canonical code tables (T.81 Annex C): for each length l, codes [mincode[l], maxcode[l]]
    int32_t mincode[17] = {}, maxcode[18] = {}, valptr[17] = {};
    uint8_t vals[256] = {};
    // 9-bit lookahead: (length << 8) | symbol, 0 = longer code
    uint16_t fast[512] = {};
};

bool build_huff(Huff& h, const uint8_t counts[16], const uint8_t* vals, int nvals) {
    std::memcpy(h.vals, vals, nvals);
    int code = 0, k = 0;
    std::memset(h.fast, 0, sizeof h.fast);
    for (int l = 1; l <= 16; ++l) {
        h.valptr[l] = k;
        h.mincode[l] = code;
        for (int i = 0; i < counts[l - 1]; ++i, ++k, ++code) {
            // over-subscribed code (T.81 C.2): an l-bit code must stay below 2^l.  Checked before the
            // lookahead fill, whose index code << (9 - l) would otherwise run past fast[512]
            if (code >= (1 << l) || k >= nvals) return false;
            if (l <= 9) {
                int lo = code << (9 - l), n = 1 << (9 - l);
                for (int j = 0; j < n; ++j) h.fast[lo + j] = (uint16_t)((l << 8) | h.vals[k]);
            }
        }
        h.maxcode[l] = counts[l - 1] ? code - 1 : -1;
        if (code > (1 << l)) return false;  // over-subscribed code
        code <<= 1;
    }
    h.maxcode[17] = 0x7fffffff;
    h.present = true;
    return true;
}

struct Bits {
    const uint8_t* p;
    const uint8_t* end;
    uint64_t acc = 0;
    int n = 0;
    bool marker = false;  // hit a marker: feed zero bits (libjpeg's behaviour on truncated data)
    void fill() {
        while (n <= 56) {
            uint32_t b = 0;
            if (!marker && p < end) {
                b = *p;
                if (b == 0xFF) {
                    uint8_t nx = p + 1 < end ? p[1] : 0xD9;
                    if (nx == 0x00) {
                        p += 2;
                    } else {
                        marker = true;
                        b = 0;
                    }
                } else {
                    ++p;
                }
            }
            acc |= (uint64_t)b << (56 - n);
            n += 8;
        }
    }
    uint32_t peek(int k) {
        if (n < k) fill();
        return (uint32_t)(acc >> (64 - k));
    }
    void skip(int k) {
        acc <<= k;
        n -= k;
    }
    uint32_t get(int k) {
        if (k == 0) return 0;
        uint32_t v = peek(k);
        skip(k);
        return v;
    }
    int decode(const Huff& h) {
        uint32_t look = peek(9);
        uint16_t f = h.fast[look];
        if (f) {
            skip(f >> 8);
            return f & 0xFF;
        }
        uint32_t code = peek(16);
        for (int l = 10; l <= 16; ++l) {
            int32_t c = (int32_t)(code >> (16 - l));
            if (c <= h.maxcode[l]) {
                skip(l);
                return h.vals[h.valptr[l] + c - h.mincode[l]];
            }
        }
        skip(16);
        return -1;  // no such code: corrupt data
    }
    // restart marker: drop buffered bits, skip to after RSTn
    void restart() {
        acc = 0;
        n = 0;
        marker = false;
        while (p + 1 < end && !(p[0] == 0xFF && p[1] >= 0xD0 && p[1] <= 0xD7)) ++p;
        if (p + 1 < end) p += 2;
    }
};

inline int extend(uint32_t v, int s) { return s == 0 ? 0 : (v < (1u << (s - 1)) ? (int)v - (1 << s) + 1 : (int)v); }

struct Comp {
    int id, h, v, tq;
    int bw, bh;                  // blocks per row / column, padded to whole MCUs
    std::vector<int16_t> coef;   // bw * bh blocks of 64 natural-order coefficients
    int dc_pred = 0, td = 0, ta = 0;
};

// libjpeg jidctint.c jpeg_idct_islow: LL&M with CONST_BITS 13, PASS1_BITS 2; outputs through the
// post-IDCT range-limit table (x & 1023 indexing; jdmaster.c prepare_range_limit_table).
constexpr int CB = 13, P1 = 2;
constexpr int32_t F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633,
                  F1501 = 12299, F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;
inline int32_t descale(int64_t x, int n) { return (int32_t)((x + ((int64_t)1 << (n - 1))) >> n); }
inline uint8_t idct_limit(int32_t v) {
    int m = v & 1023;
    if (m < 128) return (uint8_t)(m + 128);
    if (m < 512) return 255;
    if (m < 896) return 0;
    return (uint8_t)(m - 896);
}

template <typename T>
inline void idct_1d(T c0, T c1, T c2, T c3, T c4, T c5, T c6, T c7, int64_t out[8]) {
    int64_t z2 = c2, z3 = c6;
    int64_t z1 = (z2 + z3) * F0541;
    int64_t tmp2 = z1 + z3 * (-F1847);
    int64_t tmp3 = z1 + z2 * F0765;
    z2 = c0;
    z3 = c4;
    int64_t tmp0 = (z2 + z3) * (1 << CB);
    int64_t tmp1 = (z2 - z3) * (1 << CB);
    int64_t t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    int64_t o0 = c7, o1 = c5, o2 = c3, o3 = c1;
    z1 = o0 + o3;
    z2 = o1 + o2;
    z3 = o0 + o2;
    int64_t z4 = o1 + o3;
    int64_t z5 = (z3 + z4) * F1175;
    o0 *= F0298;
    o1 *= F2053;
    o2 *= F3072;
    o3 *= F1501;
    z1 *= -F0899;
    z2 *= -F2562;
    z3 *= -F1961;
    z4 *= -F0390;
    z3 += z5;
    z4 += z5;
    o0 += z1 + z3;
    o1 += z2 + z4;
    o2 += z2 + z3;
    o3 += z1 + z4;
    out[0] = t10 + o3;
    out[7] = t10 - o3;
    out[1] = t11 + o2;
    out[6] = t11 - o2;
    out[2] = t12 + o1;
    out[5] = t12 - o1;
    out[3] = t13 + o0;
    out[4] = t13 - o0;
}

void idct_block(const int16_t* coef, const uint16_t* q, uint8_t* out, int stride) {
    int32_t ws[64];
    for (int c = 0; c < 8; ++c) {
        const int16_t* in = coef + c;
        bool ac0 = !in[8] && !in[16] && !in[24] && !in[32] && !in[40] && !in[48] && !in[56];
        if (ac0) {  // same value the full pass gives: (dc << 13 + 2^10) >> 11 == dc << 2
            int32_t dc = (int32_t)in[0] * q[c] * (1 << P1);
            for (int r = 0; r < 8; ++r) ws[r * 8 + c] = dc;
            continue;
        }
        int64_t o[8];
        idct_1d<int64_t>((int64_t)in[0] * q[c], (int64_t)in[8] * q[8 + c], (int64_t)in[16] * q[16 + c],
                         (int64_t)in[24] * q[24 + c], (int64_t)in[32] * q[32 + c], (int64_t)in[40] * q[40 + c],
                         (int64_t)in[48] * q[48 + c], (int64_t)in[56] * q[56 + c], o);
        for (int r = 0; r < 8; ++r) ws[r * 8 + c] = descale(o[r], CB - P1);
    }
    for (int r = 0; r < 8; ++r) {
        const int32_t* w = ws + r * 8;
        int64_t o[8];
        idct_1d<int64_t>(w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7], o);
        for (int c = 0; c < 8; ++c) out[r * stride + c] = idct_limit(descale(o[c], CB + P1 + 3));
    }
}

inline uint8_t clamp8(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

struct Decoder {
    const uint8_t* d;
    size_t len;
    std::string err;
    uint16_t qt[4][64] = {};
    bool qt_present[4] = {};
    Huff dc[4], ac[4];
    std::vector<Comp> comps;
    int width = 0, height = 0, hmax = 1, vmax = 1, mcux = 0, mcuy = 0, restart_interval = 0;
    bool frame = false, progressive = false, jfif = false, adobe = false;
    int adobe_transform = -1;

    int fail(int rc, const std::string& m) {
        err = m;
        return rc;
    }

    int read_sof(const uint8_t* p, int L) {
        if (L < 8 || p[0] != 8) return fail(RR_E_LIMIT, "JPEG sample precision other than 8 bits");
        height = (p[1] << 8) | p[2];
        width = (p[3] << 8) | p[4];
        int nc = p[5];
        if (width == 0 || height == 0) return fail(RR_E_LIMIT, "JPEG without image height (DNL) or width");
        if (nc != 1 && nc != 3) return fail(RR_E_LIMIT, "JPEG with other than 1 or 3 components (CMYK)");
        if (L < 6 + 3 * nc) return fail(RR_E_IO, "corrupt JPEG frame header");
        comps.resize(nc);
        for (int i = 0; i < nc; ++i) {
            Comp& c = comps[i];
            c.id = p[6 + 3 * i];
            c.h = p[7 + 3 * i] >> 4;
            c.v = p[7 + 3 * i] & 15;
            c.tq = p[8 + 3 * i] & 3;
            if (c.h < 1 || c.v < 1 || c.h > 4 || c.v > 4) return fail(RR_E_IO, "corrupt JPEG sampling factors");
            hmax = std::max(hmax, c.h);
            vmax = std::max(vmax, c.v);
        }
        if (nc == 3) {
            bool ok = comps[1].h == 1 && comps[1].v == 1 && comps[2].h == 1 && comps[2].v == 1 &&
                      ((comps[0].h == 1 && comps[0].v == 1) || (comps[0].h == 2 && comps[0].v == 1) ||
                       (comps[0].h == 2 && comps[0].v == 2));
            if (!ok) return fail(RR_E_LIMIT, "JPEG chroma sampling other than 4:4:4, 4:2:2 or 4:2:0");
        } else {
            hmax = vmax = comps[0].h = comps[0].v = 1;  // a lone component is never interleaved
        }
        mcux = (width + 8 * hmax - 1) / (8 * hmax);
        mcuy = (height + 8 * vmax - 1) / (8 * vmax);
        for (Comp& c : comps) {
            c.bw = mcux * c.h;
            c.bh = mcuy * c.v;
            c.coef.assign((size_t)c.bw * c.bh * 64, 0);
        }
        frame = true;
        return RR_OK;
    }

    int read_dht(const uint8_t* p, int L) {
        int i = 0;
        while (i + 17 <= L) {
            int tc = p[i] >> 4, th = p[i] & 15;
            if (tc > 1 || th > 3) return fail(RR_E_IO, "corrupt JPEG Huffman table");
            int total = 0;
            for (int k = 0; k < 16; ++k) total += p[i + 1 + k];
            if (total > 256 || i + 17 + total > L) return fail(RR_E_IO, "corrupt JPEG Huffman table");
            if (!build_huff(tc ? ac[th] : dc[th], p + i + 1, p + i + 17, total))
                return fail(RR_E_IO, "corrupt JPEG Huffman table");
            i += 17 + total;
        }
        return RR_OK;
    }

    int read_dqt(const uint8_t* p, int L) {
        int i = 0;
        while (i < L) {
            int pq = p[i] >> 4, tq = p[i] & 15;
            if (tq > 3 || pq > 1 || i + 1 + 64 * (pq + 1) > L) return fail(RR_E_IO, "corrupt JPEG quantisation table");
            for (int k = 0; k < 64; ++k)
                qt[tq][kZigzag[k]] = pq ? (uint16_t)((p[i + 1 + 2 * k] << 8) | p[i + 2 + 2 * k]) : p[i + 1 + k];
            qt_present[tq] = true;
            i += 1 + 64 * (pq + 1);
        }
        return RR_OK;
    }

    // sequential: one whole block (T.81 F.2.2)
    bool decode_block(Bits& b, Comp& c, int16_t* blk) {
        int s = b.decode(dc[c.td]);
        if (s < 0 || s > 11) return false;
        c.dc_pred += extend(b.get(s), s);
        blk[0] = (int16_t)c.dc_pred;
        for (int k = 1; k < 64;) {
            int rs = b.decode(ac[c.ta]);
            if (rs < 0) return false;
            int r = rs >> 4, sz = rs & 15;
            if (sz == 0) {
                if (r != 15) break;  // EOB
                k += 16;
                continue;
            }
            k += r;
            if (k > 63) return false;
            blk[kZigzag[k]] = (int16_t)extend(b.get(sz), sz);
            ++k;
        }
        return true;
    }

    // progressive (T.81 G.1.2; libjpeg jdphuff.c): DC first / refine, AC first / refine with EOB runs
    int ss = 0, se = 63, ah = 0, al = 0, eobrun = 0;
    bool decode_dc_first(Bits& b, Comp& c, int16_t* blk) {
        int s = b.decode(dc[c.td]);
        if (s < 0 || s > 11) return false;
        c.dc_pred += extend(b.get(s), s);
        blk[0] = (int16_t)(c.dc_pred * (1 << al));
        return true;
    }
    bool decode_dc_refine(Bits& b, Comp&, int16_t* blk) {
        if (b.get(1)) blk[0] = (int16_t)(blk[0] | (1 << al));
        return true;
    }
    bool decode_ac_first(Bits& b, Comp& c, int16_t* blk) {
        if (eobrun > 0) {
            --eobrun;
            return true;
        }
        for (int k = ss; k <= se; ++k) {
            int rs = b.decode(ac[c.ta]);
            if (rs < 0) return false;
            int r = rs >> 4, s = rs & 15;
            if (s) {
                k += r;
                if (k > 63) return false;
                blk[kZigzag[k]] = (int16_t)(extend(b.get(s), s) * (1 << al));
            } else if (r == 15) {
                k += 15;
            } else {
                eobrun = (1 << r) - 1;
                if (r) eobrun += (int)b.get(r);
                break;
            }
        }
        return true;
    }
    bool decode_ac_refine(Bits& b, Comp& c, int16_t* blk) {
        const int p1 = 1 << al, m1 = -(1 << al);
        auto correct = [&](int16_t& v) {  // a correction bit for an already nonzero coefficient
            if (b.get(1) && (v & p1) == 0) v = (int16_t)(v >= 0 ? v + p1 : v + m1);
        };
        int k = ss;
        if (eobrun == 0) {
            for (; k <= se; ++k) {
                int rs = b.decode(ac[c.ta]);
                if (rs < 0) return false;
                int r = rs >> 4, s = rs & 15, val = 0;
                if (s) {
                    val = b.get(1) ? p1 : m1;
                } else if (r != 15) {
                    eobrun = 1 << r;
                    if (r) eobrun += (int)b.get(r);
                    break;  // the rest of the band goes through the EOB-run pass below
                }
                // skip r zero-history coefficients, correcting the nonzero ones passed over
                for (; k <= se; ++k) {
                    int16_t& v = blk[kZigzag[k]];
                    if (v != 0) {
                        correct(v);
                    } else {
                        if (--r < 0) break;
                    }
                }
                if (val) {
                    if (k > 63) return false;
                    blk[kZigzag[k]] = (int16_t)val;
                }
            }
        }
        if (eobrun > 0) {
            for (; k <= se; ++k) {
                int16_t& v = blk[kZigzag[k]];
                if (v != 0) correct(v);
            }
            --eobrun;
        }
        return true;
    }

    // one scan (interleaved if several components); leaves pos at the next marker after its data
    int read_scan(const uint8_t* p, int L, size_t& pos) {
        if (!frame) return fail(RR_E_IO, "JPEG scan before the frame header");
        if (L < 1) return fail(RR_E_IO, "corrupt JPEG scan header");
        int ns = p[0];
        if (ns < 1 || ns > (int)comps.size() || L < 4 + 2 * ns) return fail(RR_E_IO, "corrupt JPEG scan header");
        ss = p[1 + 2 * ns];
        se = p[2 + 2 * ns];
        ah = p[3 + 2 * ns] >> 4;
        al = p[3 + 2 * ns] & 15;
        enum { SEQ, DC_FIRST, DC_REFINE, AC_FIRST, AC_REFINE } mode = SEQ;
        if (progressive) {
            bool ok = ss <= se && se <= 63 && al <= 13 && (ss == 0 ? se == 0 : ns == 1);
            if (!ok) return fail(RR_E_IO, "corrupt progressive JPEG scan parameters");
            mode = ss == 0 ? (ah ? DC_REFINE : DC_FIRST) : (ah ? AC_REFINE : AC_FIRST);
        } else if (ss != 0 || se != 63 || ah != 0 || al != 0) {
            return fail(RR_E_IO, "corrupt sequential JPEG scan parameters");
        }
        std::vector<Comp*> sc;
        for (int i = 0; i < ns; ++i) {
            Comp* c = nullptr;
            for (Comp& k : comps)
                if (k.id == p[1 + 2 * i]) c = &k;
            if (!c) return fail(RR_E_IO, "JPEG scan names an unknown component");
            c->td = p[2 + 2 * i] >> 4;
            c->ta = p[2 + 2 * i] & 15;
            bool need_dc = mode == SEQ || mode == DC_FIRST, need_ac = mode == SEQ || mode == AC_FIRST || mode == AC_REFINE;
            if (c->td > 3 || c->ta > 3 || (need_dc && !dc[c->td].present) || (need_ac && !ac[c->ta].present))
                return fail(RR_E_IO, "JPEG scan uses a missing Huffman table");
            if (!qt_present[c->tq]) return fail(RR_E_IO, "JPEG component uses a missing quantisation table");
            c->dc_pred = 0;
            sc.push_back(c);
        }
        eobrun = 0;
        Bits b{d + pos, d + len};
        auto block = [&](Comp& c, int16_t* blk) {
            switch (mode) {
                case SEQ: return decode_block(b, c, blk);
                case DC_FIRST: return decode_dc_first(b, c, blk);
                case DC_REFINE: return decode_dc_refine(b, c, blk);
                case AC_FIRST: return decode_ac_first(b, c, blk);
                default: return decode_ac_refine(b, c, blk);
            }
        };
        int todo = restart_interval;
        auto restart = [&]() {
            if (restart_interval && todo == 0) {
                b.restart();
                for (Comp* c : sc) c->dc_pred = 0;
                eobrun = 0;
                todo = restart_interval;
            }
        };
        if (ns == 1) {  // non-interleaved: the component's own block grid, ceil(size / 8) blocks
            Comp& c = *sc[0];
            int bx = (((width * c.h + hmax - 1) / hmax) + 7) / 8, by = (((height * c.v + vmax - 1) / vmax) + 7) / 8;
            for (int y = 0; y < by; ++y)
                for (int x = 0; x < bx; ++x) {
                    restart();
                    if (!block(c, &c.coef[((size_t)y * c.bw + x) * 64]))
                        return fail(RR_E_IO, "corrupt JPEG entropy-coded data");
                    --todo;
                }
        } else {
            for (int my = 0; my < mcuy; ++my)
                for (int mx = 0; mx < mcux; ++mx) {
                    restart();
                    for (Comp* c : sc)
                        for (int v = 0; v < c->v; ++v)
                            for (int h = 0; h < c->h; ++h) {
                                size_t blk = (size_t)(my * c->v + v) * c->bw + (size_t)mx * c->h + h;
                                if (!block(*c, &c->coef[blk * 64])) return fail(RR_E_IO, "corrupt JPEG entropy-coded data");
                            }
                    --todo;
                }
        }
        const uint8_t* q = b.p;  // the next marker that is not a restart marker
        while (q + 1 < d + len && !(q[0] == 0xFF && q[1] != 0x00 && !(q[1] >= 0xD0 && q[1] <= 0xD7))) ++q;
        pos = (size_t)(q - d);
        return RR_OK;
    }

    int run(std::vector<uint8_t>& rgba, uint32_t& w, uint32_t& h) {
        if (len < 4 || d[0] != 0xFF || d[1] != 0xD8) return fail(RR_E_IO, "not a JPEG file");
        size_t pos = 2;
        bool scanned = false;
        while (true) {
            while (pos < len && d[pos] != 0xFF) ++pos;  // tolerate fill / garbage between segments
            while (pos < len && d[pos] == 0xFF) ++pos;
            if (pos >= len) break;
            uint8_t m = d[pos++];
            if (m == 0xD9) break;                          // EOI
            if (m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;
            if (pos + 2 > len) return fail(RR_E_IO, "truncated JPEG");
            int L = (d[pos] << 8) | d[pos + 1];
            if (L < 2 || pos + L > len) return fail(RR_E_IO, "truncated JPEG segment");
            const uint8_t* p = d + pos + 2;
            int n = L - 2;
            pos += L;
            int rc = RR_OK;
            switch (m) {
                case 0xC0:
                case 0xC1:
                    if (frame) return fail(RR_E_IO, "JPEG with two frame headers");
                    rc = read_sof(p, n);
                    break;
                case 0xC2:
                    if (frame) return fail(RR_E_IO, "JPEG with two frame headers");
                    progressive = true;
                    rc = read_sof(p, n);
                    break;
                case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xC9: case 0xCA: case 0xCB:
                case 0xCD: case 0xCE: case 0xCF:
                    return fail(RR_E_LIMIT, "JPEG process other than Huffman-coded sequential or progressive "
                                            "(lossless, hierarchical or arithmetic-coded)");
                case 0xC4: rc = read_dht(p, n); break;
                case 0xDB: rc = read_dqt(p, n); break;
                case 0xDD:
                    if (n < 2) return fail(RR_E_IO, "corrupt JPEG restart interval");
                    restart_interval = (p[0] << 8) | p[1];
                    break;
                case 0xDA:
                    rc = read_scan(p, n, pos);
                    scanned = true;
                    break;
                case 0xE0:
                    if (n >= 5 && !std::memcmp(p, "JFIF\0", 5)) jfif = true;
                    break;
                case 0xEE:
                    if (n >= 12 && !std::memcmp(p, "Adobe", 5)) {
                        adobe = true;
                        adobe_transform = p[11];
                    }
                    break;
                default: break;
            }
            if (rc != RR_OK) return rc;
        }
        if (!frame || !scanned) return fail(RR_E_IO, "JPEG without image data");
        return output(rgba, w, h);
    }

    // jdapimin.c default_decompress_parms: is a 3-component file YCbCr or RGB?
    bool is_ycc() const {
        if (jfif) return true;
        if (adobe) return adobe_transform != 0;
        return !(comps[0].id == 'R' && comps[1].id == 'G' && comps[2].id == 'B');
    }

    int output(std::vector<uint8_t>& rgba, uint32_t& w, uint32_t& h) {
        // IDCT every component into its padded sample plane
        std::vector<std::vector<uint8_t>> plane(comps.size());
        for (size_t i = 0; i < comps.size(); ++i) {
            Comp& c = comps[i];
            int pw = c.bw * 8;
            plane[i].assign((size_t)pw * c.bh * 8, 0);
            for (int by = 0; by < c.bh; ++by)
                for (int bx = 0; bx < c.bw; ++bx)
                    idct_block(&c.coef[((size_t)by * c.bw + bx) * 64], qt[c.tq], &plane[i][((size_t)by * 8) * pw + bx * 8], pw);
        }
        w = (uint32_t)width;
        h = (uint32_t)height;
        rgba.assign((size_t)width * height * 4, 255);
        if (comps.size() == 1) {
            int pw = comps[0].bw * 8;
            for (int y = 0; y < height; ++y)
                for (int x = 0; x < width; ++x) {
                    uint8_t g = plane[0][(size_t)y * pw + x];
                    uint8_t* o = &rgba[4 * ((size_t)y * width + x)];
                    o[0] = o[1] = o[2] = g;
                }
            return RR_OK;
        }
        // chroma at full resolution (jdsample.c h2v1 / h2v2 fancy upsampling; 4:4:4 as is)
        const int lw = comps[0].bw * 8;
        const int cw = comps[1].bw * 8, ch = comps[1].bh * 8;
        const int cols = (width + hmax - 1) / hmax;  // chroma samples per row that carry image data
        std::vector<uint8_t> up[2];
        for (int k = 0; k < 2; ++k) {
            const std::vector<uint8_t>& src = plane[1 + k];
            if (hmax == 1) {
                up[k] = src;
                continue;
            }
            std::vector<uint8_t>& dst = up[k];
            dst.assign((size_t)lw * height, 0);
            const int rows = (height + vmax - 1) / vmax;
            for (int y = 0; y < height; ++y) {
                uint8_t* o = &dst[(size_t)y * lw];
                if (cols <= 2) {  // jdsample.c: fancy only for downsampled_width > 2, else replication
                    const uint8_t* in = &src[(size_t)(y / vmax) * cw];
                    for (int x = 0; x < cols; ++x) o[2 * x] = o[2 * x + 1] = in[x];
                } else if (vmax == 1) {  // h2v1: (3 * this + neighbour + 1 | 2) >> 2
                    const uint8_t* in = &src[(size_t)y * cw];
                    o[0] = in[0];
                    o[1] = (uint8_t)((in[0] * 3 + in[1] + 2) >> 2);
                    for (int x = 1; x < cols - 1; ++x) {
                        o[2 * x] = (uint8_t)((in[x] * 3 + in[x - 1] + 1) >> 2);
                        o[2 * x + 1] = (uint8_t)((in[x] * 3 + in[x + 1] + 2) >> 2);
                    }
                    int x = cols - 1;
                    o[2 * x] = (uint8_t)((in[x] * 3 + in[x - 1] + 1) >> 2);
                    o[2 * x + 1] = in[x];
                } else {  // h2v2: vertical 3:1 column sums, then horizontal triangle with 8 / 7 bias
                    int cy = y >> 1;
                    int ny = (y & 1) ? cy + 1 : cy - 1;  // the farther input row for this output row
                    // libjpeg uses the (padded) neighbouring row groups at the image edges: rows of the
                    // component's own plane past its data are edge-replicated by the decoder's context
                    ny = std::min(std::max(ny, 0), std::max(rows - 1, 0));
                    if (ny >= ch) ny = ch - 1;
                    const uint8_t* i0 = &src[(size_t)cy * cw];
                    const uint8_t* i1 = &src[(size_t)ny * cw];
                    auto colsum = [&](int x) { return (int)i0[x] * 3 + i1[x]; };
                    int t = colsum(0), nx = colsum(1), last;
                    o[0] = (uint8_t)((t * 4 + 8) >> 4);
                    o[1] = (uint8_t)((t * 3 + nx + 7) >> 4);
                    last = t;
                    t = nx;
                    for (int x = 1; x < cols - 1; ++x) {
                        nx = colsum(x + 1);
                        o[2 * x] = (uint8_t)((t * 3 + last + 8) >> 4);
                        o[2 * x + 1] = (uint8_t)((t * 3 + nx + 7) >> 4);
                        last = t;
                        t = nx;
                    }
                    int x = cols - 1;
                    o[2 * x] = (uint8_t)((t * 3 + last + 8) >> 4);
                    o[2 * x + 1] = (uint8_t)((t * 4 + 7) >> 4);
                }
            }
        }
        const int uw = hmax == 1 ? cw : lw;
        const bool ycc = is_ycc();
        // jdcolor.c ycc_rgb_convert: SCALEBITS 16 tables
        constexpr int32_t ONE_HALF = 1 << 15, FR = 91881, FB = 116130, FGR = 46802, FGB = 22554;
        for (int y = 0; y < height; ++y)
            for (int x = 0; x < width; ++x) {
                int Y = plane[0][(size_t)y * lw + x];
                int cb = up[0][(size_t)y * uw + x], cr = up[1][(size_t)y * uw + x];
                uint8_t* o = &rgba[4 * ((size_t)y * width + x)];
                if (!ycc) {
                    o[0] = (uint8_t)Y;
                    o[1] = (uint8_t)cb;
                    o[2] = (uint8_t)cr;
                    continue;
                }
                int xr = cr - 128, xb = cb - 128;
                int r = Y + (int)((FR * xr + ONE_HALF) >> 16);
                int g = Y + (int)(((-FGB) * xb + ONE_HALF + (-FGR) * xr) >> 16);
                int b = Y + (int)((FB * xb + ONE_HALF) >> 16);
                o[0] = clamp8(r);
                o[1] = clamp8(g);
                o[2] = clamp8(b);
            }
        return RR_OK;
    }
};
}  // namespace

int decode_jpeg_rgba(const uint8_t* data, size_t len, std::vector<uint8_t>& rgba, uint32_t& width,
                     uint32_t& height, std::string& err) {
    Decoder dec{data, len};
    int rc = dec.run(rgba, width, height);
    if (rc != RR_OK) err = dec.err;
    return rc;
}
}  // namespace rr
