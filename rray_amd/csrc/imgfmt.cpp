// imgfmt.cpp — the texture formats besides PNG and JPEG that the reference's `image::open` decodes with its default
// features (texture.rs:15-19: image::open(path).to_rgba8()): BMP, TGA, PNM (P1-P6) and GIF (first frame).  Every
// decoder produces RGBA8 rows top to bottom, as to_rgba8 does; the sampler reads the RGB channels.  Parity: the
// 8-bit layouts are checked against PIL's decoding of generated files (tests/test_abi_host.py); samples of other
// widths (16-bit BMP, TGA) are scaled by round(v * 255 / (2^n - 1)), the image crate's lookup tables — unpinned.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rray/rray.h"
#include "png.hpp"

namespace rr {
namespace {

constexpr uint64_t kMaxTexels = 1ull << 28;  // a texture's texel limit (1 GiB of RGBA8), as for PNG

uint32_t le16(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8; }
uint32_t le32(const uint8_t* p) { return le16(p) | le16(p + 2) << 16; }
uint8_t scale_bits(uint32_t v, uint32_t max) { return max == 255 ? (uint8_t)v : (uint8_t)((v * 255 + max / 2) / max); }

int fail(std::string& err, int code, const std::string& msg) {
    err = msg;
    return code;
}

// a channel of a BMP bitfield mask: the value's bits under the mask, shifted down, scaled to 8 bits
struct Field {
    uint32_t mask = 0, shift = 0, max = 0;
    explicit Field(uint32_t m = 0) : mask(m) {
        if (!m) return;
        while (!((m >> shift) & 1u)) ++shift;
        max = m >> shift;
    }
    uint8_t get(uint32_t v) const { return mask ? scale_bits((v & mask) >> shift, max) : 0; }
};

bool contiguous(uint32_t m) {
    if (!m) return true;
    while (!(m & 1u)) m >>= 1;
    return (m & (m + 1)) == 0 && m <= 0xffffu;
}

}  // namespace

// BMP: BITMAPCOREHEADER and BITMAPINFOHEADER (and its V4 / V5 extensions); 1 / 4 / 8-bit palettes, 16 / 24 / 32-bit
// BI_RGB and BI_BITFIELDS; bottom-up or top-down rows, padded to 4 bytes.  RLE-compressed bitmaps return RR_E_LIMIT.
int decode_bmp_rgba(const uint8_t* d, size_t n, std::vector<uint8_t>& rgba, uint32_t& width, uint32_t& height,
                    std::string& err) {
    if (n < 26 || d[0] != 'B' || d[1] != 'M') return fail(err, RR_E_IO, "not a BMP file");
    const uint32_t data_off = le32(d + 10), hsize = le32(d + 14);
    if (hsize != 12 && hsize < 40) return fail(err, RR_E_LIMIT, "BMP header version outside the decoder");
    if (14 + (size_t)hsize > n) return fail(err, RR_E_IO, "truncated BMP header");
    int64_t w, h;
    uint32_t bpp, comp = 0, ncolors = 0;
    if (hsize == 12) {
        w = le16(d + 18);
        h = (int16_t)le16(d + 20);
        bpp = le16(d + 24);
    } else {
        w = (int32_t)le32(d + 18);
        h = (int32_t)le32(d + 22);
        bpp = le16(d + 28);
        comp = le32(d + 30);
        ncolors = le32(d + 46);
    }
    const bool top_down = h < 0;
    if (h < 0) h = -h;
    if (w <= 0 || h <= 0 || w > 65535 || h > 65535 || (uint64_t)w * (uint64_t)h > kMaxTexels)
        return fail(err, RR_E_LIMIT, "BMP size outside 1..65535 or above 2^28 texels");
    if (comp != 0 && comp != 3 && comp != 6) return fail(err, RR_E_LIMIT, "RLE / JPEG / PNG-compressed BMP");
    uint32_t rm = 0, gm = 0, bm = 0;
    if (bpp == 16) {
        rm = 0x7c00, gm = 0x03e0, bm = 0x001f;  // BI_RGB 16-bit: 5-5-5
    } else if (bpp == 32 || bpp == 24) {
        rm = 0xff0000, gm = 0x00ff00, bm = 0x0000ff;
    }
    if (comp == 3 || comp == 6) {
        if (bpp != 16 && bpp != 32) return fail(err, RR_E_IO, "BMP bitfields need 16 or 32 bits per pixel");
        const size_t mo = hsize >= 52 ? 14 + 40 : 14 + hsize;  // V2+ headers hold the masks, v1 follows with them
        if (mo + 12 > n) return fail(err, RR_E_IO, "truncated BMP masks");
        rm = le32(d + mo), gm = le32(d + mo + 4), bm = le32(d + mo + 8);
        if (!contiguous(rm) || !contiguous(gm) || !contiguous(bm))
            return fail(err, RR_E_LIMIT, "BMP bitfield masks outside the decoder");
    }
    std::vector<uint8_t> pal;
    if (bpp <= 8) {
        if (bpp != 1 && bpp != 4 && bpp != 8) return fail(err, RR_E_IO, "BMP bit depth");
        const uint32_t entry = hsize == 12 ? 3 : 4, count = ncolors ? ncolors : (1u << bpp);
        const size_t po = 14 + hsize;
        if (count > 256 || po + (size_t)count * entry > n) return fail(err, RR_E_IO, "truncated BMP palette");
        for (uint32_t i = 0; i < count; ++i) pal.insert(pal.end(), {d[po + i * entry + 2], d[po + i * entry + 1], d[po + i * entry]});
    } else if (bpp != 16 && bpp != 24 && bpp != 32) {
        return fail(err, RR_E_IO, "BMP bit depth");
    }
    const size_t stride = (((size_t)w * bpp + 31) / 32) * 4;
    if ((size_t)data_off + stride * (size_t)h > n) return fail(err, RR_E_IO, "truncated BMP pixel data");
    const Field fr(rm), fg(gm), fb(bm);
    rgba.assign((size_t)w * h * 4, 255);
    for (int64_t y = 0; y < h; ++y) {
        const uint8_t* row = d + data_off + stride * (size_t)(top_down ? y : h - 1 - y);
        for (int64_t x = 0; x < w; ++x) {
            uint8_t* o = &rgba[4 * ((size_t)y * w + x)];
            if (bpp <= 8) {
                const size_t bit = (size_t)x * bpp;
                const uint32_t v = (row[bit / 8] >> (8 - bpp - bit % 8)) & ((1u << bpp) - 1);
                if (3 * (size_t)v + 2 >= pal.size()) return fail(err, RR_E_IO, "BMP palette index out of range");
                std::memcpy(o, &pal[3 * v], 3);
            } else if (bpp == 24) {
                o[0] = row[3 * x + 2], o[1] = row[3 * x + 1], o[2] = row[3 * x];
            } else {
                const uint32_t v = bpp == 16 ? le16(row + 2 * x) : le32(row + 4 * x);
                o[0] = fr.get(v), o[1] = fg.get(v), o[2] = fb.get(v);
            }
        }
    }
    width = (uint32_t)w;
    height = (uint32_t)h;
    return RR_OK;
}

// TGA: colour-mapped (1 / 9), true-colour (2 / 10) and grey (3 / 11), raw or run-length encoded; 8-bit grey,
// 15 / 16 / 24 / 32-bit BGR(A) pixels and palette entries; the image origin bit (top or bottom rows first) and the
// right-to-left bit.
int decode_tga_rgba(const uint8_t* d, size_t n, std::vector<uint8_t>& rgba, uint32_t& width, uint32_t& height,
                    std::string& err) {
    if (n < 18) return fail(err, RR_E_IO, "truncated TGA header");
    const uint32_t idlen = d[0], cmtype = d[1], type = d[2];
    const uint32_t cm_first = le16(d + 3), cm_len = le16(d + 5), cm_bits = d[7];
    const uint32_t w = le16(d + 12), h = le16(d + 14), bits = d[16], desc = d[17];
    const uint32_t base = type & 7u;
    if (!(base == 1 || base == 2 || base == 3) || (type & ~0xbu) != 0) return fail(err, RR_E_LIMIT, "TGA image type");
    if (w == 0 || h == 0) return fail(err, RR_E_IO, "TGA of zero size");
    if ((uint64_t)w * h > kMaxTexels) return fail(err, RR_E_LIMIT, "TGA above 2^28 texels");
    const bool rle = (type & 8u) != 0;
    size_t pos = 18 + idlen;
    const auto px_bgr = [](const uint8_t* p, uint32_t nbits, uint8_t* o) {
        if (nbits == 15 || nbits == 16) {
            const uint32_t v = le16(p);
            o[0] = scale_bits((v >> 10) & 31u, 31), o[1] = scale_bits((v >> 5) & 31u, 31), o[2] = scale_bits(v & 31u, 31);
        } else {
            o[0] = p[2], o[1] = p[1], o[2] = p[0];
        }
    };
    std::vector<uint8_t> cmap;
    if (cmtype == 1) {
        const uint32_t eb = (cm_bits + 7) / 8;
        if (!(cm_bits == 15 || cm_bits == 16 || cm_bits == 24 || cm_bits == 32)) return fail(err, RR_E_LIMIT, "TGA palette entry size");
        if (pos + (size_t)cm_len * eb > n) return fail(err, RR_E_IO, "truncated TGA palette");
        cmap.resize((size_t)(cm_first + cm_len) * 3, 0);
        for (uint32_t i = 0; i < cm_len; ++i) px_bgr(d + pos + (size_t)i * eb, cm_bits, &cmap[3 * (size_t)(cm_first + i)]);
        pos += (size_t)cm_len * eb;
    } else if (cmtype != 0) {
        return fail(err, RR_E_LIMIT, "TGA colour-map type");
    }
    if (base == 1 && (cmtype != 1 || (bits != 8 && bits != 16))) return fail(err, RR_E_IO, "TGA colour-mapped layout");
    if (base == 2 && !(bits == 15 || bits == 16 || bits == 24 || bits == 32)) return fail(err, RR_E_LIMIT, "TGA pixel size");
    if (base == 3 && bits != 8) return fail(err, RR_E_LIMIT, "TGA grey pixel size");
    const uint32_t bpp = (bits + 7) / 8;
    // the pixels in file order, decoded to RGB
    std::vector<uint8_t> pix((size_t)w * h * 3);
    const auto decode = [&](const uint8_t* p, uint8_t* o) -> bool {
        if (base == 1) {
            const uint32_t idx = bpp == 1 ? p[0] : le16(p);
            if (3 * (size_t)idx + 2 >= cmap.size()) return false;
            std::memcpy(o, &cmap[3 * (size_t)idx], 3);
        } else if (base == 3) {
            o[0] = o[1] = o[2] = p[0];
        } else {
            px_bgr(p, bits, o);
        }
        return true;
    };
    for (size_t i = 0, total = (size_t)w * h; i < total;) {
        if (!rle) {
            if (pos + bpp > n || !decode(d + pos, &pix[3 * i])) return fail(err, RR_E_IO, "truncated or bad TGA pixel data");
            pos += bpp;
            ++i;
            continue;
        }
        if (pos >= n) return fail(err, RR_E_IO, "truncated TGA run");
        const uint32_t hdr = d[pos++], count = (hdr & 0x7fu) + 1;
        if (i + count > total) return fail(err, RR_E_IO, "TGA run past the image");
        for (uint32_t k = 0; k < count; ++k) {
            const size_t src = (hdr & 0x80u) ? pos : pos + (size_t)k * bpp;
            if (src + bpp > n || !decode(d + src, &pix[3 * (i + k)])) return fail(err, RR_E_IO, "truncated TGA run");
        }
        pos += (hdr & 0x80u) ? bpp : (size_t)count * bpp;
        i += count;
    }
    const bool top = (desc & 0x20u) != 0, rtl = (desc & 0x10u) != 0;
    rgba.assign((size_t)w * h * 4, 255);
    for (uint32_t y = 0; y < h; ++y)
        for (uint32_t x = 0; x < w; ++x) {
            const size_t sy = top ? y : h - 1 - y, sx = rtl ? w - 1 - x : x;
            std::memcpy(&rgba[4 * ((size_t)y * w + x)], &pix[3 * (sy * w + sx)], 3);
        }
    width = w;
    height = h;
    return RR_OK;
}

// PNM: P1 / P4 bitmaps (1 = black), P2 / P5 grey and P3 / P6 RGB with maxval 255 (other maxvals return RR_E_LIMIT).
int decode_pnm_rgba(const uint8_t* d, size_t n, std::vector<uint8_t>& rgba, uint32_t& width, uint32_t& height,
                    std::string& err) {
    if (n < 3 || d[0] != 'P' || d[1] < '1' || d[1] > '6') return fail(err, RR_E_IO, "not a PNM file");
    const int kind = d[1] - '0';
    size_t pos = 2;
    const auto skip_ws = [&]() {
        for (;;) {
            while (pos < n && (d[pos] == ' ' || d[pos] == '\t' || d[pos] == '\n' || d[pos] == '\r' || d[pos] == '\v' ||
                               d[pos] == '\f'))
                ++pos;
            if (pos < n && d[pos] == '#') {
                while (pos < n && d[pos] != '\n' && d[pos] != '\r') ++pos;
                continue;
            }
            return;
        }
    };
    const auto number = [&](uint32_t& v) -> bool {
        skip_ws();
        if (pos >= n || d[pos] < '0' || d[pos] > '9') return false;
        uint64_t x = 0;
        while (pos < n && d[pos] >= '0' && d[pos] <= '9') {
            x = x * 10 + (d[pos++] - '0');
            if (x > 0xffffffffull) return false;
        }
        v = (uint32_t)x;
        return true;
    };
    uint32_t w = 0, h = 0, maxval = 1;
    if (!number(w) || !number(h) || (kind != 1 && kind != 4 && !number(maxval))) return fail(err, RR_E_IO, "bad PNM header");
    if (w == 0 || h == 0 || (uint64_t)w * h > kMaxTexels) return fail(err, RR_E_LIMIT, "PNM size");
    if (kind != 1 && kind != 4 && maxval != 255) return fail(err, RR_E_LIMIT, "PNM maxval other than 255");
    const bool binary = kind >= 4;
    if (binary) ++pos;  // the single whitespace byte after the header
    rgba.assign((size_t)w * h * 4, 255);
    const int ch = (kind == 3 || kind == 6) ? 3 : 1;
    for (uint32_t y = 0; y < h; ++y) {
        for (uint32_t x = 0; x < w; ++x) {
            uint8_t* o = &rgba[4 * ((size_t)y * w + x)];
            uint32_t v[3] = {0, 0, 0};
            if (kind == 4) {
                const size_t at = pos + (size_t)y * ((w + 7) / 8) + x / 8;
                if (at >= n) return fail(err, RR_E_IO, "truncated PNM data");
                v[0] = ((d[at] >> (7 - x % 8)) & 1u) ? 0u : 255u;
            } else if (kind == 1) {
                skip_ws();
                if (pos >= n || (d[pos] != '0' && d[pos] != '1')) return fail(err, RR_E_IO, "bad PBM sample");
                v[0] = d[pos++] == '1' ? 0u : 255u;
            } else {
                for (int c = 0; c < ch; ++c) {
                    if (binary) {
                        if (pos >= n) return fail(err, RR_E_IO, "truncated PNM data");
                        v[c] = d[pos++];
                    } else if (!number(v[c]) || v[c] > maxval) {
                        return fail(err, RR_E_IO, "bad PNM sample");
                    }
                }
            }
            if (ch == 1) v[1] = v[2] = v[0];
            o[0] = (uint8_t)v[0], o[1] = (uint8_t)v[1], o[2] = (uint8_t)v[2];
        }
    }
    width = w;
    height = h;
    return RR_OK;
}

// GIF (87a / 89a): the first image of the file on the logical screen, as image's GifDecoder gives it (frame pixels
// at the frame's offset, the rest of the screen and transparent pixels (0, 0, 0, 0)); local or global colour table,
// interlaced rows.
int decode_gif_rgba(const uint8_t* d, size_t n, std::vector<uint8_t>& rgba, uint32_t& width, uint32_t& height,
                    std::string& err) {
    if (n < 13 || std::memcmp(d, "GIF8", 4) != 0) return fail(err, RR_E_IO, "not a GIF file");
    const uint32_t sw = le16(d + 6), sh = le16(d + 8), flags = d[10];
    size_t pos = 13;
    std::vector<uint8_t> gct;
    if (flags & 0x80u) {
        const size_t sz = 3u << ((flags & 7u) + 1);
        if (pos + sz > n) return fail(err, RR_E_IO, "truncated GIF colour table");
        gct.assign(d + pos, d + pos + sz);
        pos += sz;
    }
    int transparent = -1;
    for (;;) {
        if (pos >= n) return fail(err, RR_E_IO, "GIF without an image");
        const uint8_t b = d[pos++];
        if (b == 0x3b) return fail(err, RR_E_IO, "GIF without an image");
        if (b == 0x21) {  // extension: graphic control (transparency) or skipped
            if (pos >= n) return fail(err, RR_E_IO, "truncated GIF extension");
            const uint8_t label = d[pos++];
            bool first = true;
            for (;;) {
                if (pos >= n) return fail(err, RR_E_IO, "truncated GIF extension");
                const uint32_t len = d[pos++];
                if (len == 0) break;
                if (pos + len > n) return fail(err, RR_E_IO, "truncated GIF extension");
                if (label == 0xf9 && first && len >= 4) transparent = (d[pos] & 1u) ? d[pos + 3] : -1;
                first = false;
                pos += len;
            }
            continue;
        }
        if (b != 0x2c) return fail(err, RR_E_IO, "bad GIF block");
        break;
    }
    if (pos + 9 > n) return fail(err, RR_E_IO, "truncated GIF image descriptor");
    const uint32_t fx = le16(d + pos), fy = le16(d + pos + 2), fw = le16(d + pos + 4), fh = le16(d + pos + 6);
    const uint32_t iflags = d[pos + 8];
    pos += 9;
    // the frame's own size bounds the LZW output buffer: checked before anything is allocated for it
    if (fw == 0 || fh == 0 || (uint64_t)fw * fh > kMaxTexels) return fail(err, RR_E_LIMIT, "GIF frame size");
    std::vector<uint8_t> lct;
    if (iflags & 0x80u) {
        const size_t sz = 3u << ((iflags & 7u) + 1);
        if (pos + sz > n) return fail(err, RR_E_IO, "truncated GIF colour table");
        lct.assign(d + pos, d + pos + sz);
        pos += sz;
    }
    const std::vector<uint8_t>& ct = lct.empty() ? gct : lct;
    if (ct.empty()) return fail(err, RR_E_IO, "GIF image without a colour table");
    if (pos >= n) return fail(err, RR_E_IO, "truncated GIF image data");
    const uint32_t min_code = d[pos++];
    if (min_code < 2 || min_code > 11) return fail(err, RR_E_IO, "bad GIF LZW code size");
    std::vector<uint8_t> lzw;
    for (;;) {
        if (pos >= n) return fail(err, RR_E_IO, "truncated GIF image data");
        const uint32_t len = d[pos++];
        if (len == 0) break;
        if (pos + len > n) return fail(err, RR_E_IO, "truncated GIF image data");
        lzw.insert(lzw.end(), d + pos, d + pos + len);
        pos += len;
    }
    // LZW (variable code width 3..12, clear and end codes)
    const size_t npx = (size_t)fw * fh;
    std::vector<uint8_t> idx;
    idx.reserve(npx);
    const uint32_t clear = 1u << min_code, eoi = clear + 1;
    std::vector<uint16_t> prefix(4096);
    std::vector<uint8_t> suffix(4096), stack;
    uint32_t width_bits = min_code + 1, next = clear + 2, prev = 0xffff;
    uint8_t first_char = 0;
    uint64_t acc = 0;
    uint32_t nacc = 0;
    size_t bp = 0;
    for (uint32_t i = 0; i < clear; ++i) suffix[i] = (uint8_t)i;
    while (idx.size() < npx) {
        while (nacc < width_bits && bp < lzw.size()) acc |= (uint64_t)lzw[bp++] << nacc, nacc += 8;
        if (nacc < width_bits) break;
        const uint32_t code = (uint32_t)(acc & ((1u << width_bits) - 1));
        acc >>= width_bits;
        nacc -= width_bits;
        if (code == clear) {
            width_bits = min_code + 1;
            next = clear + 2;
            prev = 0xffff;
            continue;
        }
        if (code == eoi) break;
        if (prev == 0xffff) {
            if (code >= clear) return fail(err, RR_E_IO, "bad GIF LZW stream");
            idx.push_back((uint8_t)code);
            prev = code;
            first_char = (uint8_t)code;
            continue;
        }
        uint32_t cur = code;
        stack.clear();
        if (code >= next) {
            if (code != next) return fail(err, RR_E_IO, "bad GIF LZW stream");
            stack.push_back(first_char);
            cur = prev;
        }
        while (cur >= clear) {
            stack.push_back(suffix[cur]);
            cur = prefix[cur];
        }
        stack.push_back((uint8_t)cur);
        first_char = (uint8_t)cur;
        for (size_t k = stack.size(); k-- > 0 && idx.size() < npx;) idx.push_back(stack[k]);
        if (next < 4096) {
            prefix[next] = (uint16_t)prev;
            suffix[next] = first_char;
            ++next;
            if (next == (1u << width_bits) && width_bits < 12) ++width_bits;
        }
        prev = code;
    }
    if (idx.size() < npx) idx.resize(npx, 0);  // a short stream leaves the rest at index 0
    width = sw ? sw : fw;
    height = sh ? sh : fh;
    if (width == 0 || height == 0 || (uint64_t)width * height > kMaxTexels) return fail(err, RR_E_LIMIT, "GIF screen size");
    rgba.assign((size_t)width * height * 4, 0);
    // interlaced frames store rows in four passes: 0, 8, 16 ...; 4, 12 ...; 2, 6 ...; 1, 3 ...
    std::vector<uint32_t> order;
    if (iflags & 0x40u) {
        for (uint32_t start : {0u, 4u, 2u, 1u})
            for (uint32_t r = start; r < fh; r += (start == 0 ? 8u : start == 4 ? 8u : start == 2 ? 4u : 2u)) order.push_back(r);
    } else {
        for (uint32_t r = 0; r < fh; ++r) order.push_back(r);
    }
    for (uint32_t k = 0; k < fh; ++k) {
        const uint32_t y = fy + order[k];
        if (y >= height) continue;
        for (uint32_t x = 0; x < fw; ++x) {
            if (fx + x >= width) continue;
            const uint32_t v = idx[(size_t)k * fw + x];
            if ((int)v == transparent || 3 * (size_t)v + 2 >= ct.size()) continue;
            uint8_t* o = &rgba[4 * ((size_t)y * width + fx + x)];
            o[0] = ct[3 * v], o[1] = ct[3 * v + 1], o[2] = ct[3 * v + 2], o[3] = 255;
        }
    }
    return RR_OK;
}

}  // namespace rr
