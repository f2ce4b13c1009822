// png.cpp — RGBA8 PNG encoder over zlib (filter 0 per row; lossless, so decoded pixels
// equal the reference's image-crate output), and the texture reader (texture.rs:15-19: image::open + to_rgba8):
// PNG of every colour type, bit depth and interlace method; JPEG through jpeg.cpp; BMP / TGA / PNM / GIF through
// imgfmt.cpp.
#include "png.hpp"

#include <zlib.h>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/rray/rray.h"

namespace rr {
namespace {
void put32(std::vector<uint8_t>& v, uint32_t x) {
    v.push_back((uint8_t)(x >> 24));
    v.push_back((uint8_t)(x >> 16));
    v.push_back((uint8_t)(x >> 8));
    v.push_back((uint8_t)x);
}
void chunk(std::vector<uint8_t>& out, const char* type, const std::vector<uint8_t>& data) {
    put32(out, (uint32_t)data.size());
    size_t start = out.size();
    out.insert(out.end(), type, type + 4);
    out.insert(out.end(), data.begin(), data.end());
    uLong crc = crc32(0L, out.data() + start, (uInt)(out.size() - start));
    put32(out, (uint32_t)crc);
}
uint32_t get32(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }
int paeth(int a, int b, int c) {
    int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc) return a;
    return pb <= pc ? b : c;
}
}  // namespace

int read_image_rgba(const std::string& path, std::vector<uint8_t>& rgba, uint32_t& width, uint32_t& height,
                  std::string& err) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) {
        err = "cannot open texture " + path;
        return RR_E_IO;
    }
    std::vector<uint8_t> file;
    uint8_t buf[65536];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) file.insert(file.end(), buf, buf + n);
    std::fclose(f);
    if (file.size() >= 3 && file[0] == 0xFF && file[1] == 0xD8 && file[2] == 0xFF) {
        int rc = decode_jpeg_rgba(file.data(), file.size(), rgba, width, height, err);
        if (rc != RR_OK) err = path + ": " + err;
        return rc;
    }
    // the other formats by signature (TGA has none: by extension, as image::open chooses every format)
    int (*other)(const uint8_t*, size_t, std::vector<uint8_t>&, uint32_t&, uint32_t&, std::string&) = nullptr;
    const auto ext_is = [&](const char* e) {
        const size_t k = std::strlen(e);
        if (path.size() < k) return false;
        for (size_t i = 0; i < k; ++i)
            if (std::tolower((unsigned char)path[path.size() - k + i]) != e[i]) return false;
        return true;
    };
    if (file.size() >= 2 && file[0] == 'B' && file[1] == 'M')
        other = decode_bmp_rgba;
    else if (file.size() >= 4 && std::memcmp(file.data(), "GIF8", 4) == 0)
        other = decode_gif_rgba;
    else if (file.size() >= 2 && file[0] == 'P' && file[1] >= '1' && file[1] <= '6')
        other = decode_pnm_rgba;
    else if (ext_is(".tga"))
        other = decode_tga_rgba;
    if (other) {
        int rc = other(file.data(), file.size(), rgba, width, height, err);
        if (rc != RR_OK) err = path + ": " + err;
        return rc;
    }
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    if (file.size() < 8 || std::memcmp(file.data(), sig, 8) != 0) {
        err = path + ": not PNG, JPEG, BMP, GIF, PNM or TGA (other image formats need a host-side decoder: pass texels in "
                     "rr_scene_desc)";
        return RR_E_LIMIT;
    }
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> idat, plte;
    size_t pos = 8;
    bool end = false;
    while (!end && pos + 12 <= file.size()) {
        uint32_t len = get32(&file[pos]);
        if (pos + 12 + (size_t)len > file.size()) break;
        const uint8_t* type = &file[pos + 4];
        const uint8_t* data = &file[pos + 8];
        if (!std::memcmp(type, "IHDR", 4) && len >= 13) {
            w = get32(data);
            h = get32(data + 4);
            depth = data[8];
            ctype = data[9];
            interlace = data[12];
        } else if (!std::memcmp(type, "PLTE", 4)) {
            plte.assign(data, data + len);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), data, data + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            end = true;
        }
        pos += 12 + (size_t)len;
    }
    if (w == 0 || h == 0 || ctype < 0 || idat.empty()) {
        err = path + ": corrupt PNG";
        return RR_E_IO;
    }
    const int channels = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 3 ? 1 : ctype == 4 ? 2 : ctype == 6 ? 4 : 0;
    const bool depth_ok = ctype == 0   ? (depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16)
                          : ctype == 3 ? (depth == 1 || depth == 2 || depth == 4 || depth == 8)
                                       : (depth == 8 || depth == 16);
    if (channels == 0 || !depth_ok || interlace > 1) {
        err = path + ": PNG layout outside the PNG specification (color type / bit depth / interlace method)";
        return RR_E_IO;
    }
    if (ctype == 3 && plte.size() < 3) {
        err = path + ": palette PNG without PLTE";
        return RR_E_IO;
    }
    if ((uint64_t)w * h > (1ull << 28)) {
        err = path + ": texture larger than 2^28 texels";
        return RR_E_LIMIT;
    }
    // the sub-images: the whole image, or Adam7's seven passes (x0, y0, dx, dy), each filtered separately
    struct Pass {
        uint32_t x0, y0, dx, dy, pw, ph;
    };
    static const uint32_t adam7[7][4] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4},
                                         {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
    std::vector<Pass> passes;
    if (interlace == 0) {
        passes.push_back({0, 0, 1, 1, w, h});
    } else {
        for (const auto& q : adam7) {
            const uint32_t pw = w > q[0] ? (w - q[0] + q[2] - 1) / q[2] : 0, ph = h > q[1] ? (h - q[1] + q[3] - 1) / q[3] : 0;
            if (pw && ph) passes.push_back({q[0], q[1], q[2], q[3], pw, ph});
        }
    }
    const auto stride_of = [&](uint32_t pw) { return ((size_t)pw * channels * depth + 7) / 8; };
    size_t total = 0;
    for (const Pass& ps : passes) total += (stride_of(ps.pw) + 1) * ps.ph;
    const size_t bpp = std::max<size_t>(1, (size_t)channels * depth / 8);
    std::vector<uint8_t> raw(total);
    z_stream zs{};
    if (inflateInit(&zs) != Z_OK) {
        err = "zlib init failed";
        return RR_E_IO;
    }
    zs.next_in = idat.data();
    zs.avail_in = (uInt)idat.size();
    zs.next_out = raw.data();
    zs.avail_out = (uInt)raw.size();
    int zr = inflate(&zs, Z_FINISH);
    inflateEnd(&zs);
    if ((zr != Z_STREAM_END && zr != Z_BUF_ERROR) || zs.avail_out != 0) {
        err = path + ": corrupt PNG image data";
        return RR_E_IO;
    }
    // a sample of `depth` bits at sample index k of an unfiltered row -> 8 bits, as the image crate's to_rgba8 gives it:
    // sub-byte grey scaled by 255 / (2^depth - 1); 16-bit by FromPrimitive<u16> for u8, round(c * 255 / 65535) =
    // (c + 128) / 257 (image 0.25 color.rs; not vendored: no reference-held 16-bit PNG pins it)
    const auto sample8 = [&](const uint8_t* row, size_t k) -> uint8_t {
        if (depth == 8) return row[k];
        if (depth == 16) return (uint8_t)((((uint32_t)row[2 * k] << 8 | row[2 * k + 1]) + 128u) / 257u);
        const size_t bit = k * (size_t)depth;
        const int v = (row[bit / 8] >> (8 - depth - (int)(bit % 8))) & ((1 << depth) - 1);
        return ctype == 3 ? (uint8_t)v : (uint8_t)(v * 255 / ((1 << depth) - 1));
    };
    rgba.assign((size_t)w * h * 4, 255);
    size_t off = 0;
    for (const Pass& ps : passes) {
        const size_t stride = stride_of(ps.pw);
        std::vector<uint8_t> prev(stride, 0);
        for (uint32_t y = 0; y < ps.ph; ++y) {  // unfilter in place (filter types 0-4; the previous row of this pass)
            uint8_t* row = &raw[off + (size_t)y * (stride + 1)];
            const uint8_t ft = row[0];
            uint8_t* cur = row + 1;
            for (size_t i = 0; i < stride; ++i) {
                int a = i >= bpp ? cur[i - bpp] : 0, b = prev[i], c = i >= bpp ? prev[i - bpp] : 0;
                int pred = ft == 0 ? 0 : ft == 1 ? a : ft == 2 ? b : ft == 3 ? (a + b) / 2 : ft == 4 ? paeth(a, b, c) : -1;
                if (pred < 0) {
                    err = path + ": bad PNG filter type";
                    return RR_E_IO;
                }
                cur[i] = (uint8_t)(cur[i] + pred);
            }
            std::memcpy(prev.data(), cur, stride);
            for (uint32_t x = 0; x < ps.pw; ++x) {
                uint8_t* o = &rgba[4 * ((size_t)(ps.y0 + y * ps.dy) * w + ps.x0 + (size_t)x * ps.dx)];
                const size_t k = (size_t)x * channels;
                if (ctype == 3) {
                    const int v = sample8(cur, k);
                    if (3 * (size_t)v + 2 >= plte.size()) {
                        err = path + ": palette index out of range";
                        return RR_E_IO;
                    }
                    o[0] = plte[3 * v];
                    o[1] = plte[3 * v + 1];
                    o[2] = plte[3 * v + 2];
                    continue;
                }
                switch (ctype) {
                    case 0: o[0] = o[1] = o[2] = sample8(cur, k); break;
                    case 4: o[0] = o[1] = o[2] = sample8(cur, k); o[3] = sample8(cur, k + 1); break;
                    case 2: o[0] = sample8(cur, k); o[1] = sample8(cur, k + 1); o[2] = sample8(cur, k + 2); break;
                    default:
                        o[0] = sample8(cur, k);
                        o[1] = sample8(cur, k + 1);
                        o[2] = sample8(cur, k + 2);
                        o[3] = sample8(cur, k + 3);
                        break;
                }
            }
        }
        off += (stride + 1) * ps.ph;
    }
    width = w;
    height = h;
    return RR_OK;
}

bool write_png_rgba(const char* path, const uint8_t* rgba, uint32_t w, uint32_t h) {
    std::vector<uint8_t> raw;
    raw.reserve((size_t)h * (1 + 4 * (size_t)w));
    for (uint32_t y = 0; y < h; ++y) {
        raw.push_back(0);
        raw.insert(raw.end(), rgba + (size_t)y * w * 4, rgba + (size_t)(y + 1) * w * 4);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) return false;
    z.resize(zlen);
    std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::vector<uint8_t> ihdr;
    put32(ihdr, w);
    put32(ihdr, h);
    ihdr.insert(ihdr.end(), {8, 6, 0, 0, 0});  // 8-bit RGBA, deflate, adaptive filtering, no interlace
    chunk(out, "IHDR", ihdr);
    chunk(out, "IDAT", z);
    chunk(out, "IEND", {});
    FILE* f = std::fopen(path, "wb");
    if (!f) return false;
    bool ok = std::fwrite(out.data(), 1, out.size(), f) == out.size();
    ok = (std::fclose(f) == 0) && ok;
    return ok;
}
}  // namespace rr
