// png.hpp — RGBA8 PNG writer (canvas.rs:124-131 writes RGBA8 through the image crate) and the
// texture reader (texture.rs:15-19: decode, to_rgba8).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace rr {
bool write_png_rgba(const char* path, const uint8_t* rgba, uint32_t width, uint32_t height);
// Texture file -> RGBA8 rows top to bottom.  PNG: every colour type, bit depth and interlace method; JPEG: baseline /
// extended sequential / progressive (jpeg.cpp); BMP, TGA, PNM and GIF (imgfmt.cpp).  Returns RR_OK, RR_E_IO
// (unreadable / corrupt) or RR_E_LIMIT (a layout outside these decoders).
int read_image_rgba(const std::string& path, std::vector<uint8_t>& rgba, uint32_t& width, uint32_t& height,
                  std::string& err);
// jpeg.cpp: the JPEG decoder on a file's bytes
int decode_jpeg_rgba(const uint8_t* data, size_t len, std::vector<uint8_t>& rgba, uint32_t& width,
                     uint32_t& height, std::string& err);
// imgfmt.cpp: the other formats image::open decodes with its default features, on a file's bytes
int decode_bmp_rgba(const uint8_t* data, size_t len, std::vector<uint8_t>& rgba, uint32_t& width, uint32_t& height,
                    std::string& err);
int decode_tga_rgba(const uint8_t* data, size_t len, std::vector<uint8_t>& rgba, uint32_t& width, uint32_t& height,
                    std::string& err);
int decode_pnm_rgba(const uint8_t* data, size_t len, std::vector<uint8_t>& rgba, uint32_t& width, uint32_t& height,
                    std::string& err);
int decode_gif_rgba(const uint8_t* data, size_t len, std::vector<uint8_t>& rgba, uint32_t& width, uint32_t& height,
                    std::string& err);
}
