// png.hpp — RGBA8 PNG writer (canvas.rs:124-131 writes RGBA8 through the image crate).
#pragma once
#include <cstdint>

namespace rr {
bool write_png_rgba(const char* path, const uint8_t* rgba, uint32_t width, uint32_t height);
}
