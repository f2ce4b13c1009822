// Host-only AddressSanitizer harness for the texture reader (rray_amd/csrc/png.cpp read_image_rgba: PNG, JPEG and
// imgfmt.cpp's BMP / TGA / PNM / GIF): reads every file named on the command line and prints
// "<rc> <width> <height>" per file.  Built and run by tests/test_abi_host.py::test_corrupt_textures_under_asan with
// g++ -fsanitize=address (no GPU code involved).
#include <cstdio>
#include <string>
#include <vector>

#include "../rray_amd/csrc/png.hpp"

int main(int argc, char** argv) {
    for (int i = 1; i < argc; ++i) {
        std::vector<uint8_t> rgba;
        uint32_t w = 0, h = 0;
        std::string err;
        const int rc = rr::read_image_rgba(argv[i], rgba, w, h, err);
        if (rc == 0 && rgba.size() != (size_t)w * h * 4) return 3;
        std::printf("%d %u %u\n", rc, w, h);
    }
    return 0;
}
