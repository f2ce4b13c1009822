// Host-only AddressSanitizer harness for the JPEG front-end (rray_amd/csrc/jpeg.cpp): decodes every file
// named on the command line and prints "<rc> <width> <height>" per file.  Built and run by
// tests/test_jpeg.py::test_corrupt_jpegs_under_asan with g++ -fsanitize=address (no GPU code involved).
#include <cstdio>
#include <string>
#include <vector>

#include "../rray_amd/csrc/png.hpp"

int main(int argc, char** argv) {
    for (int i = 1; i < argc; ++i) {
        FILE* f = std::fopen(argv[i], "rb");
        if (!f) return 2;
        std::vector<uint8_t> data;
        unsigned char buf[65536];
        size_t n;
        while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) data.insert(data.end(), buf, buf + n);
        std::fclose(f);
        std::vector<uint8_t> rgba;
        uint32_t w = 0, h = 0;
        std::string err;
        const int rc = rr::decode_jpeg_rgba(data.data(), data.size(), rgba, w, h, err);
        std::printf("%d %u %u\n", rc, w, h);
    }
    return 0;
}
