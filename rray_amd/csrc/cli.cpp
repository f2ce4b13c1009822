// cli.cpp — `rray` drop-in CLI (src/main.rs:49-77): same flags and defaults.
//   rray -W <width=800> -H <height=600> -s <scene.yaml> -o <output.png> -a <aa=1, max 5>
// Renders on GPU 0 (RRAY_DEVICE=<id> picks another one); RRAY_DEVICES=<id,id,...> or RRAY_DEVICES=all
// splits the frame over several GPUs of this host (rr_create_multi: row tiles + one RCCL transfer per part).
// No CPU fallback.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rray/rray.h"

static int usage(const char* msg) {
    if (msg) std::fprintf(stderr, "error: %s\n", msg);
    std::fprintf(stderr,
                 "A simple raytracer\n\nUsage: rray [OPTIONS] --scene <SCENE>\n\nOptions:\n"
                 "  -W, --width <WIDTH>    Width of the generated image, default is 800 [default: 800]\n"
                 "  -H, --height <HEIGHT>  Height of the generated image, default is 600 [default: 600]\n"
                 "  -s, --scene <SCENE>    Scene file in YAML format\n"
                 "  -o, --output <OUTPUT>  Name of the output file, default is output.png [default: output.png]\n"
                 "  -a, --aa <AA>          Anti-aliasing level (default 1) (max 5) [default: 1]\n"
                 "  -h, --help             Print help\n  -V, --version          Print version\n");
    return 2;
}

static bool parse_usize(const char* s, long long& out) {
    if (!s || !*s) return false;
    for (const char* p = s; *p; ++p)
        if (*p < '0' || *p > '9') return false;
    out = std::atoll(s);
    return true;
}

int main(int argc, char** argv) {
    long long width = 800, height = 600, aa = 1;
    std::string scene, output = "output.png";
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto val = [&](const char* name) -> const char* {
            if (i + 1 >= argc) {
                usage((std::string("missing value for ") + name).c_str());
                std::exit(2);
            }
            return argv[++i];
        };
        if (a == "-h" || a == "--help") return usage(nullptr), 0;
        if (a == "-V" || a == "--version") return std::printf("rray 1.0\n"), 0;
        if (a == "-W" || a == "--width") {
            if (!parse_usize(val("--width"), width)) return usage("width must be a positive number");
        } else if (a == "-H" || a == "--height") {
            if (!parse_usize(val("--height"), height)) return usage("height must be a positive number");
        } else if (a == "-s" || a == "--scene") {
            scene = val("--scene");
        } else if (a == "-o" || a == "--output") {
            output = val("--output");
        } else if (a == "-a" || a == "--aa") {
            if (!parse_usize(val("--aa"), aa)) return usage("must be a positive number");  // main.rs:21-27
            if (aa > 5) return usage("value must be less than or equal to 5");
        } else {
            return usage(("unexpected argument '" + a + "'").c_str());
        }
    }
    if (scene.empty()) return usage("the following required arguments were not provided: --scene <SCENE>");
    if (width <= 0 || height <= 0 || aa <= 0) return usage("width, height and aa must be >= 1");
    std::vector<int> devices;
    if (const char* ds = std::getenv("RRAY_DEVICES")) {
        if (std::strcmp(ds, "all") == 0) {
            int n = 0;
            rr_device_count(&n);
            for (int i = 0; i < n; ++i) devices.push_back(i);
        } else {
            for (const char* p = ds; *p;) {
                char* end = nullptr;
                long v = std::strtol(p, &end, 10);
                if (end == p || v < 0) return usage("RRAY_DEVICES must be `all` or a comma-separated list of ids");
                devices.push_back((int)v);
                p = *end == ',' ? end + 1 : end;
                if (*end && *end != ',') return usage("RRAY_DEVICES must be `all` or a comma-separated list of ids");
            }
        }
        if (devices.empty()) {
            std::fprintf(stderr, "rray: no GPU device available\n");
            return 1;
        }
    } else {
        devices.push_back(std::getenv("RRAY_DEVICE") ? std::atoi(std::getenv("RRAY_DEVICE")) : 0);
    }
    int rc = rr_render_scene_from_file_devices(scene.c_str(), width, height, output.c_str(), (int)aa,
                                               (int)devices.size(), devices.data());
    if (rc != RR_OK) {
        std::fprintf(stderr, "rray: %s (code %d)\n", rr_last_error(), rc);
        return 1;
    }
    return 0;
}
