// Host diagnostic: chunk statistics of a YAML scene's flattening (count, bounding-sphere radii).
// Build: g++ -O2 -std=c++17 -D__host__= -D__device__= -Iinclude -Irray_amd/csrc tools/diag/chunk_stats.cpp \
//        -Lrray_amd/_lib -lrray_amd -Wl,-rpath,$PWD/rray_amd/_lib -o /tmp/chunk_stats
#include <cmath>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <algorithm>
#include <vector>

#include "rray/rray.h"
#include "flatten.hpp"

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: chunk_stats scene.yaml obj_root\n");
        return 2;
    }
    std::ifstream f(argv[1]);
    std::stringstream ss;
    ss << f.rdbuf();
    rr_scene* sc = nullptr;
    rr_camera cam;
    if (rr_scene_from_yaml(ss.str().c_str(), argv[2], 64, 64, 1, &sc, &cam) != 0) {
        std::fprintf(stderr, "yaml: %s\n", rr_last_error());
        return 1;
    }
    rr::HostScene hs;
    std::string err;
    if (rr::flatten_scene(*rr_scene_desc_of(sc), hs, err) != 0) {
        std::fprintf(stderr, "flatten: %s\n", err.c_str());
        return 1;
    }
    std::vector<double> rs;
    double node_r = 0.0;
    int bounded_nodes = 0;
    for (const auto& c : hs.culls)
        if (std::isfinite(c.r)) {
            node_r += c.r;
            ++bounded_nodes;
        }
    for (const auto& ch : hs.chunks)
        if (std::isfinite(ch.cull.r)) rs.push_back(ch.cull.r);
    std::sort(rs.begin(), rs.end());
    double sum = 0.0, sum2 = 0.0;
    for (double r : rs) {
        sum += r;
        sum2 += r * r;
    }
    std::printf("nodes %zu (bounded %d, mean node radius %.4f), chunks %zu (bounded %zu): radius mean %.4f rms %.4f "
                "median %.4f p90 %.4f max %.4f\n",
                hs.nodes.size(), bounded_nodes, node_r / std::max(1, bounded_nodes), hs.chunks.size(), rs.size(),
                sum / rs.size(), std::sqrt(sum2 / rs.size()), rs[rs.size() / 2], rs[rs.size() * 9 / 10], rs.back());
    rr_scene_free(sc);
    return 0;
}
