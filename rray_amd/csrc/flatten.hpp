// flatten.hpp — rr_scene_desc (the reference's object registry) -> HBM layout (rr_device.hpp).
#pragma once
#include <string>
#include <vector>

#include "rr_device.hpp"
#include "rr_math.hpp"

namespace rr {

struct HostScene {
    std::vector<DevNode> nodes;
    std::vector<DevCull> culls;  // one per node
    std::vector<DevCull> inner;  // one per node: a ball inside the set the node's exact test reports (r 0: none)
    std::vector<DevChunk> chunks;
    std::vector<DevGroup> groups;
    std::vector<DevTri> tris;
    std::vector<DevShape> shapes;
    std::vector<DevMaterial> mats;
    std::vector<DevPattern> pats;
    std::vector<DevLight> lights;
    std::vector<DevTexture> textures;
    std::vector<uint32_t> texels;
    std::vector<int32_t> node_of_object;  // object id -> node index (-1 if not in the scene tree)
    std::vector<char> chunk_break;        // node starts a spatial bucket (reorder_spatial -> build_chunks)
    int32_t has_transparent = 0;
    int32_t has_secondary = 0;            // some material reflective != 0 or transparency != 0
    int32_t max_children = 0;             // max secondary rays one shading event queues (0, 1 or 2)
    int32_t tri_inline = 0;               // every triangle node carries p1/e1/e2 inline (NF_TRI_INLINE)
    int32_t has_csg = 0;
    int32_t has_quad = 0;
    int32_t complex_patterns = 0;         // tree-evaluated patterns (pattern_tree)
    int64_t n_top_leaves = 0;             // leaves tested by every ray (reference full scan)
};

// Returns RR_OK or an error code (message in `err`).
int flatten_scene(const rr_scene_desc& d, HostScene& out, std::string& err);

// Inverse + affinity check: row 3 of the inverse must be (+-0,+-0,+-0,1) so that a point's w stays
// exactly 1 and a vector's w stays +-0 (proved for affine inputs in DESIGN.md).
bool inverse_3x4(const M4& transform, const double* given_inverse, double out12[12], M4* full, std::string& err);

}  // namespace rr
