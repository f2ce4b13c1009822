// rr_device.hpp — the flattened scene as it sits in HBM (shared by host flattener and kernels).
//
// The reference keeps Arc<dyn Object> in a mutex-guarded registry (object/db.rs:11-13) and
// walks it per ray.  Here the registry is flattened once per scene, in Scene.ids order with each
// group's children inlined (depth-first), which is exactly the tie-break order of the
// reference's stable sorts (scene.rs:104, group.rs:88).  Every record is read wave-uniformly
// (all 64 lanes test the same node), so the loads become scalar (SMEM) broadcasts.
#pragma once
#include <stdint.h>

#include "../../include/rray/rray.h"

namespace rr {

enum NodeFlags : int32_t {
    NF_IDENT = 1,       // inverse transform is exactly the identity (skip the ray transform)
    NF_IN_CSG = 2,      // inside a CSG subtree: intersected only through the CSG's evaluation
    NF_DIAG = 4,        // inverse is diagonal + translation (scale / translate objects): 3 products per
                        // transform instead of 9 (device_core.inc xf_ray_node)
    NF_TRI_INLINE = 8,  // triangle with an identity inverse (every OBJ face): inv[0..8] hold its p1, e1, e2
                        // (DevTri order), so the walk's exact test needs no dependent DevTri load; the
                        // identity itself is implied by NF_IDENT (also set)
    NF_OWN_SAFE = 16,   // sphere / plane outside any CSG whose world-to-object transform is conditioned well enough
                        // that a shadow ray leaving its own surface point outward cannot hit it (flatten.cpp
                        // mark_own_safe; the walks skip that exact test, device_core.inc walk_nodes `own`)
    NF_CSG_LHIT0 = 256, // bit (8 + d): for the CSG at position d of this leaf's ancestor chain,
                        // left.includes(this leaf) (csg.rs:86-88 with Object::includes semantics)
};
__host__ __device__ inline bool is_container(int kind) { return kind == RR_GROUP || kind == RR_CSG; }

// One flattened object.  128 B, 16-B aligned.
struct alignas(16) DevNode {
    double inv[12];   // rows 0..2 of the inverse transform (row 3 verified == 0,0,0,1)
    int32_t kind;     // RR_SPHERE ..
    int32_t flags;    // NodeFlags
    int32_t material; // DevMaterial index (leaves)
    int32_t skip;     // first node index after this node's subtree
    int32_t parent;   // parent node index (-1 = scene top level)
    int32_t aux;      // group index (groups) / triangle index (triangles)
    int32_t depth;    // number of group ancestors
    int32_t rank;     // position in the reference's DFS order (tie-break key; nodes are stored
                      // with siblings in spatial order, see flatten.cpp)
};
static_assert(sizeof(DevNode) == 128, "DevNode layout");

// Per group / CSG: bounding box in its own space (group.rs:128-149, csg.rs get_aabb) and its
// ancestor chain (groups and CSGs).
struct alignas(16) DevGroup {
    double aabb[6];                      // min xyz, max xyz
    int32_t anc[RR_MAX_GROUP_DEPTH];     // node indices root-first; anc[depth-1] == this node
    int32_t depth;                       // number of containers from the root down to and incl. this one
    int32_t csg_op;                      // RR_CSG_* (CSG nodes)
};

// Cylinder / cone parameters (cylinder.rs:29-37, cone.rs:30-38).
struct alignas(16) DevShape {
    double minimum, maximum;
    int32_t closed;
    int32_t pad;
};

// Per triangle: Möller-Trumbore data (triangle.rs:52-68) + normals.
struct alignas(16) DevTri {
    double p1[3], e1[3], e2[3];
    double normal[3];          // normalize(e2 x e1)
    double n1[3], n2[3], n3[3];  // smooth-triangle vertex normals
    int32_t smooth;
    int32_t pad;
};

struct alignas(16) DevMaterial {  // material.rs:35-44
    double ambient, diffuse, specular, shininess, reflective, transparency, refractive_index;
    int32_t pattern;
    // root: 1 = Solid (or the default white), colour in `color` (a Solid's colour does not depend
    // on the point, pattern.rs:151-153); 0 = evaluate pattern_at.  (Inlining a Stripe / Ring /
    // Checker root as well made the record 224 B and cost the fused kernel 34 more spilled VGPRs.)
    int32_t root;
    double color[3];
};

// DevPattern.flags: NF_IDENT (identity transform) plus, for Stripe / Ring / Checker, whether child
// a / b is a Solid whose colour is stored inline (ca / cb), saving the dependent child load.
enum PatternFlags : int32_t { PF_A_SOLID = 2, PF_B_SOLID = 4 };
struct alignas(16) DevPattern {  // pattern.rs:23-27
    double inv[12];
    double color[3];
    double scale;
    double ca[3], cb[3];  // inline Solid children (PF_A_SOLID / PF_B_SOLID)
    int32_t kind, a, b, flags;
    double persistence;  // Perturbed / Noise (pattern.rs:16-19)
    int32_t octaves, pad;
};

struct alignas(16) DevLight {  // light.rs:17-21
    double position[3];   // area: corner + u*0.5 + v*0.5 (light.rs:41-45)
    double intensity[3];
    double corner[3], u[3], v[3];
    int32_t kind, level;
};

// Image texture (texture.rs:6-11): RGBA8 texels packed one u32 each (byte 0 = red), rows top to
// bottom, at texels[offset ..].
struct alignas(16) DevTexture {
    uint64_t offset;
    uint32_t width, height;
};

struct DevCamera {
    int64_t hsize, vsize;
    double half_width, half_height, pixel_size;
    double inv[16];  // full 4x4 inverse of the camera transform (camera.rs:85)
    double origin[4];  // inverse * point(0, 0, 0), the same for every pixel (computed on the host)
};

// Conservative bounding sphere of a node's content in WORLD space (so any run of consecutive nodes,
// at any group depth, can be tested against one world-space ray bundle): f32 centre + radius,
// inflated so that every ray the exact f64 test can report as intersecting passes the f32 cull
// (DESIGN.md §3.5).  radius = +inf: never culled (planes, unbounded groups).
struct alignas(16) DevCull {
    float c[3];
    float r;
};

// A run of consecutive nodes (<= 64) with the world-space bounding sphere of their culls.
// Runs of one kind, which the walks test without per-node kind / flag / transform dispatch (walk_nodes):
// run >= 0: every node is a triangle with its data inline (NF_TRI_INLINE), outside any CSG, and a child of node
// `run` (a mesh); CR_SPHERE_DIAG: every node is a top-level sphere with a diagonal inverse (NF_DIAG).  One field,
// so the walks read one value per chunk.
enum ChunkRun : int32_t { CR_NONE = -1, CR_SPHERE_DIAG = -2 };
struct alignas(16) DevChunk {
    DevCull cull;
    int32_t start, count;
    int32_t run, pad;
};

struct DevScene {
    const DevCull* culls;
    const DevCull* inner;     // per node: a ball inside what its exact test reports (spheres; r == 0: none)
    const DevChunk* chunks;
    const DevNode* nodes;
    const DevGroup* groups;
    const DevTri* tris;
    const DevMaterial* mats;
    const DevPattern* pats;
    const DevLight* lights;
    const DevShape* shapes;
    const DevTexture* textures;
    const uint32_t* texels;
    int32_t n_nodes, n_lights;
    int32_t n_chunks;
    int32_t has_area;         // some light is an area light (the shade kernels stage its samples in LDS)
    int32_t has_transparent;  // any material with transparency != 0 (enables the n1/n2 walk)
    int32_t has_groups;
    int32_t general;          // CSGs or cylinders / cones present: the kernels' G = 2 variant
    int32_t lds_culls;        // culls + chunks staged in LDS per workgroup (fits in RR_LDS_CULL_BYTES)
    int32_t complex_patterns; // some pattern is Gradient / Blend / Perturbed / Noise / Texture
    int32_t tri_inline;       // every triangle node is NF_TRI_INLINE (the walks read p1/e1/e2 from the node)
    int32_t n_free;           // trailing chunks holding one unbounded top-level leaf each (planes): the
                              // last n_free nodes, tested without culling before the chunk passes
    int32_t free_planes;      // every one of them is a plane with an identity inverse (no dispatch in the walks)
    float bs_c[3], bs_r;      // sphere around every bounded node's cull (bs_r < 0: none); rays whose origin
                              // lies far outside it are culled from a point nearer to it (make_bundle)
};
// Node culls (16 B each) and chunk records (32 B each) are copied into LDS by every walking
// workgroup when together they fit in this many bytes.  Small scenes gain from it (C5 2.5 %, C1
// 1 %); at C2's 17 KB the per-workgroup staging costs more than the walks' L1/L2 reads of the few
// candidate chunks save (global culls 0.173 vs LDS 0.175 ms per frame; C3 equal).
constexpr int RR_LDS_CULL_BYTES = 8 * 1024;
constexpr int RR_BUNDLE_MIN_NODES = 8;  // walks of scenes with at most this many nodes build no ray bundle

// Per-launch counters (u64, zeroed by the host before each launch).
enum Counter {
    C_RAYS = 0,
    C_SHADOW,
    C_SHADE,
    C_N1N2,
    C_GROUP_TESTS,
    C_GROUP_HITS,
    C_SAMPLES,
    C_PRIM_TESTS,
    C_WORK,  // work-queue head
    C_FLOPS_TRACE,   // f64 flops of the exact tests executed (SURVEY §8d model), per walk kind
    C_FLOPS_SHADOW,
    C_FLOPS_N1N2,
    C_VISITS_TRACE,  // node visits x 64 (one per lane of a wave that ran a candidate's exact test)
    C_VISITS_SHADOW,
    C_VISITS_N1N2,
    C_NAN,  // rays whose intersection list holds a NaN t among >= 2 entries (the reference's sort panics)
    C_COUNT
};
// Counters live in RR_CNT_SLOTS copies (slot = blockIdx % RR_CNT_SLOTS, RR_CNT_STRIDE u64 each) so
// that concurrent workgroups' device-scope atomics hit different addresses; the host sums them.
constexpr int RR_CNT_SLOTS = 256;
constexpr int RR_CNT_STRIDE = 16;
static_assert(C_COUNT <= RR_CNT_STRIDE, "counter slot layout");

}  // namespace rr
