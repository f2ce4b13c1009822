// kernels.hpp — host-visible launch interface of render.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <utility>
#include <vector>

#include "rr_device.hpp"
#include "wavefront.hpp"

namespace rr {

// Arguments of one wavefront level (see wavefront.hpp).
struct LevelArgs {
    DevCamera cam;           // level-0 ray source (when rays0 == nullptr)
    int64_t hs;              // supersampled width
    int64_t lrows;           // part-local supersampled rows (level-0 camera rays run in 8x8 tiles)
    int32_t aa, part, nparts, block_rows;
    uint32_t aa_magic, br_magic;  // floor(2^32 / d) for d = aa, block_rows (>= 2; 0 when d == 1)
    int32_t tile_fast;       // level-0 tiles all full 8x8 and the batch tile-aligned: wave = one tile
    uint32_t tiles_per_row;  // hs / 8 (tile_fast)
    int32_t cam_affine;      // camera inverse row 3 == (0, 0, 0, 1)
    int64_t base;            // first local sample of this batch
    const double* rays0;     // level-0 explicit rays (o xyz, d xyz); nullptr: camera rays
    int32_t level, rem;      // level d and `remaining` = max_depth - d
    int64_t n;               // events at this level (n_dev == null) or this level's capacity (the grid)
    const unsigned int* n_dev;  // level >= 1: the live event count, written by the previous level's appends
    // segmented queues (fused levels, wavefront.hpp): this level's events are seg_count[s] events at
    // s * seg_cap (nseg > 1; level 0 has one segment), its children go to segment blockIdx % nseg_out of
    // the next level at s * seg_cap_out, counted in seg_out_count[s]
    int32_t nseg, nseg_out;
    int64_t seg_cap, seg_cap_out;
    const unsigned int* seg_count;
    unsigned int* seg_out_count;
    const Event* ev;         // level >= 1 input queue
    HitRec* hit;
    double* n12;
    CombRec* comb;           // this level's pending sums (indexed by event)
    CombRec* parent_comb;    // level - 1 (children deliver into their parent's slot)
    CombExt* comb_ext;       // refraction halves (null when no material is transparent)
    CombExt* parent_ext;
    ChainRec* chain[RR_MAX_DEPTH + 1];  // FUSED levels: each level's pending surface sums (in the comb buffers)
    double* out;             // level 0: canvas / color_at results (3 doubles per local sample), or null
    void* avg;               // aa == 1: the averaged image written directly (canvas.rs:85-96 with aa = 1)
    const float* tile_bundles;  // level 0, tile_fast, affine camera: per-tile camera-ray bundles (tile_bundle_kernel,
                                // RR_TILE_BUNDLE_FLOATS each, indexed by tile), or null: built in the walk
    // fused level 0 of a one-batch tile_fast frame (group scenes' kernels): the tile each wave renders (launch slot -> tile, the costliest
    // first: tile_order_kernel), or null (launch order); and where each wave stores its tile's cost in clock
    // cycles (or null).  The order changes only which wave renders which tile, never a result.
    const uint32_t* tile_perm;
    uint32_t* tile_cost;
    int32_t order_group;     // tile_perm's units: 1 (one wave's tile each) or 4 (a block's four tiles)
    int32_t pad_children;    // fused levels: children in per-wave 64-slot blocks (holes: Event.parent == -2)
    // chain kernels (chain_kernel): the deep queue (segmented like the fused levels' queues: the camera launch
    // appends to seg_out_count / seg_cap_out, the deep launch reads seg_count / seg_cap) and the depth at which
    // chains leave their camera wave for it (0: they never do)
    DeepRec* deep;
    int32_t deep_from;
    // pixel waves (aa == 3, chain kernels, render_common.inc pixel_wave): level-0 waves of 7 whole pixels, averaged in
    // the wave; pw_wpb waves per band of two output rows, pw_rows the part's output rows
    int32_t pw;
    uint32_t pw_wpb;
    int32_t pw_rows;
    int32_t aa_wave;         // 2 / 4 / 8: every pixel's aa x aa samples lie in one wave's 8x8 tile and no
                             // sample has a secondary ray: the wave box-averages and writes avg (0: off)
    int32_t avg_f32;         // avg holds floats (RR_OUT_AVG_F32)
    Event* next;
    int32_t* pending;        // this level's events with children
    int32_t* n1n2_list;
    unsigned int* lcount;    // LC_* (zeroed per level)
    uint64_t seed;
    int32_t jitter_mode;
    unsigned long long* counters;  // C_* totals
    unsigned long long* counters_zero;  // the next frame's counter buffer, zeroed by this frame's kernels (or null)
};

struct CombArgs {
    int32_t level;
    int64_t n;                 // capacity of this level's pending list (sizes the grid)
    const unsigned int* n_dev; // the live pending count (LC_PENDING of the level)
    int64_t base;
    const int32_t* pending;
    const CombRec* comb;
    CombRec* parent_comb;
    const CombExt* comb_ext;  // as LevelArgs
    CombExt* parent_ext;
    double* out;  // level 0: canvas (3 doubles per local sample), or null
    void* avg;    // as LevelArgs
    int32_t avg_f32;
    int64_t hs, lrows;  // lrows > 0: level-0 events are in tile order (tile_to_local)
};

// The walking kernels' dynamic LDS (render_levels.inc): the scene's culls (when staged), then with <=
// RR_PRELIT_LIGHTS lights (PRE) every light's prelit terms ([light][6][256] doubles) and the area-light
// stage (scenes with an area light).
constexpr int RR_PRELIT_LIGHTS = 2;
constexpr size_t RR_AREA_STAGE_BYTES = 3 * 256 * 8 + 3 * 256 * 4;
constexpr size_t RR_CHAIN_STAGE_BYTES = 10 * 256 * 8 + 4 * 256 * 4;  // chain kernels: parked ray, level-0 record, Px0, own

// Level-0 camera events run in 8x8-sample tiles of the part-local supersampled canvas (8-row bands,
// 8-column tiles inside a band; the last band / column may be narrower) so that a wave's 64 rays
// form a tight bundle for the culling in walk_nodes.  Maps tile-order index t to the row-major
// local sample index (a bijection on [0, hs*lrows)).
__host__ __device__ inline int64_t tile_to_local(int64_t t, int64_t hs, int64_t lrows) {
    const int64_t band = t / (8 * hs);
    int64_t k = t - band * 8 * hs;
    const int64_t y0 = band * 8;
    const int64_t hb = lrows - y0 < 8 ? lrows - y0 : 8;
    const int64_t tc = k / (8 * hb);
    k -= tc * 8 * hb;
    const int64_t x0 = tc * 8;
    const int64_t wc = hs - x0 < 8 ? hs - x0 : 8;
    const int64_t dy = k / wc;
    return (y0 + dy) * hs + x0 + (k - dy * wc);
}
// the same in 32 bits (device: parts hold < 2^31 samples)
__host__ __device__ inline uint32_t tile_to_local_u32(uint32_t t, uint32_t hs, uint32_t lrows) {
    const uint32_t band = t / (8u * hs);
    uint32_t k = t - band * 8u * hs;
    const uint32_t y0 = band * 8u;
    const uint32_t hb = lrows - y0 < 8u ? lrows - y0 : 8u;
    const uint32_t tc = k / (8u * hb);
    k -= tc * 8u * hb;
    const uint32_t x0 = tc * 8u;
    const uint32_t wc = hs - x0 < 8u ? hs - x0 : 8u;
    const uint32_t dy = k / wc;
    return (y0 + dy) * hs + x0 + (k - dy * wc);
}

// Optional per-kernel timing: when `prof` is non-null every launch is bracketed by HIP events on
// the launch stream and appended to it (resolved on the host after a synchronise).
enum KernelId { K_TRACE = 0, K_N1N2, K_SHADE, K_SHADOW, K_FINISH, K_COMBINE, K_AA, K_TRACE_SHADE, K_CHAIN, K_DEEP, K_COUNT };
struct KernelProf {
    std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> marks;
    std::vector<hipEvent_t> pool;
    size_t used = 0;
    hipEvent_t get();
};

hipError_t launch_level(const DevScene& S, const LevelArgs& A, hipStream_t stream, KernelProf* prof = nullptr);
// One camera-ray bundle per full 8x8 tile of the part (A: level-0 tile_fast arguments of the whole part), into
// out (n_tiles x RR_TILE_BUNDLE_FLOATS floats): exactly the bundle make_bundle's cam_tile path builds in the walk.
constexpr int RR_TILE_BUNDLE_FLOATS = 12;
hipError_t launch_tile_bundles(const DevScene& S, const LevelArgs& A, float* out, int64_t n_tiles, hipStream_t stream);
// the same per pixel wave (A.pw): the bundle of the wave's 12 x 6-sample footprint from its corner rays
hipError_t launch_pixel_wave_bundles(const LevelArgs& A, float* out, int64_t n_waves, hipStream_t stream);
// cost = a guess of each tile's cost from its camera bundle (the nodes of the chunks it may reach), for a layout's
// first frame, before any tile has been timed
hipError_t launch_tile_guess(const DevScene& S, const float* bundles, uint32_t* cost, int64_t n_tiles, hipStream_t stream);
// perm = tiles by decreasing recorded cost (LevelArgs.tile_cost), for the next frames' level-0 launches;
// scratch = 256 u32 of device memory (bucket counters)
constexpr int RR_ORDER_GROUP = 4;
// group: the sort's unit, 1 tile or RR_ORDER_GROUP consecutive tiles (one launch block's waves; perm then maps a launch
// block to a tile group)
hipError_t launch_tile_order(const uint32_t* cost, uint32_t* perm, uint32_t* scratch, int64_t n_tiles, int group,
                             hipStream_t stream);
// trace + shade run as one kernel per level (no transparent material, so no n1/n2 walk between them);
// those levels finish their reflection chains themselves and need no combine pass
bool fused_levels(const DevScene& S);
// one (G, LC) variant of a level's kernels (render_levels.inc), instantiated in its own translation
// unit render_levels_g<G>_<lds|gl>.hip; G = 0 flat, 1 groups, 2 general; LC = culls staged in LDS
template <int G, bool LC>
void launch_level_t(const DevScene& S, const LevelArgs& A, hipStream_t stream, KernelProf* prof);
hipError_t launch_combine(const CombArgs& C, hipStream_t stream, KernelProf* prof = nullptr);
// Fused scenes whose materials reflect: the whole reflection chain of every level-0 event inside its wave
// (render_levels.inc chain_kernel), one launch per batch with no recursion queues
bool chain_levels(const DevScene& S, int max_children, int max_depth);
template <int G, bool LC>
void launch_chain_t(const DevScene& S, const LevelArgs& A, hipStream_t stream, KernelProf* prof, bool deep);
// deep: the deep queue's launch (one block per segment, A.nseg segments), else the camera launch
hipError_t launch_chain(const DevScene& S, const LevelArgs& A, hipStream_t stream, KernelProf* prof = nullptr,
                        bool deep = false);
// Scenes with a transparent material: every camera sample's whole color_at tree (reflected and refracted children,
// shade_hit's sums) inside its camera lane with an explicit per-lane stack (render_tree.inc tree_kernel), one launch
// per batch with no recursion queues and no combine passes.  RRAY_NO_TREE=1 keeps the per-level kernels.
bool tree_levels(const DevScene& S);
template <int G, bool LC>
void launch_tree_t(const DevScene& S, const LevelArgs& A, hipStream_t stream, KernelProf* prof);
hipError_t launch_tree(const DevScene& S, const LevelArgs& A, hipStream_t stream, KernelProf* prof = nullptr);
hipError_t launch_aa(const double* canvas, double* out, int64_t width, int64_t rows, int32_t aa, hipStream_t stream,
                     KernelProf* prof = nullptr);
hipError_t launch_aa_f32(const double* canvas, float* out, int64_t width, int64_t rows, int32_t aa, hipStream_t stream,
                         KernelProf* prof = nullptr);
hipError_t launch_shadow_query(const DevScene& S, const double* pts, const double* lps, int64_t n, int32_t* out,
                               unsigned long long* counters, hipStream_t stream);

}  // namespace rr
