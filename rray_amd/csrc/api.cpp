// api.cpp — the C ABI of include/rray/rray.h: device context, scene upload, the wavefront level
// loop that replaces Camera::render (camera.rs:107-121), and the batch query entry points.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rray/rray.h"
#include "device_guard.hpp"
#include "flatten.hpp"
#include "kernels.hpp"
#include "multi.hpp"
#include "partition.hpp"
#include "trace.hpp"
#include "rr_math.hpp"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
#define HIPCHK(expr)                                                                            \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return fail(RR_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));          \
    } while (0)

// grow-only device buffer
struct DBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t want) {
        if (want <= bytes) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        size_t cap = std::max(want, (size_t)256);
        hipError_t e = hipMalloc(&p, cap);
        if (e == hipSuccess) bytes = cap;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T>
    T* as() const {
        return static_cast<T*>(p);
    }
};

}  // namespace

void rr_set_error(const char* msg) { g_err = msg ? msg : ""; }

struct rr_ctx {
    rr_group* group = nullptr;  // multi-device context (multi.cpp): everything below is unused
    int device = 0;
    hipStream_t stream = nullptr;
    bool has_scene = false;
    rr::HostScene host;
    rr::DevScene S{};
    DBuf culls, inner, chunks, nodes, groups, shapes, tris, mats, pats, lights, textures, texels;
    // workspace
    DBuf counters, lcount, hit, n12, n1n2, ev_a, ev_b, canvas, rays0, qout;
    DBuf deep, deep_count;  // chain kernels' deep queue (rr::DeepRec segments) and its segment counters
    // per-tile camera-ray bundles of the last camera / part layout (tile_bundle_kernel), reused while they match
    DBuf tiles;
    struct TileKey {
        rr::DevCamera cam;
        int64_t hs, lrows;
        int32_t aa, part, nparts, block_rows;
        int32_t pw, pad;
    } tile_key{};
    bool tiles_valid = false;
    // level-0 launch order of one-batch fused frames: every wave stores its tile's cost (clock cycles) and the
    // tiles are re-sorted costliest-first on the first frame of a part layout and every kRR_ORDER_EVERY frames
    DBuf tile_cost, tile_perm, tile_hist;
    int64_t order_tiles = 0;  // the layout the order was built for (tiles; key below)
    TileKey order_key{};
    bool order_valid = false;
    uint32_t perm_tail[3] = {0, 0, 0};  // the order's entries past the last tile (their own indices), copied from here
    int order_age = 0;
    std::vector<DBuf> comb, comb_ext, pend;  // one per level (comb_ext: scenes with transparency)
    unsigned long long* h_counters = nullptr;
    // counters: [frame buffer 0][frame buffer 1][queries]; frames alternate (`epoch`), and each
    // frame's first kernels zero the other buffer for the next frame
    int epoch = 0;
    bool zero_next = false;
    unsigned long long* stats_src = nullptr;  // buffer holding the last frame's counters
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipEvent_t ev_in = nullptr, ev_out = nullptr;
    // the stream of the last render (compared, never used: a caller may destroy its stream before the context) and
    // ev_out, recorded after the last render's work on it — what later renders on other streams and the context's
    // teardown wait for (the round-4 teardown hang: rr_destroy synchronised a group's render stream after the group
    // had destroyed it)
    hipStream_t last_st = nullptr;
    bool have_out = false;
    // canvas-path frames: the per-pass box averages run on aa_stream (run_levels AaPasses)
    hipStream_t aa_stream = nullptr;
    std::vector<hipEvent_t> pass_ev;
    hipEvent_t aa_done = nullptr;
    rr_stats last{};
    bool stats_pending = false;
    bool frame_timed = true;  // e0/e1 bracket the last frame
    // camera samples per wavefront pass: large, so that the deep levels of a frame (few, slow,
    // incoherent rays) run once per frame rather than once per batch; the queues of a 2^27-sample
    // pass need ~50 GB at depth 5, well inside the 288 GB of HBM
    int64_t batch = (int64_t)1 << 27;
    // bytes the worst-case recursion queues of one batch may take (run_levels shrinks the batch to fit;
    // half of the free HBM at context creation, RRAY_QUEUE_BUDGET_MB overrides)
    size_t queue_budget = (size_t)32 << 30;
    // per-kernel timing (rr_kernel_times)
    bool profile = false;
    rr::KernelProf prof;
    double kms[rr::K_COUNT] = {0};
    uint64_t kcount[rr::K_COUNT] = {0};
};

namespace {

template <class T>
hipError_t upload(DBuf& b, const std::vector<T>& v, hipStream_t st) {
    hipError_t e = b.ensure(std::max<size_t>(v.size() * sizeof(T), 16));
    if (e != hipSuccess) return e;
    if (!v.empty()) e = hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, st);
    return e;
}

int check_opts(const rr_camera* cam, const rr_render_opts* o) {
    if (!cam || !o) return fail(RR_E_ARG, "null camera/options");
    if (o->aa < 1) return fail(RR_E_ARG, "aa must be >= 1");
    if (o->max_depth < 0 || o->max_depth > RR_MAX_DEPTH) return fail(RR_E_LIMIT, "max_depth out of range");
    if (o->nparts < 1 || o->part < 0 || o->part >= o->nparts) return fail(RR_E_ARG, "bad part/nparts");
    if (cam->hsize <= 0 || cam->vsize <= 0 || cam->hsize % o->aa || cam->vsize % o->aa)
        return fail(RR_E_ARG, "camera size must be a positive multiple of aa");
    if (cam->hsize > (1ll << 31) || cam->vsize > (1ll << 31)) return fail(RR_E_LIMIT, "camera too large");
    if (o->row_begin != 0 || o->row_end != 0) {  // a band of output rows (ABI 10)
        if (o->part != 0 || o->nparts != 1) return fail(RR_E_ARG, "a band (row_begin / row_end) is part 0 of 1");
        if (o->row_begin < 0 || o->row_end <= o->row_begin || o->row_end > cam->vsize / o->aa)
            return fail(RR_E_ARG, "band rows out of range: need 0 <= row_begin < row_end <= height");
    }
    return RR_OK;
}

// output rows of the part (interleaved blocks) or band (rr_render_opts row_begin / row_end)
int64_t opts_rows(const rr_render_opts* o, int64_t H) {
    if (o->row_begin != 0 || o->row_end != 0) return (int64_t)o->row_end - o->row_begin;
    return rr::part_rows_count(H, o->part, o->nparts, o->block_rows > 0 ? o->block_rows : 8);
}

rr::DevCamera dev_camera(const rr_camera* c) {
    rr::DevCamera d{};
    d.hsize = c->hsize;
    d.vsize = c->vsize;
    d.half_width = c->half_width;
    d.half_height = c->half_height;
    d.pixel_size = c->pixel_size;
    rr::M4 t{};
    for (int i = 0; i < 16; ++i) t.m[i] = c->transform[i];
    rr::M4 inv = rr::inverse(t);  // camera.rs:85 (cached inverse, same value)
    for (int i = 0; i < 16; ++i) d.inv[i] = inv.m[i];
    for (int r = 0; r < 4; ++r)  // camera.rs:86 with the kernel's operation order (no contraction)
        d.origin[r] = d.inv[4 * r] * 0.0 + d.inv[4 * r + 1] * 0.0 + d.inv[4 * r + 2] * 0.0 + d.inv[4 * r + 3] * 1.0;
    return d;
}

// Runs the wavefront levels for `total` level-0 events; level-0 rays come from the camera or from
// ctx->rays0 (color_at).  Results (color_at values) land in `out` (3 doubles per event).
// The context's workspace is used on one stream at a time: a call on another stream than the
// previous one first waits for it (one event, only when the stream changes).
hipError_t claim_stream(rr_ctx* c, hipStream_t st) {
    if (c->have_out && c->last_st != st) {
        hipError_t e = hipStreamWaitEvent(st, c->ev_out, 0);
        if (e != hipSuccess) return e;
    }
    c->last_st = st;
    return hipSuccess;
}
// marks the end of the work a call enqueued on `st` (claim_stream and sync_ctx wait for it)
hipError_t release_stream(rr_ctx* c, hipStream_t st) {
    hipError_t e = hipEventRecord(c->ev_out, st);
    if (e == hipSuccess) c->have_out = true;
    return e;
}
// Scope guard of a call's work on `st`: ev_out is recorded on every exit after claim_stream, error returns
// included, so work a failed call already launched is still covered by what the next call and rr_destroy wait for.
struct StreamClaim {
    rr_ctx* c;
    hipStream_t st;
    bool released = false;
    hipError_t release() {
        released = true;
        return release_stream(c, st);
    }
    ~StreamClaim() {
        if (!released) (void)release_stream(c, st);
    }
};
hipError_t sync_ctx(rr_ctx* c) {
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess && c->have_out) e = hipEventSynchronize(c->ev_out);
    return e;
}

constexpr int kRR_ORDER_EVERY = 64;  // frames between re-sorts of the level-0 tile order
constexpr size_t kCounterBytes = (size_t)rr::RR_CNT_SLOTS * rr::RR_CNT_STRIDE * sizeof(unsigned long long);
unsigned long long* frame_counters(rr_ctx* c, int k) {
    return c->counters.as<unsigned long long>() + (size_t)k * rr::RR_CNT_SLOTS * rr::RR_CNT_STRIDE;
}

// Worst-case queue bytes of a batch of nb level-0 events: every shading event queues max_children
// children (k), so level d holds at most nb * k^d events.  The levels are launched for that capacity
// and read their live counts from HBM (no host round trip between levels).
struct LevelPlan {
    int64_t cap[RR_MAX_DEPTH + 1];  // capacity per level (array size; segmented: nseg * seg_cap)
    int64_t seg_cap[RR_MAX_DEPTH + 1];  // segmented (fused) levels >= 1: capacity of each of RR_NSEG segments
    int levels;                     // levels launched (depth + 1, or 1 without secondary rays)
    int64_t ev_cap[2];              // ev_a (odd levels), ev_b (even levels >= 2)
    int64_t max_cap;
    size_t bytes;
};
// fused: levels >= 1 in RR_NSEG segments (wavefront.hpp); level 0's block b fills segment b % RR_NSEG
// of level 1, so a segment holds at most ceil(blocks / RR_NSEG) * 256 * k events, and a segment of
// level d feeds only the same segment of level d + 1
LevelPlan plan_levels(int64_t nb, int k, int max_depth, bool ext, bool fused = false) {
    LevelPlan p{};
    int64_t w = nb;
    for (int d = 0; d <= max_depth; ++d) {
        p.cap[d] = w;
        p.levels = d + 1;
        p.max_cap = std::max(p.max_cap, w);
        const bool kids = d < max_depth && k > 0;
        if (!kids) break;
        p.bytes += (size_t)w * (sizeof(rr::CombRec) + (ext ? sizeof(rr::CombExt) : 0) + sizeof(int32_t));
        if (fused) {
            p.seg_cap[d + 1] = d == 0 ? (((nb + 255) / 256 + rr::RR_NSEG - 1) / rr::RR_NSEG) * 256 * k : p.seg_cap[d] * k;
            p.seg_cap[d + 1] = (p.seg_cap[d + 1] + 255) / 256 * 256;
            w = rr::RR_NSEG * p.seg_cap[d + 1];
        } else {
            w *= k;
        }
        int64_t& e = p.ev_cap[d % 2];  // level d+1 lands in ev_a when d is even
        e = std::max(e, w);
    }
    p.bytes += (size_t)p.max_cap * (sizeof(rr::HitRec) + 2 * sizeof(double) + sizeof(int32_t));
    p.bytes += (size_t)(p.ev_cap[0] + p.ev_cap[1]) * sizeof(rr::Event);
    return p;
}

// pixel waves of a part (A.pw): bands of two output rows, pw_wpb waves each
int64_t pixel_waves(const rr::LevelArgs& A) { return (int64_t)((A.pw_rows + 1) / 2) * A.pw_wpb; }

// level-0 index math: magic divisors, and the wave-uniform tile path when every tile is a full 8x8 and the
// batch starts on a tile boundary
void set_level0_index(rr::LevelArgs& A) {
    A.aa_magic = A.aa > 1 ? (uint32_t)((1ull << 32) / (uint64_t)A.aa) : 0u;
    A.br_magic = A.block_rows > 1 ? (uint32_t)((1ull << 32) / (uint64_t)A.block_rows) : 0u;
    A.tile_fast = !A.rays0 && A.lrows > 0 && A.hs % 8 == 0 && A.lrows % 8 == 0 && A.base % 64 == 0 ? 1 : 0;
    A.tiles_per_row = (uint32_t)(A.hs / 8);
}

// The per-tile camera bundles of this render's part (tile_bundle_kernel), recomputed only when the camera or
// the part layout changed since the last render on this context.  Null when the tiles are not all full 8x8
// or the camera is not affine (the walks build their bundles themselves then).
int tile_bundles(rr_ctx* c, const rr::LevelArgs& base_args, hipStream_t st, const float** out) {
    *out = nullptr;
    rr::LevelArgs T = base_args;
    T.base = 0;
    T.level = 0;
    set_level0_index(T);
    if ((!T.tile_fast && !T.pw) || !T.cam_affine) return RR_OK;
    // few-node flat scenes with LDS culls walk node by node without bundles (walk_nodes)
    if (!c->S.has_groups && !c->S.general && c->S.lds_culls && c->S.n_nodes <= rr::RR_BUNDLE_MIN_NODES) return RR_OK;
    // one bundle per 8x8 tile, or per pixel wave (A.pw)
    const int64_t n_tiles = T.pw ? pixel_waves(T) : T.hs * T.lrows / 64;
    const size_t want = (size_t)n_tiles * rr::RR_TILE_BUNDLE_FLOATS * sizeof(float);
    if (want > c->tiles.bytes) {
        HIPCHK(c->tiles.ensure(want));
        c->tiles_valid = false;
    }
    rr_ctx::TileKey key{};
    key.cam = T.cam;
    key.hs = T.hs;
    key.lrows = T.lrows;
    key.aa = T.aa;
    key.part = T.part;
    key.nparts = T.nparts;
    key.block_rows = T.block_rows;
    key.pw = T.pw;
    if (!c->tiles_valid || std::memcmp(&key, &c->tile_key, sizeof key) != 0) {
        if (T.pw)
            HIPCHK(rr::launch_pixel_wave_bundles(T, c->tiles.as<float>(), n_tiles, st));
        else
            HIPCHK(rr::launch_tile_bundles(c->S, T, c->tiles.as<float>(), n_tiles, st));
        c->tile_key = key;
        c->tiles_valid = true;
    }
    *out = c->tiles.as<float>();
    return RR_OK;
}

// The averaged image can be written by the level-0 waves themselves (deliver_wave_avg) when every
// pixel's samples lie in one wave's 8x8 tile (aa in {2, 4, 8}, full tiles: the tile_fast layout) and no
// sample spawns a secondary ray (fused levels with no reflective / transparent material, or depth 0).
bool wave_avg_ok(const rr_ctx* c, int32_t aa, int64_t hs, int64_t local_rows, int max_depth) {
    // (reflection chains run inside the level-0 wave, chain_levels: every sample is final in its wave too)
    // (and the color_at trees of transparent scenes, tree_levels, likewise)
    return (aa == 2 || aa == 4 || aa == 8) && hs % 8 == 0 && local_rows % 8 == 0 && local_rows > 0 &&
           ((rr::fused_levels(c->S) &&
             (c->host.max_children == 0 || max_depth == 0 || rr::chain_levels(c->S, c->host.max_children, max_depth))) ||
            rr::tree_levels(c->S));
}

// The box average of a canvas-path frame (aa outside the in-wave cases, e.g. C3's aa = 3) overlapped with the
// render: the frame runs in passes of whole output rows, and each pass's rows are averaged on the context's
// second stream while the next pass renders (the render is VALU-bound, the average HBM-bound).  Null: no passes.
struct AaPasses {
    void* avg;
    int32_t f32;
    int64_t width;  // output pixels per row
    int32_t aa;
};

int run_levels(rr_ctx* c, const rr::LevelArgs& base_args, int64_t total, int max_depth, double* out, hipStream_t st,
               void* avg = nullptr, int32_t avg_f32 = 0, int32_t aa_wave = 0, const AaPasses* aap = nullptr) {
    const bool ext = c->host.has_transparent != 0;
    const bool fused = rr::fused_levels(c->S);
    // reflection chains inside the level-0 waves (chain_kernel), or the color_at trees of transparent scenes
    // (tree_kernel): one level, no recursion queues
    const bool tree = rr::tree_levels(c->S);
    const bool chain = tree || rr::chain_levels(c->S, c->host.max_children, max_depth);
    const int k = chain ? 0 : c->host.max_children;
    const int plan_depth = chain ? 0 : max_depth;
    // batch: at most c->batch camera samples, shrunk (power-of-two steps, tile-aligned) until the
    // worst-case queues fit the context's budget and every event index fits in int32
    int64_t B = std::max<int64_t>(64, std::min<int64_t>(c->batch, total));
    for (;;) {
        const LevelPlan p = plan_levels(B, k, plan_depth, ext, fused);
        const int64_t last = p.cap[p.levels - 1];
        if (B <= 4096 || (p.bytes <= c->queue_budget && last < ((int64_t)1 << 31) && p.max_cap < ((int64_t)1 << 31)))
            break;
        B = std::max<int64_t>(4096, (B / 2) & ~(int64_t)63);
    }
    // AA passes: batches of whole output rows (a multiple of lcm(8, aa) sample rows, so every batch is whole
    // 8-row tile bands and whole pixels), about kRR_AA_PASSES of them
    bool passes = false;
    if (aap && out && !base_args.rays0 && base_args.hs % 8 == 0 && base_args.lrows % 8 == 0) {
        int64_t rows_unit = 8;
        while (rows_unit % aap->aa) rows_unit += 8;
        const int64_t unit = rows_unit * base_args.hs;
        const int64_t units = total / unit;
        // default one pass: measured on C3 (chain kernel), 2 / 4 / 8 passes cost 7.29 / 7.61 / 8.01 ms per frame
        // against 7.08 — each pass ends in its own tail of long chains, and the averages did not overlap it
        const int np = std::max(1, std::atoi(std::getenv("RRAY_AA_PASSES") ? std::getenv("RRAY_AA_PASSES") : "1"));
        if (total % unit == 0 && units >= 2 && np > 1 && B >= unit) {
            const int64_t per = std::min((units + np - 1) / np, B / unit);
            B = per * unit;
            passes = true;
            if (!c->aa_stream) HIPCHK(hipStreamCreateWithFlags(&c->aa_stream, hipStreamNonBlocking));
        }
    }
    const LevelPlan P = plan_levels(B, k, plan_depth, ext, fused);
    if (P.max_cap >= ((int64_t)1 << 31)) return fail(RR_E_LIMIT, "recursion queues exceed 2^31 events (lower max_depth)");
    if ((int)c->comb.size() < P.levels) {
        c->comb.resize(P.levels);
        c->comb_ext.resize(P.levels);
        c->pend.resize(P.levels);
    }
    if (!fused && !tree) {  // hit records and n1/n2 lists: the unfused trace / n1n2 / shade kernels only
        HIPCHK(c->hit.ensure(P.max_cap * sizeof(rr::HitRec)));
        HIPCHK(c->n12.ensure(P.max_cap * 2 * sizeof(double)));
        HIPCHK(c->n1n2.ensure(P.max_cap * sizeof(int32_t)));
    }
    for (int d = 0; d + 1 < P.levels; ++d) {
        HIPCHK(c->comb[d].ensure(P.cap[d] * sizeof(rr::CombRec)));
        if (ext) HIPCHK(c->comb_ext[d].ensure(P.cap[d] * sizeof(rr::CombExt)));
        HIPCHK(c->pend[d].ensure(P.cap[d] * sizeof(int32_t)));
    }
    if (P.ev_cap[0]) HIPCHK(c->ev_a.ensure(P.ev_cap[0] * sizeof(rr::Event)));
    if (P.ev_cap[1]) HIPCHK(c->ev_b.ensure(P.ev_cap[1] * sizeof(rr::Event)));
    unsigned int* lc = c->lcount.as<unsigned int>();
    // deep chains (chain_kernel DEEP): frames whose samples are delivered one by one (not the in-wave AA average)
    // can send the chains still reflecting at depth RR_DEEP_FROM to a packed, segmented queue for a second launch.
    // Opt-in (RRAY_DEEP=1): on C3 the deep launch took 1.85 ms for what the camera waves did in 1.54 — the deep
    // rays' walks are latency-bound whether their waves are full or not
    const bool spill = chain && !tree && aa_wave == 0 && !base_args.pw && max_depth >= rr::RR_DEEP_FROM && std::getenv("RRAY_DEEP") &&
                       std::atoi(std::getenv("RRAY_DEEP")) == 1;
    const int64_t deep_seg_cap = (int64_t)256 << rr::RR_DEEP_SHIFT;
    const int64_t deep_nseg = (((B + 255) / 256) + (1 << rr::RR_DEEP_SHIFT) - 1) >> rr::RR_DEEP_SHIFT;
    if (spill) HIPCHK(c->deep.ensure((size_t)deep_nseg * deep_seg_cap * sizeof(rr::DeepRec)));
    if (spill && (size_t)(deep_nseg + 2) * sizeof(unsigned int) > c->deep_count.bytes)
        HIPCHK(c->deep_count.ensure((size_t)(deep_nseg + 2) * sizeof(unsigned int)));
    // cost-ordered level-0 tiles: one-batch fused frames of full 8x8 tiles whose level 0 is the whole frame (no
    // secondary rays) in scenes with groups, where tile costs spread widest (mesh silhouettes against floor:
    // C4 0.596 -> 0.511 ms per frame).  Flat scenes' tiles cost alike (C2 +0.6 % with the order), and frames
    // with reflections lose their children queues' tile order (C3 +2 %): both keep launch order.
    rr::LevelArgs T0 = base_args;
    T0.base = 0;
    set_level0_index(T0);
    // chain frames order their camera waves too (tiles or pixel waves; the chains' depths spread tile costs widely)
    const int64_t n_tiles = T0.pw ? pixel_waves(T0) : T0.tile_fast ? T0.hs * T0.lrows / 64 : 0;
    // the order's unit: single waves, so a block's four waves cost alike (the costliest first) and the block's
    // resources free together.  Groups of a block's four adjacent tiles (RRAY_ORDER_GROUP=4: their output rows join
    // into whole cache lines) measured slower: C3 6.33 vs 7.17 ms, C4 0.510 vs 0.520 ms, C5 equal
    int order_group = 1;
    if (const char* g = std::getenv("RRAY_ORDER_GROUP")) order_group = std::atoi(g) == rr::RR_ORDER_GROUP ? rr::RR_ORDER_GROUP : 1;
    const bool order_ok = (fused || tree) && !c->S.general && B >= total && n_tiles > 0 && n_tiles < ((int64_t)1 << 31) &&
                          (order_group == 1 || n_tiles % 4 == 0) &&  // the group order permutes a block's four tiles
                          (T0.pw || n_tiles * 64 == total) &&
                          ((c->S.has_groups && (k == 0 || max_depth == 0)) || (chain && !std::getenv("RRAY_NO_CHAIN_ORDER")));
    // the launch's last block may hold up to three wave slots past the last tile (n_tiles not a multiple of 4: a
    // pixel-wave part of 270 output rows has 148 230 waves): the order and cost arrays run to whole blocks, the extra
    // slots' order entries are their own indices (their lanes are past the launch's samples and do nothing but record
    // a cost nobody sorts).  Until round 6 such layouts ran unordered: C3's 8-part rows among them.
    const int64_t n_pad = (n_tiles + 3) & ~(int64_t)3;
    if (order_ok) {
        HIPCHK(c->tile_cost.ensure((size_t)n_pad * sizeof(uint32_t)));
        HIPCHK(c->tile_perm.ensure((size_t)n_pad * sizeof(uint32_t)));
        HIPCHK(c->tile_hist.ensure(256 * sizeof(uint32_t)));
        rr_ctx::TileKey key{};  // the layout only: a camera change keeps the order (costs stay a good guess)
        key.hs = T0.hs;
        key.lrows = T0.lrows;
        key.aa = T0.aa;
        key.part = T0.part;
        key.nparts = T0.nparts;
        key.block_rows = T0.block_rows;
        key.pw = T0.pw;
        key.pad = (chain ? 1 : 0) | (order_group == 1 ? 2 : 0);  // chain and level-0-only frames of one layout, and
                                                                  // each order unit, keep orders of their own
        if (c->order_tiles != n_tiles || std::memcmp(&key, &c->order_key, sizeof key) != 0) {
            c->order_valid = false;
            c->order_tiles = n_tiles;
            c->order_key = key;
            if (n_pad > n_tiles) {  // the identity for the slots past the last tile
                for (int64_t t = n_tiles; t < n_pad; ++t) c->perm_tail[t - n_tiles] = (uint32_t)t;
                HIPCHK(hipMemcpyAsync(c->tile_perm.as<uint32_t>() + n_tiles, c->perm_tail,
                                      (size_t)(n_pad - n_tiles) * sizeof(uint32_t), hipMemcpyHostToDevice, st));
            }
        }
        // a layout's first frame: order by a guess from the camera bundles (launch order left the first frame's
        // slowest tiles last: C4 0.59 vs 0.51 ms), and re-sort by the measured costs right after it
        if (!c->order_valid && T0.tile_bundles && !std::getenv("RRAY_NO_TILE_GUESS")) {
            HIPCHK(rr::launch_tile_guess(c->S, T0.tile_bundles, c->tile_cost.as<uint32_t>(), n_tiles, st));
            HIPCHK(rr::launch_tile_order(c->tile_cost.as<uint32_t>(), c->tile_perm.as<uint32_t>(),
                                         c->tile_hist.as<uint32_t>(), n_tiles, order_group, st));
            c->order_valid = true;
            c->order_age = kRR_ORDER_EVERY - 1;
        }
    }
    for (int64_t base = 0; base < total; base += B) {
        const int64_t nb = std::min(B, total - base);
        const LevelPlan p = plan_levels(nb, k, plan_depth, ext, fused);
        // per-level queue counters [level][LC_*], zeroed once per batch (appends, pending, n1/n2 lists)
        // (the in-wave chains and trees use none: no memset in their frames, which cost a C1 frame 9.6 us as two fills)
        if (p.levels > 1 || (ext && !tree))
            HIPCHK(hipMemsetAsync(lc, 0, (size_t)p.levels * rr::LC_COUNT * sizeof(unsigned int), st));
        if (spill) HIPCHK(hipMemsetAsync(c->deep_count.p, 0, (size_t)deep_nseg * sizeof(unsigned int), st));
        for (int d = 0; d < p.levels; ++d) {
            const bool children_possible = d + 1 < p.levels;
            rr::LevelArgs A = base_args;
            A.base = base;
            set_level0_index(A);
            A.level = d;
            A.rem = max_depth - d;
            A.n = p.cap[d];
            A.n_dev = d > 0 ? lc + (d - 1) * rr::LC_COUNT + rr::LC_CHILDREN : nullptr;
            A.nseg = fused && d > 0 ? rr::RR_NSEG : 1;
            A.nseg_out = fused ? rr::RR_NSEG : 1;
            A.seg_cap = fused && d > 0 ? p.seg_cap[d] : 0;
            A.seg_cap_out = fused && children_possible ? p.seg_cap[d + 1] : 0;
            A.seg_count = lc + d * rr::LC_COUNT + rr::LC_SEG0;
            A.seg_out_count = children_possible ? lc + (d + 1) * rr::LC_COUNT + rr::LC_SEG0 : nullptr;
            // level d reads ev_b when d is even (d >= 2), ev_a when odd; writes the other one
            A.ev = d == 0 ? nullptr : (d % 2 ? c->ev_a : c->ev_b).as<rr::Event>();
            A.hit = c->hit.as<rr::HitRec>();
            A.n12 = c->n12.as<double>();
            A.comb = children_possible ? c->comb[d].as<rr::CombRec>() : nullptr;
            A.parent_comb = d > 0 ? c->comb[d - 1].as<rr::CombRec>() : nullptr;
            A.comb_ext = ext && children_possible ? c->comb_ext[d].as<rr::CombExt>() : nullptr;
            A.parent_ext = ext && d > 0 ? c->comb_ext[d - 1].as<rr::CombExt>() : nullptr;
            for (int q = 0; q <= RR_MAX_DEPTH; ++q)
                A.chain[q] = q + 1 < p.levels ? c->comb[q].as<rr::ChainRec>() : nullptr;
            A.out = out;
            A.avg = avg;
            A.avg_f32 = avg_f32;
            A.aa_wave = (d == 0 && A.tile_fast) ? aa_wave : 0;
            if (A.pw) {  // pixel waves: the launch holds whole waves of 7 pixels (one batch, chain kernels only)
                if (!chain || B < total) return fail(RR_E_ARG, "internal: pixel waves need one chain-kernel batch");
                A.n = pixel_waves(A) * 64;
            }
            // fused levels queue each wave's reflected rays in a 64-slot block of its own, at the lanes they
            // left (holes marked): a secondary wave is one camera tile's rays, as coherent as they come.
            // Packed queues mixed 2-4 tiles per wave (C3 10.54 -> 8.98 ms with the blocks); the area-light
            // scenes' block-wide sample dealing prefers packed waves (C5 2.27 vs 2.30 ms)
            A.pad_children = fused && !c->S.has_area ? 1 : 0;
            if (aa_wave && !A.aa_wave) return fail(RR_E_ARG, "internal: in-wave AA average without full tiles");
            // null when no material is reflective or transparent (or at the last level)
            A.next = children_possible ? (d % 2 ? c->ev_b : c->ev_a).as<rr::Event>() : nullptr;
            A.pending = children_possible ? c->pend[d].as<int32_t>() : nullptr;
            A.n1n2_list = c->n1n2.as<int32_t>();
            A.lcount = lc + d * rr::LC_COUNT;
            if (order_ok && d == 0) {
                A.tile_perm = c->order_valid ? c->tile_perm.as<uint32_t>() : nullptr;
                // the waves record their costs only in a frame the sort below reads (every kRR_ORDER_EVERY-th):
                // each record is one scattered 4-byte store per wave, a partial line that L2 writes back alone
                // (47 MB of the C3 chain kernel's 0.55 GB of writes per frame, profiles/r05/attrib_c3.txt)
                const bool sort_after = !c->order_valid || c->order_age + 1 >= kRR_ORDER_EVERY;
                A.tile_cost = sort_after ? c->tile_cost.as<uint32_t>() : nullptr;
                A.order_group = order_group;
            }
            A.counters = frame_counters(c, c->epoch);
            A.counters_zero = (c->zero_next && d == 0 && base == 0) ? frame_counters(c, c->epoch ^ 1) : nullptr;
            if (tree) {
                HIPCHK(rr::launch_tree(c->S, A, st, c->profile ? &c->prof : nullptr));
            } else if (chain) {
                if (spill) {  // camera launch appends to the deep queue's segments (level 1's counters)
                    A.deep = c->deep.as<rr::DeepRec>();
                    A.deep_from = rr::RR_DEEP_FROM;
                    A.nseg_out = (int32_t)deep_nseg;
                    A.seg_out_count = c->deep_count.as<unsigned int>();
                    A.seg_cap_out = deep_seg_cap;
                }
                HIPCHK(rr::launch_chain(c->S, A, st, c->profile ? &c->prof : nullptr));
                if (spill) {  // the deep launch: one block per segment
                    rr::LevelArgs D = A;
                    D.nseg = (int32_t)deep_nseg;
                    D.seg_count = A.seg_out_count;
                    D.seg_cap = deep_seg_cap;
                    D.seg_out_count = nullptr;
                    D.counters_zero = nullptr;
                    HIPCHK(rr::launch_chain(c->S, D, st, c->profile ? &c->prof : nullptr, true));
                }
            } else
                HIPCHK(rr::launch_level(c->S, A, st, c->profile ? &c->prof : nullptr));
            if (order_ok && d == 0 && (!c->order_valid || ++c->order_age >= kRR_ORDER_EVERY)) {
                HIPCHK(rr::launch_tile_order(c->tile_cost.as<uint32_t>(), c->tile_perm.as<uint32_t>(),
                                             c->tile_hist.as<uint32_t>(), n_tiles, order_group, st));
                c->order_valid = true;
                c->order_age = 0;
            }
        }
        // bottom-up shade_hit sums of the events with children (scene.rs:172-177); fused levels finish
        // their chains in the kernels
        for (int d = p.levels - 2; d >= 0 && !rr::fused_levels(c->S); --d) {
            rr::CombArgs C{};
            C.level = d;
            C.n = p.cap[d];
            C.n_dev = lc + d * rr::LC_COUNT + rr::LC_PENDING;
            C.base = base;
            C.pending = c->pend[d].as<int32_t>();
            C.comb = c->comb[d].as<rr::CombRec>();
            C.parent_comb = d > 0 ? c->comb[d - 1].as<rr::CombRec>() : nullptr;
            C.comb_ext = ext ? c->comb_ext[d].as<rr::CombExt>() : nullptr;
            C.parent_ext = ext && d > 0 ? c->comb_ext[d - 1].as<rr::CombExt>() : nullptr;
            C.out = out;
            C.avg = avg;
            C.avg_f32 = avg_f32;
            C.hs = base_args.hs;
            C.lrows = base_args.rays0 ? 0 : base_args.lrows;
            HIPCHK(rr::launch_combine(C, st, c->profile ? &c->prof : nullptr));
        }
        if (passes) {  // this batch's output rows, averaged on the second stream after the batch
            const int64_t y0 = base / base_args.hs / aap->aa, y1 = (base + nb) / base_args.hs / aap->aa;
            const size_t pi = (size_t)(base / B);
            while (c->pass_ev.size() <= pi) {
                hipEvent_t e = nullptr;
                HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
                c->pass_ev.push_back(e);
            }
            HIPCHK(hipEventRecord(c->pass_ev[pi], st));
            HIPCHK(hipStreamWaitEvent(c->aa_stream, c->pass_ev[pi], 0));
            const double* src = out + 3 * y0 * aap->aa * base_args.hs;
            if (aap->f32)
                HIPCHK(rr::launch_aa_f32(src, static_cast<float*>(aap->avg) + 3 * y0 * aap->width, aap->width, y1 - y0,
                                         aap->aa, c->aa_stream, c->profile ? &c->prof : nullptr));
            else
                HIPCHK(rr::launch_aa(src, static_cast<double*>(aap->avg) + 3 * y0 * aap->width, aap->width, y1 - y0,
                                     aap->aa, c->aa_stream, c->profile ? &c->prof : nullptr));
        }
    }
    if (passes) {  // the caller's stream continues after the last pass's average
        HIPCHK(hipEventRecord(c->aa_done, c->aa_stream));
        HIPCHK(hipStreamWaitEvent(st, c->aa_done, 0));
    } else if (aap) {  // one pass: the average follows on the caller's stream
        const int64_t rows = total / base_args.hs / aap->aa;
        if (aap->f32)
            HIPCHK(rr::launch_aa_f32(out, static_cast<float*>(aap->avg), aap->width, rows, aap->aa, st,
                                     c->profile ? &c->prof : nullptr));
        else
            HIPCHK(rr::launch_aa(out, static_cast<double*>(aap->avg), aap->width, rows, aap->aa, st,
                                 c->profile ? &c->prof : nullptr));
    }
    return RR_OK;
}

void collect_stats(rr_ctx* c, rr_stats* s) {
    std::memset(s, 0, sizeof(*s));
    unsigned long long h[rr::RR_CNT_STRIDE] = {};
    for (int sl = 0; sl < rr::RR_CNT_SLOTS; ++sl)
        for (int k = 0; k < rr::C_COUNT; ++k) h[k] += c->h_counters[sl * rr::RR_CNT_STRIDE + k];
    s->rays = h[rr::C_RAYS];
    s->shadow_rays = h[rr::C_SHADOW];
    s->shade_events = h[rr::C_SHADE];
    s->n1n2_scans = h[rr::C_N1N2];
    s->group_tests = h[rr::C_GROUP_TESTS];
    s->group_hits = h[rr::C_GROUP_HITS];
    s->samples = h[rr::C_SAMPLES];
    s->prim_tests = h[rr::C_PRIM_TESTS];
    for (int k = 0; k < 3; ++k) {
        s->exact_flops[k] = h[rr::C_FLOPS_TRACE + k];
        s->wave_visits[k] = h[rr::C_VISITS_TRACE + k];
    }
    s->nan_rays = h[rr::C_NAN];
}
int nan_fail(uint64_t n) {
    return fail(RR_E_NAN, std::to_string(n) +
                              " ray(s) met a NaN intersection t in a list of >= 2 entries: the reference panics in "
                              "Vec::sort_by(partial_cmp().unwrap()) (scene.rs:104)");
}

int resolve_prof(rr_ctx* c) {
    for (auto& m : c->prof.marks) {
        HIPCHK(hipEventSynchronize(m.second.second));
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, m.second.first, m.second.second));
        c->kms[m.first] += ms;
        c->kcount[m.first] += 1;
    }
    c->prof.marks.clear();
    c->prof.used = 0;
    return RR_OK;
}

int finish_stats(rr_ctx* c) {
    if (!c->stats_pending) return RR_OK;
    float ms = 0.f;
    if (c->frame_timed) {
        HIPCHK(hipEventSynchronize(c->e1));
        HIPCHK(hipEventElapsedTime(&ms, c->e0, c->e1));
    } else {
        HIPCHK(sync_ctx(c));
    }
    // the counters of the last render stay in HBM until the next one zeroes them: copy on demand
    // (a per-frame device-to-host copy behind a cross-stream wait blocks the host in HIP)
    HIPCHK(hipMemcpy(c->h_counters, c->stats_src ? c->stats_src : frame_counters(c, c->epoch), kCounterBytes,
                     hipMemcpyDeviceToHost));
    collect_stats(c, &c->last);
    c->last.kernel_ms = ms;
    c->stats_pending = false;
    return RR_OK;
}

}  // namespace

namespace rr {
// Every check rr_render_device makes before it enqueues anything (the multi-device group validates all
// of its parts with it first, so a bad argument never leaves peers waiting in a collective).
int render_validate(rr_ctx* c, const rr_camera* cam, const rr_render_opts* o) {
    if (!c) return fail(RR_E_ARG, "null context");
    if (c->group) return fail(RR_E_ARG, "multi-device context: use rr_render_gather_device or rr_render");
    if (!c->has_scene) return fail(RR_E_ARG, "no scene uploaded");
    int rc = check_opts(cam, o);
    if (rc != RR_OK) return rc;
    const int64_t rows = opts_rows(o, cam->vsize / o->aa);
    if (rows * o->aa * cam->hsize >= ((int64_t)1 << 31))
        return fail(RR_E_LIMIT, "a part must hold fewer than 2^31 samples (use more parts)");
    return RR_OK;
}
}  // namespace rr

extern "C" {

int32_t rr_abi_version(void) { return RR_ABI_VERSION; }
const char* rr_last_error(void) { return g_err.c_str(); }

int rr_device_count(int* out) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    if (out) *out = n;
    return e == hipSuccess ? RR_OK : fail(RR_E_HIP, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
}

int rr_create(int device, rr_ctx** out) {
    rr::DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!out) return fail(RR_E_ARG, "null out");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(RR_E_HIP, "no HIP device available");
    if (device < 0 || device >= n) return fail(RR_E_ARG, "device index out of range");
    HIPCHK(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(RR_E_HIP, std::string("device is ") + prop.gcnArchName + ", this build targets gfx950 only");
    rr_ctx* c = new rr_ctx();
    c->device = device;
    if (const char* b = std::getenv("RRAY_BATCH")) c->batch = std::max<int64_t>(1024, std::atoll(b));
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0) c->queue_budget = free_b / 2;
    if (const char* q = std::getenv("RRAY_QUEUE_BUDGET_MB")) c->queue_budget = (size_t)std::max(1ll, std::atoll(q)) << 20;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&c->e0);
    if (e == hipSuccess) e = hipEventCreate(&c->e1);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_out, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->aa_done, hipEventDisableTiming);
    if (e == hipSuccess)
        e = hipHostMalloc((void**)&c->h_counters, kCounterBytes, hipHostMallocDefault);
    if (e == hipSuccess) e = c->counters.ensure(3 * kCounterBytes);
    if (e == hipSuccess) e = hipMemset(c->counters.p, 0, 3 * kCounterBytes);
    if (e == hipSuccess) e = c->lcount.ensure((RR_MAX_DEPTH + 1) * rr::LC_COUNT * sizeof(unsigned int));
    if (e != hipSuccess) {
        rr_destroy(c);
        return fail(RR_E_HIP, std::string("context setup: ") + hipGetErrorString(e));
    }
    *out = c;
    return RR_OK;
}

int rr_create_multi(int n, const int* device_ids, rr_ctx** out) {
    rr::DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!out) return fail(RR_E_ARG, "null out");
    *out = nullptr;
    rr_group* g = nullptr;
    int rc = rr::group_create_local(n, device_ids, &g);
    if (rc != RR_OK) return rc;
    rr_ctx* c = new rr_ctx();
    c->group = g;
    *out = c;
    return RR_OK;
}

int rr_create_rank(int device, int nranks, int rank, const uint8_t* unique_id, rr_ctx** out) {
    rr::DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!out) return fail(RR_E_ARG, "null out");
    *out = nullptr;
    rr_group* g = nullptr;
    int rc = rr::group_create_rank(device, nranks, rank, unique_id, &g);
    if (rc != RR_OK) return rc;
    rr_ctx* c = new rr_ctx();
    c->group = g;
    *out = c;
    return RR_OK;
}

int rr_context_info(const rr_ctx* c, int32_t* nranks, int32_t* rank, int32_t* ndevices) {
    if (!c) return fail(RR_E_ARG, "null context");
    if (c->group) return rr::group_info(c->group, nranks, rank, ndevices);
    if (nranks) *nranks = 1;
    if (rank) *rank = 0;
    if (ndevices) *ndevices = 1;
    return RR_OK;
}

void rr_destroy(rr_ctx* c) {
    rr::DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!c) return;
    if (c->group) {
        rr::group_destroy(c->group);
        delete c;
        return;
    }
    (void)hipSetDevice(c->device);
    rr::trace("rr_destroy %p: synchronise", (void*)c);
    if (c->stream) (void)sync_ctx(c);
    rr::trace("rr_destroy %p: free", (void*)c);
    for (DBuf* b : {&c->culls, &c->inner, &c->chunks, &c->nodes, &c->groups, &c->shapes, &c->tris, &c->mats, &c->pats, &c->lights, &c->textures, &c->texels, &c->counters,
                    &c->lcount, &c->hit, &c->n12, &c->n1n2, &c->ev_a, &c->ev_b, &c->canvas, &c->rays0, &c->qout, &c->tiles,
                    &c->tile_cost, &c->tile_perm, &c->tile_hist, &c->deep, &c->deep_count})
        b->release();
    for (auto& b : c->comb) b.release();
    for (auto& b : c->comb_ext) b.release();
    for (auto& b : c->pend) b.release();
    for (hipEvent_t e : c->prof.pool) (void)hipEventDestroy(e);
    if (c->h_counters) (void)hipHostFree(c->h_counters);
    if (c->e0) (void)hipEventDestroy(c->e0);
    if (c->e1) (void)hipEventDestroy(c->e1);
    if (c->ev_in) (void)hipEventDestroy(c->ev_in);
    if (c->ev_out) (void)hipEventDestroy(c->ev_out);
    if (c->aa_done) (void)hipEventDestroy(c->aa_done);
    for (hipEvent_t e : c->pass_ev) (void)hipEventDestroy(e);
    if (c->aa_stream) (void)hipStreamDestroy(c->aa_stream);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    rr::trace("rr_destroy %p: done", (void*)c);
    delete c;
}

int rr_scene_upload(rr_ctx* c, const rr_scene_desc* d) {
    rr::DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!c || !d) return fail(RR_E_ARG, "null context/descriptor");
    if (c->group) return rr::group_upload(c->group, d);
    std::string err;
    rr::HostScene hs;
    int rc = rr::flatten_scene(*d, hs, err);
    if (rc != RR_OK) return fail(rc, err);
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(sync_ctx(c));  // renders in flight may still read the previous scene
    hipStream_t st = c->stream;
    HIPCHK(upload(c->culls, hs.culls, st));
    HIPCHK(upload(c->inner, hs.inner, st));
    HIPCHK(upload(c->chunks, hs.chunks, st));
    HIPCHK(upload(c->nodes, hs.nodes, st));
    HIPCHK(upload(c->groups, hs.groups, st));
    HIPCHK(upload(c->shapes, hs.shapes, st));
    HIPCHK(upload(c->tris, hs.tris, st));
    HIPCHK(upload(c->mats, hs.mats, st));
    HIPCHK(upload(c->pats, hs.pats, st));
    HIPCHK(upload(c->lights, hs.lights, st));
    HIPCHK(upload(c->textures, hs.textures, st));
    HIPCHK(upload(c->texels, hs.texels, st));
    HIPCHK(hipStreamSynchronize(st));
    c->host = std::move(hs);
    // the level-0 tile order is the previous scene's tile costs: drop it (the next frame records new ones).
    // The tile bundles depend on the camera only; they are rebuilt too, for a clean start
    c->order_valid = false;
    c->order_age = 0;
    c->tiles_valid = false;
    rr::DevScene& S = c->S;
    S.culls = c->culls.as<rr::DevCull>();
    S.inner = c->inner.as<rr::DevCull>();
    S.chunks = c->chunks.as<rr::DevChunk>();
    S.n_chunks = (int32_t)c->host.chunks.size();
    S.n_free = 0;
    for (int k = S.n_chunks - 1; k >= 0; --k) {  // lone unbounded top-level leaves at the end of the order
        const rr::DevChunk& ch = c->host.chunks[k];
        const rr::DevNode& nd = c->host.nodes[ch.start];
        if (ch.count != 1 || ch.cull.r < HUGE_VALF || nd.parent != -1 || rr::is_container(nd.kind) ||
            ch.start != (int32_t)c->host.nodes.size() - 1 - S.n_free)
            break;
        ++S.n_free;
    }
    S.free_planes = 1;
    for (int k = 0; k < S.n_free; ++k) {
        const rr::DevNode& nd = c->host.nodes[c->host.nodes.size() - 1 - k];
        if (nd.kind != RR_PLANE || !(nd.flags & rr::NF_IDENT)) S.free_planes = 0;
    }
    S.nodes = c->nodes.as<rr::DevNode>();
    S.groups = c->groups.as<rr::DevGroup>();
    S.shapes = c->shapes.as<rr::DevShape>();
    S.tris = c->tris.as<rr::DevTri>();
    S.mats = c->mats.as<rr::DevMaterial>();
    S.pats = c->pats.as<rr::DevPattern>();
    S.lights = c->lights.as<rr::DevLight>();
    S.textures = c->textures.as<rr::DevTexture>();
    S.texels = c->texels.as<uint32_t>();
    S.n_nodes = (int32_t)c->host.nodes.size();
    S.n_lights = (int32_t)c->host.lights.size();
    S.has_transparent = c->host.has_transparent;
    S.has_area = 0;
    for (const rr::DevLight& l : c->host.lights) S.has_area |= l.kind == RR_LIGHT_AREA ? 1 : 0;
    S.complex_patterns = c->host.complex_patterns;
    S.tri_inline = c->host.tri_inline;
    S.has_groups = c->host.groups.empty() ? 0 : 1;
    S.general = (c->host.has_csg || c->host.has_quad) ? 1 : 0;
    const size_t lds_bytes = (size_t)S.n_nodes * sizeof(rr::DevCull) + (size_t)S.n_chunks * sizeof(rr::DevChunk);
    S.lds_culls = (lds_bytes <= (size_t)rr::RR_LDS_CULL_BYTES && !std::getenv("RRAY_GLOBAL_CULLS")) ? 1 : 0;
    // sphere around the bounded nodes' culls (make_bundle moves far ray origins next to it)
    {
        double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
        bool any = false;
        for (const rr::DevCull& cl : c->host.culls) {
            if (!(cl.r < HUGE_VALF)) continue;
            any = true;
            for (int k = 0; k < 3; ++k) {
                lo[k] = std::min(lo[k], (double)cl.c[k] - cl.r);
                hi[k] = std::max(hi[k], (double)cl.c[k] + cl.r);
            }
        }
        S.bs_r = -1.0f;
        if (any && std::isfinite(hi[0] - lo[0]) && std::isfinite(hi[1] - lo[1]) && std::isfinite(hi[2] - lo[2])) {
            double r = 0.0;
            for (int k = 0; k < 3; ++k) S.bs_c[k] = (float)(0.5 * (lo[k] + hi[k]));
            for (const rr::DevCull& cl : c->host.culls) {
                if (!(cl.r < HUGE_VALF)) continue;
                const double dx = cl.c[0] - S.bs_c[0], dy = cl.c[1] - S.bs_c[1], dz = cl.c[2] - S.bs_c[2];
                r = std::max(r, std::sqrt(dx * dx + dy * dy + dz * dz) + cl.r);
            }
            if (r < 1e30) S.bs_r = (float)r;
        }
    }
    c->has_scene = true;
    return RR_OK;
}

int rr_scene_inspect(const rr_scene_desc* d, double* inverses, double* group_aabbs, int32_t* node_of_object) {
    if (!d) return fail(RR_E_ARG, "null descriptor");
    std::string err;
    rr::HostScene hs;
    int rc = rr::flatten_scene(*d, hs, err);
    if (rc != RR_OK) return fail(rc, err);
    for (int i = 0; i < d->n_objects; ++i) {
        int node = hs.node_of_object[i];
        if (node_of_object) node_of_object[i] = node;
        if (inverses) {
            double* o = inverses + 16 * (size_t)i;
            if (node >= 0 && (hs.nodes[node].flags & rr::NF_TRI_INLINE)) {  // identity (slots hold p1/e1/e2)
                for (int k = 0; k < 12; ++k) o[k] = (k % 5 == 0) ? 1.0 : 0.0;
            } else if (node >= 0) {
                for (int k = 0; k < 12; ++k) o[k] = hs.nodes[node].inv[k];
            } else {
                for (int k = 0; k < 12; ++k) o[k] = 0.0;
            }
            o[12] = 0.0;
            o[13] = 0.0;
            o[14] = 0.0;
            o[15] = 1.0;
        }
        if (group_aabbs) {
            double* o = group_aabbs + 6 * (size_t)i;
            for (int k = 0; k < 6; ++k) o[k] = 0.0;
            if (node >= 0 && rr::is_container(hs.nodes[node].kind))
                for (int k = 0; k < 6; ++k) o[k] = hs.groups[hs.nodes[node].aux].aabb[k];
        }
    }
    return RR_OK;
}

int rr_camera_new(int64_t hsize, int64_t vsize, double fov, const double transform[16], rr_camera* out) {
    if (!out || hsize <= 0 || vsize <= 0) return fail(RR_E_ARG, "bad camera size");
    double half_view = std::tan(fov / 2.0);  // camera.rs:41-63
    double aspect = (double)hsize / (double)vsize;
    double hw, hh;
    if (aspect >= 1.0) {
        hw = half_view;
        hh = half_view / aspect;
    } else {
        hw = half_view * aspect;
        hh = half_view;
    }
    out->hsize = hsize;
    out->vsize = vsize;
    out->field_of_view = fov;
    out->half_width = hw;
    out->half_height = hh;
    out->pixel_size = (hw * 2.0) / (double)hsize;
    rr::M4 id = rr::identity();
    for (int i = 0; i < 16; ++i) out->transform[i] = transform ? transform[i] : id.m[i];
    return RR_OK;
}

int64_t rr_part_rows(int64_t height, int32_t part, int32_t nparts, int32_t block, int64_t* rows_out) {
    if (nparts < 1 || part < 0 || part >= nparts || block < 1 || height < 0) return fail(RR_E_ARG, "bad partition");
    const int64_t n = rr::part_rows_count(height, part, nparts, block);
    if (rows_out) {
        int64_t k = 0;
        for (int64_t b0 = (int64_t)part * block; b0 < height; b0 += (int64_t)nparts * block)
            for (int64_t y = b0; y < std::min<int64_t>(b0 + block, height); ++y) rows_out[k++] = y;
    }
    return n;
}

int64_t rr_stage_row_offset(int64_t height, int32_t part, int32_t nparts, int32_t block) {
    if (height < 0 || nparts < 1 || block < 1 || part < 0 || part > nparts)
        return fail(RR_E_ARG, "rr_stage_row_offset: bad arguments");
    return rr::stage_row_offset(height, part, nparts, block);
}

int rr_unshuffle_host(const double* staged, double* frame, int64_t width, int64_t height, int32_t nparts,
                      int32_t block) {
    if (!staged || !frame || width < 0 || height < 0 || nparts < 1 || block < 1)
        return fail(RR_E_ARG, "rr_unshuffle_host: bad arguments");
    const int64_t row = width * 3;
    for (int32_t p = 0; p < nparts; ++p) {  // the runs place_tile_kernel moves on rank 0 (partition.hpp)
        const double* tile = staged + rr::stage_row_offset(height, p, nparts, block) * row;
        rr::for_each_part_run(height, p, nparts, block, [&](int64_t j, int64_t y, int64_t n) {
            std::memcpy(frame + y * row, tile + j * row, (size_t)(n * row) * sizeof(double));
        });
    }
    return RR_OK;
}

int rr_create_virtual(int device, int nparts, rr_ctx** out) {
    rr::DeviceGuard device_guard;
    if (!out) return fail(RR_E_ARG, "null out");
    *out = nullptr;
    rr_group* g = nullptr;
    int rc = rr::group_create_virtual(device, nparts, &g);
    if (rc != RR_OK) return rc;
    rr_ctx* c = new rr_ctx();
    c->group = g;
    *out = c;
    return RR_OK;
}

int rr_render_device(rr_ctx* c, const rr_camera* cam, const rr_render_opts* o, void* d_canvas, void* d_avg,
                     void* hip_stream) {
    rr::DeviceGuard device_guard;  // the caller's current device is restored on return
    int rc = rr::render_validate(c, cam, o);
    if (rc != RR_OK) return rc;
    HIPCHK(hipSetDevice(c->device));
    int32_t block = o->block_rows > 0 ? o->block_rows : 8;
    const int64_t H = cam->vsize / o->aa, W = cam->hsize / o->aa;
    const int64_t rows = opts_rows(o, H);
    const int64_t local_rows = rows * o->aa;
    // a band [row_begin, row_end) is part row_begin / block of nparts = 1: the kernels' row arithmetic
    // (bi * nparts + part) * block + kb is then row_begin + the local row, with a block that divides row_begin (8
    // rows, else 2 — pixel waves need an even block — else 1)
    int32_t part = o->part;
    if (o->row_begin != 0 || o->row_end != 0) {
        if (o->row_begin % block != 0) block = o->row_begin % 2 == 0 ? 2 : 1;
        part = o->row_begin / block;
    }
    const int64_t total = local_rows * cam->hsize;
    // Everything is enqueued on the caller's stream (no cross-stream events per call: a HIP event
    // handoff between streams costs host time every frame).  The context's workspace is reused, so
    // a render on a different stream than the previous one first waits for that one.
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : c->stream;
    HIPCHK(claim_stream(c, st));
    StreamClaim claim{c, st};
    // aa == 1, or aa in {2, 4, 8} without secondary rays (wave_avg_ok): the average is written by the
    // kernels directly; the canvas only when asked for
    const bool wave_avg = d_avg && wave_avg_ok(c, o->aa, cam->hsize, local_rows, o->max_depth);
    // aa == 3 frames with reflection chains: pixel waves (7 whole pixels per wave) average in the wave too
    const bool pw = d_avg && !wave_avg && o->aa == 3 &&
                    (rr::tree_levels(c->S) || rr::chain_levels(c->S, c->host.max_children, o->max_depth)) &&
                    block % 2 == 0 && total <= c->batch && !std::getenv("RRAY_NO_PW");
    const bool direct_avg = d_avg && (o->aa == 1 || wave_avg || pw);
    double* canvas = static_cast<double*>(d_canvas);
    if (!canvas && !direct_avg) {
        HIPCHK(c->canvas.ensure(std::max<int64_t>(total, 1) * 3 * sizeof(double)));
        canvas = c->canvas.as<double>();
    }
    c->frame_timed = !(o->flags & RR_NO_FRAME_TIMING);
    if (c->frame_timed) HIPCHK(hipEventRecord(c->e0, st));
    rr::LevelArgs A{};
    A.cam = dev_camera(cam);
    A.cam_affine = A.cam.inv[12] == 0.0 && A.cam.inv[13] == 0.0 && A.cam.inv[14] == 0.0 && A.cam.inv[15] == 1.0 &&
                   A.cam.origin[3] == 1.0;
    A.hs = cam->hsize;
    A.lrows = local_rows;
    A.aa = o->aa;
    A.part = part;
    A.nparts = o->nparts;
    A.block_rows = block;
    A.rays0 = nullptr;
    A.seed = o->seed;
    A.jitter_mode = o->jitter_mode;
    if (pw) {
        A.pw = 1;
        A.pw_rows = (int32_t)rows;
        A.pw_wpb = (uint32_t)((2 * W + 6) / 7);
    }
    const int32_t f32 = (o->flags & RR_OUT_AVG_F32) ? 1 : 0;
    rc = tile_bundles(c, A, st, &A.tile_bundles);
    if (rc != RR_OK) return rc;
    c->zero_next = true;
    const AaPasses aap{d_avg, f32, W, o->aa};
    rc = run_levels(c, A, total, o->max_depth, canvas, st, direct_avg ? d_avg : nullptr, f32, wave_avg ? o->aa : 0,
                    (d_avg && !direct_avg) ? &aap : nullptr);
    c->zero_next = false;
    if (rc != RR_OK) return rc;
    c->stats_src = frame_counters(c, c->epoch);
    c->epoch ^= 1;
    if (c->frame_timed) HIPCHK(hipEventRecord(c->e1, st));
    HIPCHK(claim.release());
    c->stats_pending = true;
    // C_SAMPLES is not incremented by the wavefront kernels; it is the level-0 event count
    c->last.samples = (uint64_t)total;
    return RR_OK;
}

int rr_render_gather_device(rr_ctx* c, const rr_camera* cam, const rr_render_opts* o, void* d_frame, void* hip_stream) {
    rr::DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!c) return fail(RR_E_ARG, "null context");
    if (c->group) return rr::group_render_gather(c->group, cam, o, d_frame, hip_stream);
    if (o && (o->nparts != 1 || o->part != 0)) return fail(RR_E_ARG, "rr_render_gather_device renders the whole frame");
    if (o && (o->flags & (RR_OUT_CANVAS | RR_OUT_AVG_F32)))
        return fail(RR_E_ARG, "rr_render_gather_device writes the f64 AA-averaged image only");
    if (!d_frame) return fail(RR_E_ARG, "null frame buffer");
    return rr_render_device(c, cam, o, nullptr, d_frame, hip_stream);
}

int rr_kernel_profile(rr_ctx* c, int enable) {
    rr::DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!c) return fail(RR_E_ARG, "null context");
    if (c->group) return rr::group_kernel_profile(c->group, enable);
    HIPCHK(sync_ctx(c));
    int rc = resolve_prof(c);
    if (rc != RR_OK) return rc;
    c->profile = enable != 0;
    for (int k = 0; k < rr::K_COUNT; ++k) {
        c->kms[k] = 0.0;
        c->kcount[k] = 0;
    }
    return RR_OK;
}

int rr_kernel_times(rr_ctx* c, double* ms, uint64_t* launches, int32_t n) {
    rr::DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!c) return fail(RR_E_ARG, "null context");
    if (c->group) return rr::group_kernel_times(c->group, ms, launches, n);
    HIPCHK(sync_ctx(c));
    int rc = resolve_prof(c);
    if (rc != RR_OK) return rc;
    for (int k = 0; k < n && k < rr::K_COUNT; ++k) {
        if (ms) ms[k] = c->kms[k];
        if (launches) launches[k] = c->kcount[k];
    }
    return rr::K_COUNT;
}

int rr_last_stats(rr_ctx* c, rr_stats* s) {
    rr::DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!c || !s) return fail(RR_E_ARG, "null argument");
    if (c->group) return rr::group_last_stats(c->group, s);
    uint64_t samples = c->last.samples;
    int rc = finish_stats(c);
    if (rc != RR_OK) return rc;
    c->last.samples = samples;
    *s = c->last;
    return RR_OK;
}

int rr_render(rr_ctx* c, const rr_camera* cam, const rr_render_opts* o, double* out_canvas, double* out_avg,
              rr_stats* stats) {
    rr::DeviceGuard device_guard;  // the caller's current device is restored on return
    if (!c) return fail(RR_E_ARG, "null context");
    if (c->group) return rr::group_render(c->group, cam, o, out_canvas, out_avg, stats);
    int rc = check_opts(cam, o);
    if (rc != RR_OK) return rc;
    const int64_t H = cam->vsize / o->aa, W = cam->hsize / o->aa;
    const int64_t rows = opts_rows(o, H);
    const int64_t total = rows * o->aa * cam->hsize;
    HIPCHK(hipSetDevice(c->device));
    const bool want_avg = (o->flags & RR_OUT_AVG) && out_avg;
    HIPCHK(c->qout.ensure(std::max<int64_t>(W * rows, 1) * 3 * sizeof(double)));
    const bool want_canvas = (o->flags & RR_OUT_CANVAS) && out_canvas;
    if (want_canvas) HIPCHK(c->canvas.ensure(std::max<int64_t>(total, 1) * 3 * sizeof(double)));
    rc = rr_render_device(c, cam, o, want_canvas ? c->canvas.p : nullptr, want_avg ? c->qout.p : nullptr, nullptr);
    if (rc != RR_OK) return rc;
    if (want_canvas)
        HIPCHK(hipMemcpyAsync(out_canvas, c->canvas.p, total * 3 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    if (want_avg)
        HIPCHK(hipMemcpyAsync(out_avg, c->qout.p, W * rows * 3 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    rr_stats local;
    rc = rr_last_stats(c, stats ? stats : &local);
    if (rc != RR_OK) return rc;
    const uint64_t nan = (stats ? stats : &local)->nan_rays;
    return nan ? nan_fail(nan) : RR_OK;
}

int rr_color_at(rr_ctx* c, int64_t n, const double* origins, const double* directions, int32_t remaining,
                uint64_t seed, int32_t jitter_mode, double* out_rgb) {
    rr::DeviceGuard device_guard;  // the caller's current device is restored on return
    if (c && c->group) return rr_color_at(rr::group_local(c->group, 0), n, origins, directions, remaining, seed, jitter_mode, out_rgb);
    if (!c || (n > 0 && (!origins || !directions || !out_rgb))) return fail(RR_E_ARG, "null argument");
    if (!c->has_scene) return fail(RR_E_ARG, "no scene uploaded");
    if (remaining < 0 || remaining > RR_MAX_DEPTH) return fail(RR_E_LIMIT, "remaining out of range");
    if (n == 0) return RR_OK;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    HIPCHK(claim_stream(c, st));
    StreamClaim claim{c, st};
    std::vector<double> rays((size_t)n * 6);
    for (int64_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) {
            rays[6 * i + k] = origins[3 * i + k];
            rays[6 * i + 3 + k] = directions[3 * i + k];
        }
    HIPCHK(upload(c->rays0, rays, st));
    HIPCHK(c->qout.ensure(n * 3 * sizeof(double)));
    const int saved_epoch = c->epoch;
    c->epoch = 2;  // the query buffer (frame buffers keep their state)
    HIPCHK(hipMemsetAsync(frame_counters(c, 2), 0, kCounterBytes, st));
    rr::LevelArgs A{};
    A.hs = 1;
    A.aa = 1;
    A.part = 0;
    A.nparts = 1;
    A.block_rows = 1;
    A.rays0 = c->rays0.as<double>();
    A.seed = seed;
    A.jitter_mode = jitter_mode;
    int rc = run_levels(c, A, n, remaining, c->qout.as<double>(), st);
    c->epoch = saved_epoch;
    if (rc != RR_OK) return rc;
    HIPCHK(hipMemcpyAsync(out_rgb, c->qout.p, n * 3 * sizeof(double), hipMemcpyDeviceToHost, st));
    // the counters on the same (non-blocking) stream, then wait: out_rgb and the counters are both
    // complete on return, whatever kind of host memory the caller passed
    HIPCHK(hipMemcpyAsync(c->h_counters, frame_counters(c, 2), kCounterBytes, hipMemcpyDeviceToHost, st));
    HIPCHK(claim.release());
    HIPCHK(hipStreamSynchronize(st));
    rr_stats q;
    collect_stats(c, &q);
    return q.nan_rays ? nan_fail(q.nan_rays) : RR_OK;
}

int rr_is_shadowed(rr_ctx* c, int64_t n, const double* points, const double* light_positions, int32_t* out) {
    rr::DeviceGuard device_guard;  // the caller's current device is restored on return
    if (c && c->group) return rr_is_shadowed(rr::group_local(c->group, 0), n, points, light_positions, out);
    if (!c || (n > 0 && (!points || !light_positions || !out))) return fail(RR_E_ARG, "null argument");
    if (!c->has_scene) return fail(RR_E_ARG, "no scene uploaded");
    if (n == 0) return RR_OK;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    HIPCHK(claim_stream(c, st));
    StreamClaim claim{c, st};
    std::vector<double> buf((size_t)n * 6);
    std::memcpy(buf.data(), points, n * 3 * sizeof(double));
    std::memcpy(buf.data() + 3 * n, light_positions, n * 3 * sizeof(double));
    HIPCHK(upload(c->rays0, buf, st));
    HIPCHK(c->qout.ensure(n * sizeof(int32_t)));
    HIPCHK(rr::launch_shadow_query(c->S, c->rays0.as<double>(), c->rays0.as<double>() + 3 * n, n,
                                   c->qout.as<int32_t>(), frame_counters(c, 2), st));
    HIPCHK(hipMemcpyAsync(out, c->qout.p, n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(claim.release());
    HIPCHK(hipStreamSynchronize(st));
    return RR_OK;
}

}  // extern "C"

// ---- ABI 10: cost-balanced bands (multi.cpp) ----
extern "C" int rr_balance_bands(const double* row_cost, int64_t height, int32_t nparts, double root_extra, int32_t align,
                                int64_t* bounds) {
    if (!row_cost || !bounds || height < 1 || nparts < 1 || align < 1)
        return fail(RR_E_ARG, "rr_balance_bands: need row costs, height >= 1, nparts >= 1, align >= 1");
    rr::balance_bands(row_cost, height, nparts, root_extra, align, bounds);
    return RR_OK;
}

extern "C" int rr_group_bands(rr_ctx* c, int64_t* bounds, int32_t n) {
    if (!c || !bounds) return fail(RR_E_ARG, "null argument");
    if (!c->group) return fail(RR_E_ARG, "rr_group_bands: not a multi-device context");
    return rr::group_bands(c->group, bounds, n);
}

extern "C" int rr_group_set_bands(rr_ctx* c, const int64_t* bounds, int32_t n) {
    if (!c || !bounds) return fail(RR_E_ARG, "null argument");
    if (!c->group) return fail(RR_E_ARG, "rr_group_set_bands: not a multi-device context");
    return rr::group_set_bands(c->group, bounds, n);
}
