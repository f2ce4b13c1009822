// render.hip — wavefront kernels of the MI355X (gfx950) render path.
//
// Camera::render (camera.rs:107-121) -> Scene::color_at (scene.rs:128-136), evaluated level by
// level over HBM-resident queues (wavefront.hpp):
//   trace_kernel   closest hit per pending color_at ray           scene.rs:97-106,130
//   n1n2_kernel    container walk for transparent hits             intersection.rs:61-92
//   shade_kernel   prepare_computations, pattern, children rays,   intersection.rs:50-60, scene.rs:159-336,
//                  is_shadowed walks + lighting sum, leaf results  light.rs:47-140
//   combine_kernel bottom-up shade_hit sums of events with children scene.rs:167-177
//   aa_kernel      box average before `as u8`                      canvas.rs:76-96
// Every kernel is one work-item per queue entry; the node walks inside are wave-uniform (scalar
// broadcast loads of the flattened scene, culled per wave against the rays' bundle).
#include <algorithm>
#include <cstdlib>

#include "device_core.inc"
#include "kernels.hpp"
#include "wavefront.hpp"

namespace rr {

// floor(n / d) for d >= 1 given magic = floor(2^32 / d) (d >= 2; unused for d == 1): the high
// product is the quotient or one less for every 32-bit n, so one correction makes it exact.
__device__ __forceinline__ uint32_t magic_div(uint32_t n, uint32_t d, uint32_t magic) {
    if (d == 1u) return n;
    uint32_t q = __umulhi(n, magic);
    if (n - q * d >= d) ++q;
    return q;
}

// A level-0 event's canvas position: ls = part-local row-major sample index (the output index),
// (px, py) = supersampled canvas pixel.  Camera events run in tile order (tile_to_local); when every
// tile is a full 8x8 and the batch is tile-aligned (A.tile_fast, host-checked) a wave is exactly one
// tile, so the tile arithmetic is wave-uniform (scalar) and a lane only adds its (lane & 7, lane >> 3)
// offset — the same bijection as tile_to_local_u32 without its three per-lane divisions.
struct Px0 {
    uint32_t ls, px, py;
};
// OWN: i is this thread's own index (blockIdx.x * 256 + threadIdx.x), so the wave's tile is uniform;
// otherwise (events from a list) the same mapping is computed per lane from i.
template <bool OWN>
__device__ __forceinline__ Px0 level0_px(const LevelArgs& A, int64_t i) {
    Px0 r;
    if (A.rays0) {
        r.ls = (uint32_t)(A.base + i);
        r.px = r.py = 0u;
        return r;
    }
    const uint32_t hs = (uint32_t)A.hs;
    uint32_t lrow;
    if (A.tile_fast) {
        const uint32_t t = (uint32_t)(A.base + i);
        const uint32_t T = OWN ? (uint32_t)(A.base >> 6) + blockIdx.x * 4u + (uint32_t)uniform((int)(threadIdx.x >> 6))
                               : t >> 6;
        const uint32_t band = T / A.tiles_per_row;
        const uint32_t tc = T - band * A.tiles_per_row;
        const uint32_t lane = OWN ? threadIdx.x & 63u : t & 63u;
        lrow = band * 8u + (lane >> 3);
        r.px = tc * 8u + (lane & 7u);
        r.ls = lrow * hs + r.px;
    } else {
        const uint32_t t = (uint32_t)(A.base + i);
        r.ls = A.lrows <= 0 ? t : tile_to_local_u32(t, hs, (uint32_t)A.lrows);
        lrow = r.ls / hs;
        r.px = r.ls - lrow * hs;
    }
    // interleaved row blocks of the part -> canvas row (32-bit: rr_render_device rejects parts of
    // 2^31 samples or more)
    const uint32_t aa = (uint32_t)A.aa, br = (uint32_t)A.block_rows;
    const uint32_t k = magic_div(lrow, aa, A.aa_magic), sub = lrow - k * aa;
    const uint32_t bi = magic_div(k, br, A.br_magic), kb = k - bi * br;
    const uint32_t y = (bi * (uint32_t)A.nparts + (uint32_t)A.part) * br + kb;
    r.py = y * aa + sub;
    return r;
}
template <bool OWN>
__device__ __forceinline__ Px0 level0_px_if(const LevelArgs& A, int64_t i) {
    if (A.level > 0) return {0u, 0u, 0u};
    return level0_px<OWN>(A, i);
}

// Camera::ray_for_pixel (camera.rs:75-93).  The camera inverse's 4th row is (0, 0, 0, 1) for every
// view_transform (checked on the host, A.cam_affine), so pixel.w == 1 == origin.w and the w terms of
// the subtraction and of the magnitude are exactly +0 (adding +0 to a sum of squares is exact).
__device__ __forceinline__ Ray camera_ray(const DevCamera& C, bool affine, uint32_t px, uint32_t py) {
    double xoffset = ((double)px + 0.5) * C.pixel_size;
    double yoffset = ((double)py + 0.5) * C.pixel_size;
    double wx = C.half_width - xoffset;
    double wy = C.half_height - yoffset;
    const double* M = C.inv;
    const double* ow = C.origin;  // M * point(0, 0, 0): pixel-independent, computed on the host
    if (affine) {
        double pw[3];
        for (int r = 0; r < 3; ++r) pw[r] = M[4 * r] * wx + M[4 * r + 1] * wy + M[4 * r + 2] * -1.0 + M[4 * r + 3] * 1.0;
        double dx = pw[0] - ow[0], dy = pw[1] - ow[1], dz = pw[2] - ow[2];
        double mag = sqrt(dx * dx + dy * dy + dz * dz);
        return {mk(ow[0], ow[1], ow[2]), mk(dx / mag, dy / mag, dz / mag)};
    }
    double pw[4];
    for (int r = 0; r < 4; ++r) pw[r] = M[4 * r] * wx + M[4 * r + 1] * wy + M[4 * r + 2] * -1.0 + M[4 * r + 3] * 1.0;
    double dx = pw[0] - ow[0], dy = pw[1] - ow[1], dz = pw[2] - ow[2], dw = pw[3] - ow[3];
    double mag = sqrt(dx * dx + dy * dy + dz * dz + dw * dw);
    return {mk(ow[0], ow[1], ow[2]), mk(dx / mag, dy / mag, dz / mag)};
}

// the ray of event i at this level; q = level0_px(A, i) (used at level 0 only); camera rays also
// return their global sample id (the jitter key, as event_key) in s0
__device__ __forceinline__ Ray event_ray(const LevelArgs& A, int64_t i, const Px0& q, uint64_t& s0) {
    if (A.level > 0) {
        const Event& e = A.ev[i];
        return {mk(e.o[0], e.o[1], e.o[2]), mk(e.d[0], e.d[1], e.d[2])};
    }
    if (A.rays0) {
        const double* p = A.rays0 + 6 * (A.base + i);
        return {mk(p[0], p[1], p[2]), mk(p[3], p[4], p[5])};
    }
    s0 = (uint64_t)q.py * (uint64_t)A.hs + q.px;
    return camera_ray(A.cam, A.cam_affine, q.px, q.py);
}
template <bool OWN>
__device__ __forceinline__ Ray event_ray(const LevelArgs& A, int64_t i) {
    uint64_t s0 = 0;
    return event_ray(A, i, level0_px_if<OWN>(A, i), s0);
}
// jitter identity of event i: (global sample id, recursion path); q as for event_ray
// (s0: event_ray's sample id of a level-0 camera ray)
__device__ __forceinline__ void event_key(const LevelArgs& A, int64_t i, const Px0& q, uint64_t s0, uint64_t& sample,
                                          uint32_t& path) {
    path = A.level > 0 ? A.ev[i].path : 1u;
    if (A.level == 0) {
        sample = A.rays0 ? (uint64_t)q.ls : s0;
        return;
    }
    const uint32_t ls = A.ev[i].sample;
    if (A.rays0) {
        sample = (uint64_t)ls;
        return;
    }
    // level >= 1: the event carries its camera sample's local index (row-major)
    const uint32_t hs = (uint32_t)A.hs;
    const uint32_t lrow = ls / hs, px = ls - lrow * hs;
    const uint32_t aa = (uint32_t)A.aa, br = (uint32_t)A.block_rows;
    const uint32_t k = magic_div(lrow, aa, A.aa_magic), sub = lrow - k * aa;
    const uint32_t bi = magic_div(k, br, A.br_magic), kb = k - bi * br;
    const uint32_t y = (bi * (uint32_t)A.nparts + (uint32_t)A.part) * br + kb;
    sample = (uint64_t)(y * aa + sub) * (uint64_t)A.hs + px;
}

// Block-aggregated queue appends: the 4 waves' ballots are summed in LDS and one lane per queue
// does a single device-scope atomicAdd for the whole block (device-scope atomics are performed
// memory-side and serialise per address, so one per wave per queue was the kernels' bottleneck).
// Every thread of the (256-thread) block must call it.  Returns this lane's slot where want[q].
template <int NQ>
__device__ __forceinline__ void block_append(unsigned int* const (&ctr)[NQ], const bool (&want)[NQ],
                                             int32_t (&slot)[NQ]) {
    __shared__ unsigned int s_cnt[NQ][4];
    __shared__ unsigned int s_base[NQ][4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t m[NQ];
    for (int q = 0; q < NQ; ++q) {
        m[q] = __ballot(want[q]);
        if (lane == 0) s_cnt[q][w] = (unsigned int)__popcll(m[q]);
    }
    __syncthreads();
    if (threadIdx.x < NQ) {
        const int q = threadIdx.x;
        unsigned int total = s_cnt[q][0] + s_cnt[q][1] + s_cnt[q][2] + s_cnt[q][3];
        unsigned int run = total ? atomicAdd(ctr[q], total) : 0u;
        for (int k = 0; k < 4; ++k) {
            s_base[q][k] = run;
            run += s_cnt[q][k];
        }
    }
    __syncthreads();
    const uint64_t below_mask = lane == 0 ? 0ull : ((~0ull) >> (64 - lane));
    for (int q = 0; q < NQ; ++q) slot[q] = (int32_t)(s_base[q][w] + (unsigned int)__popcll(m[q] & below_mask));
}

// The live event count of a level.  Levels >= 1 are launched with their worst-case grid (the
// previous level's capacity x max children, known on the host) and read the real count the previous
// level's appends produced from HBM, so the host never waits for a level to finish (rray.h:
// rr_render_device is asynchronous).  Blocks past the count exit at once (block-uniform).
__device__ __forceinline__ int64_t live_count(const LevelArgs& A) {
    return A.n_dev ? (int64_t)*A.n_dev : A.n;
}

enum WalkKind { W_NONE = -1, W_TRACE = 0, W_SHADOW = 1, W_N1N2 = 2 };
// Counter flush, aggregated per workgroup: the 4 waves' totals are summed in LDS and one thread per
// counter does a single device-scope atomic (slot = blockIdx % RR_CNT_SLOTS), 4x fewer memory-side
// atomics than per-wave flushes (they were ~14 % of a C2 frame's HBM writes).  `extra` adds the fused
// kernels' closest-hit walk flops / visits.  Every thread of the (256-thread) block must call it.
constexpr int RR_FLUSH_N = 11;
__device__ void flush(const Counters& cnt, unsigned long long* counters, int walk = W_NONE,
                      uint64_t trace_flops = 0, uint64_t trace_visits = 0) {
    __shared__ unsigned long long s_acc[4][RR_FLUSH_N];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) {  // every field is wave-uniform
        const uint64_t v[RR_FLUSH_N] = {cnt.rays, cnt.shadow, cnt.shade, cnt.n1n2, cnt.gtests, cnt.ghits, cnt.tests,
                                        walk >= 0 ? (uint64_t)cnt.flops : 0ull, walk >= 0 ? (uint64_t)cnt.visits : 0ull,
                                        trace_flops, trace_visits};
        for (int k = 0; k < RR_FLUSH_N; ++k) s_acc[w][k] = v[k];
    }
    __syncthreads();
    if (threadIdx.x < RR_FLUSH_N) {
        const int k = threadIdx.x;
        const unsigned long long t = s_acc[0][k] + s_acc[1][k] + s_acc[2][k] + s_acc[3][k];
        const int slot_of[RR_FLUSH_N] = {C_RAYS, C_SHADOW, C_SHADE, C_N1N2, C_GROUP_TESTS, C_GROUP_HITS, C_PRIM_TESTS,
                                         C_FLOPS_TRACE + (walk >= 0 ? walk : 0), C_VISITS_TRACE + (walk >= 0 ? walk : 0),
                                         C_FLOPS_TRACE, C_VISITS_TRACE};
        if (t) atomicAdd(counters + (blockIdx.x & (RR_CNT_SLOTS - 1)) * RR_CNT_STRIDE + slot_of[k], t);
    }
}

__device__ __forceinline__ bool needs_n1n2(const DevMaterial& m, int rem) {
    // n1/n2 feed refracted_color (rem > 0, transparency != 0) and schlick (reflective > 0 &&
    // transparency > 0); both need transparency != 0.
    return m.transparency != 0.0 && (rem > 0 || m.reflective > 0.0);
}

// Counters are double-buffered per frame: the first level's kernels clear the buffer the next
// frame will count into, so no memset sits between frames.
__device__ __forceinline__ void zero_next_counters(const LevelArgs& A) {
    if (!A.counters_zero) return;
    const int total = RR_CNT_SLOTS * RR_CNT_STRIDE;
    for (int j = (int)(blockIdx.x * blockDim.x + threadIdx.x); j < total; j += (int)(gridDim.x * blockDim.x))
        A.counters_zero[j] = 0ull;
}

template <int G, bool LC, bool RM>
__global__ void __launch_bounds__(256) trace_kernel(DevScene S, LevelArgs A) {
    const int64_t n_live = live_count(A);
    if ((int64_t)blockIdx.x * blockDim.x >= n_live) return;
    zero_next_counters(A);
    if (LC) stage_culls(S);
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = i < n_live;
    Counters cnt = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#ifdef RR_STAMPS
    cnt.st = nullptr;
    if (A.stamps && A.level == 0) {
        const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
        cnt.st = A.stamps + (0 * (int64_t)(1 << 16) + w) * 16;
        if (w >= (1 << 16)) cnt.st = nullptr;
    }
    RR_STAMP(cnt, 0);
#endif
    Ray r = valid ? event_ray<true>(A, i) : Ray{mk(0, 0, 0), mk(0, 0, 1)};
    Hit h;
    RR_STAMP(cnt, 1);
    trace_closest<G, LC, RM>(S, r, valid, h, cnt);
    cnt.rays += popc_ballot(valid);
    if (valid) {
        HitRec hr;
        hr.t = h.t;
        hr.u = h.u;
        hr.v = h.v;
        hr.node = h.found ? h.node : -1;
        hr.k = h.k;
        A.hit[i] = hr;
    }
    bool want = false;
    if (S.has_transparent && valid && h.found) {
        DevMaterial m = S.mats[S.nodes[h.node].material];
        want = needs_n1n2(m, A.rem);
    }
    if (S.has_transparent) {  // uniform: the whole block appends
        unsigned int* const ctr[1] = {A.lcount + LC_N1N2};
        const bool wq[1] = {want};
        int32_t slot[1];
        block_append<1>(ctr, wq, slot);
        if (want) A.n1n2_list[slot[0]] = (int32_t)i;
    }
    RR_STAMP(cnt, 5);
    flush(cnt, A.counters, W_TRACE);
#ifdef RR_STAMPS
    if (cnt.st && (threadIdx.x & 63) == 0) {
        cnt.st[6] = cnt.visits;
        cnt.st[7] = __builtin_amdgcn_s_memtime();
    }
#endif
}

template <int G, bool LC, bool RM>
__global__ void __launch_bounds__(256) n1n2_kernel(DevScene S, LevelArgs A) {
    const int64_t cnt_n = (int64_t)A.lcount[LC_N1N2];
    if ((int64_t)blockIdx.x * blockDim.x >= cnt_n) return;
    if (LC) stage_culls(S);
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = j < cnt_n;
    Counters cnt = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    int64_t i = valid ? A.n1n2_list[j] : 0;
    Ray r = valid ? event_ray<false>(A, i) : Ray{mk(0, 0, 0), mk(0, 0, 1)};
    Hit h;
    h.found = valid;
    h.t = 0.0;
    h.node = -1;
    h.k = 0;
    h.rank = 0;
    if (valid) {
        HitRec hr = A.hit[i];
        h.t = hr.t;
        h.u = hr.u;
        h.v = hr.v;
        h.node = hr.node;
        h.k = hr.k;
        h.rank = S.nodes[hr.node].rank;
    }
    double n1 = 1.0, n2 = 1.0;
    n1n2_walk<G, LC, RM>(S, r, h, valid, n1, n2, cnt);
    if (valid) {
        A.n12[2 * i] = n1;
        A.n12[2 * i + 1] = n2;
    }
    flush(cnt, A.counters, W_N1N2);
}

// shade_hit's final sum (scene.rs:172-177) for given child results a (reflected) and b (refracted)
__device__ __forceinline__ V3 shade_sum(V3 s, V3 a, V3 b, double refl, double transp, double R) {
    if (refl > 0.0 && transp > 0.0) return vadd(vadd(s, vmul(a, R)), vmul(b, 1.0 - R));
    return vadd(vadd(s, a), b);
}

// A finished color_at value v of event i: level 0 writes the canvas; deeper levels become the
// parent's reflected_color (v * reflective, scene.rs:281-290) or refracted_color (v * transparency,
// scene.rs:310-336) slot.  Each slot has exactly one writer.
// With aa == 1 the box average of canvas.rs:85-96 is r = 0.0; r += p; r /= 1.0, written here
// directly (same operations) instead of through the canvas and aa_kernel.
__device__ __forceinline__ void deliver(int32_t level, int64_t i, int32_t parent, int32_t slot, V3 v, double* out,
                                        void* avg, int32_t avg_f32, CombRec* parent_comb, CombExt* parent_ext,
                                        int64_t out_index) {
    if (level == 0) {
        if (out) {
            double* o = out + 3 * out_index;
            o[0] = v.x;
            o[1] = v.y;
            o[2] = v.z;
        }
        if (avg) {
            const double a0 = (0.0 + v.x) / 1.0, a1 = (0.0 + v.y) / 1.0, a2 = (0.0 + v.z) / 1.0;
            if (avg_f32) {
                float* o = static_cast<float*>(avg) + 3 * out_index;
                o[0] = (float)a0;
                o[1] = (float)a1;
                o[2] = (float)a2;
            } else {
                double* o = static_cast<double*>(avg) + 3 * out_index;
                o[0] = a0;
                o[1] = a1;
                o[2] = a2;
            }
        }
        return;
    }
    if (slot) {  // a refracted child: the scene has transparency, so the parent has its CombExt
        CombExt& e = parent_ext[parent];
        const double t = e.transp;
        e.refr_res[0] = v.x * t;
        e.refr_res[1] = v.y * t;
        e.refr_res[2] = v.z * t;
    } else {
        CombRec& p = parent_comb[parent];
        const double t = p.refl;
        p.refl_res[0] = v.x * t;
        p.refl_res[1] = v.y * t;
        p.refl_res[2] = v.z * t;
    }
}

// intensity_at (light.rs:67-96): 1 - in_shadow from is_shadowed toward the light (point) or the
// fraction of its level^2 jittered cell samples that are shadowed (area, light.rs:47-65)
template <int G, bool LC, bool RM>
__device__ __forceinline__ double shadow_amount(const DevScene& S, const LevelArgs& A, const DevLight& Lt, int li,
                                                V3 over, bool active, uint64_t sample, uint32_t path, Counters& cnt) {
    if (Lt.kind == RR_LIGHT_POINT)
        return shadowed<G, LC, RM>(S, over, mk(Lt.position[0], Lt.position[1], Lt.position[2]), active, cnt) ? 1.0 : 0.0;
    const int amount = Lt.level * Lt.level;
    int total = 0;
    for (int s = 0; s < amount; ++s) {
        const int row = s / Lt.level, col = s % Lt.level;
        double ur = 0.5, vr = 0.5;
        if (A.jitter_mode == 0) {
            ur = jitter(A.seed, sample, path, (uint32_t)li, (uint32_t)s, 0);
            vr = jitter(A.seed, sample, path, (uint32_t)li, (uint32_t)s, 1);
        }
        const double uf = ((double)col + ur) / (double)Lt.level;
        const double vf = ((double)row + vr) / (double)Lt.level;
        const V3 target = vadd(vadd(mk(Lt.corner[0], Lt.corner[1], Lt.corner[2]), vmul(mk(Lt.u[0], Lt.u[1], Lt.u[2]), uf)),
                               vmul(mk(Lt.v[0], Lt.v[1], Lt.v[2]), vf));
        total += shadowed<G, LC, RM>(S, over, target, active, cnt) ? 1 : 0;
    }
    return (double)total / (double)amount;
}

// The prelit terms follow the cull records in the walking kernels' dynamic LDS:
// [light][6 doubles][256 threads] (SoA: lanes of a wave read consecutive doubles).
constexpr int RR_PRELIT_LIGHTS = 2;
__device__ __forceinline__ double* prelit_lds(const DevScene& S, bool lc) {
    char* base = reinterpret_cast<char*>(rr_lds_culls);
    const size_t off = lc ? (size_t)S.n_nodes * sizeof(DevCull) + (size_t)S.n_chunks * sizeof(DevChunk) : 0;
    return reinterpret_cast<double*>(base + off);
}

// Per-thread shading state parked in LDS (SoA, 9 doubles x 256 threads = 18 KB) while the shadow
// walks run, so the walks do not compete with it for VGPRs: eyev, normalv, pattern colour.
struct ShadeStash {
    double v[9][256];
};
__device__ __forceinline__ void stash_put(ShadeStash& s, V3 eyev, V3 normalv, V3 pcol) {
    const int t = threadIdx.x;
    s.v[0][t] = eyev.x;
    s.v[1][t] = eyev.y;
    s.v[2][t] = eyev.z;
    s.v[3][t] = normalv.x;
    s.v[4][t] = normalv.y;
    s.v[5][t] = normalv.z;
    s.v[6][t] = pcol.x;
    s.v[7][t] = pcol.y;
    s.v[8][t] = pcol.z;
}

// one light of shade_hit's sum: surface += lighting(material, light, colour, over, eyev, normalv,
// intensity_at(light, over)) — the shadow walk first, then the lighting terms from the stash
template <int G, bool LC, bool RM>
__device__ __forceinline__ void light_step(const DevScene& S, const LevelArgs& A, int li, bool has_hit, int mat,
                                           V3 over, uint64_t sample, uint32_t path, const ShadeStash& st,
                                           V3& surface, Counters& cnt) {
    const DevLight Lt = ldc(S.lights, li);
    const double in_shadow = shadow_amount<G, LC, RM>(S, A, Lt, li, over, has_hit, sample, path, cnt);
    if (has_hit) {
        const int t = threadIdx.x;
        const V3 eyev = mk(st.v[0][t], st.v[1][t], st.v[2][t]);
        const V3 normalv = mk(st.v[3][t], st.v[4][t], st.v[5][t]);
        const V3 pcol = mk(st.v[6][t], st.v[7][t], st.v[8][t]);
        surface = vadd(surface, lighting(S.mats[mat], Lt, pcol, over, eyev, normalv, in_shadow));
    }
}

// Fused shade_hit for every event of the level (scene.rs:159-177):
//   prepare_computations + pattern (intersection.rs:50-60, material.rs:77-80), the children rays
//   (reflected_color scene.rs:281-290, refracted_color scene.rs:310-336) appended to level d+1,
//   then surface = 0 + lighting(L0, intensity_at(L0)) + ... with every is_shadowed walk
//   (scene.rs:181-214, 234-245; area lights sample level^2 jittered points, light.rs:47-65).
// The 64 lanes of a wave walk their shadow rays for the same light sample together, so the walk's
// ray bundle stays tight.  Events without children are finished here (deliver); events with
// children store their pending sum and are finished by combine_kernel after their children.
// FUSED (scenes without transparency, where no n1/n2 walk sits between trace and shade): the
// kernel first runs the closest-hit walk itself, so the hit and the ray stay in registers.
// PRE (scenes with <= RR_PRELIT_LIGHTS lights): every light's ambient and diffuse+specular terms
// (the `pow`-heavy part of lighting) are computed right after prepare_computations and parked in
// LDS, so the shadow walks run with only the walk state live; otherwise eyev / normalv / colour
// are parked and lighting runs after each walk.
// The prelit variant is held to 4 waves/SIMD (<= 128 VGPRs; ~10 VGPRs spill, measured faster than
// 3 spill-free waves: C2 0.258 vs 0.288 ms/frame).  RR_SHADE_W3 builds the spill-free variant.
// The general variant (G = 2) is not held to 4 waves: squeezed into 128 VGPRs it spills ~300
// registers, and those builds (ROCm 7.2 clang) returned wrong, run-to-run different images for
// cube / cylinder / CSG scenes with secondary rays, while every spill-free build is bit-exact.
#ifndef RR_PRE_WAVES
#define RR_PRE_WAVES 4
#endif
#ifndef RR_SHADE_W3
#define RR_SHADE_ATTR(PRE, G) __attribute__((amdgpu_waves_per_eu(((PRE) && (G) < 2) ? RR_PRE_WAVES : 2)))
#else
#define RR_SHADE_ATTR(PRE, G)
#endif
// CP: the scene has Gradient / Blend / Perturbed / Noise / Texture patterns, evaluated by the
// out-of-line pattern_tree.  Without CP the kernel carries no call at all: the call graph's register
// demand (atan2 / acos / Perlin in the callee) otherwise costs the common scenes their occupancy.
template <int G, bool LC, bool FUSED, bool PRE, bool CP, bool RM>
__global__ void __launch_bounds__(256) RR_SHADE_ATTR(PRE, G) shade_kernel(DevScene S, LevelArgs A) {
#ifdef RR_STAMPS
    // kernel entry (before the counter clear and the cull staging) and the wave's hardware slot
    if (A.stamps && A.level == 0 && (threadIdx.x & 63) == 0) {
        const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
        if (w < (1 << 16)) {
            unsigned long long* e = A.stamps + ((int64_t)(1 << 16) + w) * 16;
            e[12] = __builtin_amdgcn_s_memtime();
            e[13] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
            e[14] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
        }
    }
#endif
    const int64_t n_live = live_count(A);
    if ((int64_t)blockIdx.x * blockDim.x >= n_live) return;
    zero_next_counters(A);
    if (LC) stage_culls(S);
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = i < n_live;
    Counters cnt = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t trace_flops = 0;
    uint32_t trace_visits = 0;
#ifdef RR_STAMPS
    cnt.st = nullptr;
    if (A.stamps && A.level == 0) {
        const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
        cnt.st = w < (1 << 16) ? A.stamps + ((int64_t)(1 << 16) + w) * 16 : nullptr;
    }
    // FUSED: the (unused) trace region of the stamp buffer takes the shadow walk and extra marks
    unsigned long long* const st1 = cnt.st;
    unsigned long long* const st0 = (FUSED && cnt.st) ? cnt.st - (int64_t)(1 << 16) * 16 : nullptr;
    RR_STAMP(cnt, 0);
#else
    unsigned long long* const st0 = nullptr;
#endif
    const Px0 q0 = level0_px_if<true>(A, i);
    const uint32_t ls0 = q0.ls;
    HitRec hr;
    hr.node = -1;
    Ray r0 = {mk(0, 0, 0), mk(0, 0, 1)};  // FUSED: the event's ray, traced here
    uint64_t s0 = 0;  // level-0 sample id from event_ray
    if (FUSED) {
        if (valid) r0 = event_ray(A, i, q0, s0);
        Hit th;
        trace_closest<G, LC, RM>(S, r0, valid, th, cnt);
        cnt.rays += popc_ballot(valid);
        hr.t = th.t;
        hr.u = th.u;
        hr.v = th.v;
        hr.node = th.found ? th.node : -1;
        hr.k = th.k;
        trace_flops = cnt.flops;
        trace_visits = cnt.visits;
        cnt.flops = cnt.visits = 0;
    } else if (valid) {
        hr = A.hit[i];
    }
    const bool has_hit = valid && hr.node >= 0;
    int32_t parent = -1, slot = 0;
    if (valid && A.level > 0) {
        parent = A.ev[i].parent;
        slot = A.ev[i].slot;
    }
    cnt.shade += popc_ballot(has_hit);
    V3 over = mk(0, 0, 0), eyev = mk(0, 0, 1), normalv = mk(0, 0, 1), pcol = mk(0, 0, 0);
    int32_t mat = 0;
    double refl = 0.0, transp = 0.0, R = 0.0;
    bool do_refl = false, do_refr = false;
    Ray rr = {mk(0, 0, 0), mk(0, 0, 1)}, refr = rr;
    uint64_t sample = 0;
    uint32_t path = 1u;
    if (has_hit) {
        const Ray r = FUSED ? r0 : event_ray(A, i, q0, s0);
        Hit h;
        h.found = true;
        h.t = hr.t;
        h.u = hr.u;
        h.v = hr.v;
        h.node = hr.node;
        h.k = hr.k;
        Comps c;
        RR_STAMPX(st0, 5);
        prepare(S, r, h, c);  // intersection.rs:50-60
        RR_STAMPX(st0, 0);
        mat = S.nodes[hr.node].material;
        const DevMaterial m = S.mats[mat];
        if (S.has_transparent && needs_n1n2(m, A.rem)) {
            c.n1 = A.n12[2 * i];
            c.n2 = A.n12[2 * i + 1];
        }
        over = c.over;
        eyev = c.eyev;
        normalv = c.normalv;
        do_refl = A.rem > 0 && m.reflective != 0.0;
        if (do_refl) {
            rr.o = c.over;
            rr.d = c.reflectv;
        }
        if (A.rem > 0 && m.transparency != 0.0) {
            double n_ratio = c.n1 / c.n2;
            double cos_i = dot3(c.eyev, c.normalv);
            double sin2_t = (n_ratio * n_ratio) * (1.0 - cos_i * cos_i);
            if (!(sin2_t > 1.0)) {
                double cos_t = sqrt(1.0 - sin2_t);
                refr.o = c.under;
                refr.d = vsub(vmul(c.normalv, n_ratio * cos_i - cos_t), vmul(c.eyev, n_ratio));
                do_refr = true;
            }
        }
        refl = m.reflective;
        transp = m.transparency;
        R = (m.reflective > 0.0 && m.transparency > 0.0) ? schlick(c) : 0.0;
        event_key(A, i, q0, s0, sample, path);
    }
    RR_STAMP(cnt, 1);
    // children of this level -> next level queue; parents -> this level's pending list
    const bool pending = do_refl || do_refr;
    if (A.next) {  // null when no material is reflective or transparent (or at the last level)
        unsigned int* const ctr[3] = {A.lcount + LC_CHILDREN, A.lcount + LC_CHILDREN, A.lcount + LC_PENDING};
        const bool wq[3] = {do_refl, do_refr, pending};
        int32_t slots[3];
        block_append<3>(ctr, wq, slots);
        const uint32_t ls = A.level > 0 ? A.ev[valid ? i : 0].sample : ls0;
        if (do_refl) {
            Event e;
            e.o[0] = rr.o.x;
            e.o[1] = rr.o.y;
            e.o[2] = rr.o.z;
            e.d[0] = rr.d.x;
            e.d[1] = rr.d.y;
            e.d[2] = rr.d.z;
            e.sample = ls;
            e.path = path * 2u;
            e.parent = (int32_t)i;
            e.slot = 0;
            A.next[slots[0]] = e;
        }
        if (do_refr) {
            Event e;
            e.o[0] = refr.o.x;
            e.o[1] = refr.o.y;
            e.o[2] = refr.o.z;
            e.d[0] = refr.d.x;
            e.d[1] = refr.d.y;
            e.d[2] = refr.d.z;
            e.sample = ls;
            e.path = path * 2u + 1u;
            e.parent = (int32_t)i;
            e.slot = 1;
            A.next[slots[1]] = e;
        }
        if (pending) A.pending[slots[2]] = (int32_t)i;
    }
    RR_STAMP(cnt, 5);
    // the surface colour and (PRE) every light's ambient / diffuse+specular terms, after the children
    // are queued: point / under / reflectv and the child rays are dead by now, which keeps the
    // pattern and `pow` code below the 128-VGPR budget without spilling
    if (has_hit) {
        const DevMaterial m = S.mats[mat];
        pcol = material_color<CP>(S, m, hr.node, over);  // material.rs:77-80
        RR_STAMPX(st0, 1);
        if (PRE) {
            double* pl = prelit_lds(S, LC);
            for (int li = 0; li < S.n_lights; ++li) {
                V3 amb, dsp;
                light_terms(m, ldc(S.lights, li), pcol, over, eyev, normalv, amb, dsp);
                const double v6[6] = {amb.x, amb.y, amb.z, dsp.x, dsp.y, dsp.z};
                for (int k = 0; k < 6; ++k) pl[(li * 6 + k) * 256 + threadIdx.x] = v6[k];
            }
        }
    }
    // surface = 0 + L0 + L1 + ... (scene.rs:159-166)
    V3 surface = mk(0, 0, 0);
#ifdef RR_STAMPS
    if (st0) cnt.st = st0;
#endif
    if constexpr (PRE) {
        const double* pl = prelit_lds(S, LC);
        for (int li = 0; li < S.n_lights; ++li) {
            const DevLight Lt = ldc(S.lights, li);
            const double in_shadow = shadow_amount<G, LC, RM>(S, A, Lt, li, over, has_hit, sample, path, cnt);
            if (has_hit) {
                const int t = threadIdx.x;
                const double* q = pl + li * 6 * 256 + t;
                const V3 amb = mk(q[0], q[256], q[512]), dsp = mk(q[768], q[1024], q[1280]);
                surface = vadd(surface, light_final(amb, dsp, in_shadow));
            }
        }
    } else {
        __shared__ ShadeStash stash;
        stash_put(stash, eyev, normalv, pcol);
        for (int li = 0; li < S.n_lights; ++li)
            light_step<G, LC, RM>(S, A, li, has_hit, mat, over, sample, path, stash, surface, cnt);
    }
#ifdef RR_STAMPS
    cnt.st = st1;
#endif
    RR_STAMP(cnt, 6);
    if (pending) {
        CombRec cr;
        cr.surf[0] = surface.x;
        cr.surf[1] = surface.y;
        cr.surf[2] = surface.z;
        cr.refl_res[0] = cr.refl_res[1] = cr.refl_res[2] = 0.0;
        cr.refl = refl;
        cr.parent = parent;
        cr.flags = CF_HIT | (slot ? CF_REFRACT_CHILD : 0);
        A.comb[i] = cr;
        if (A.comb_ext) {
            CombExt ce;
            ce.refr_res[0] = ce.refr_res[1] = ce.refr_res[2] = 0.0;
            ce.transp = transp;
            ce.R = R;
            A.comb_ext[i] = ce;
        }
    } else if (valid) {  // finished: color_at = shade_hit with black children, or black on a miss
        const V3 zero = mk(0.0, 0.0, 0.0);
        const V3 v = has_hit ? shade_sum(surface, zero, zero, refl, transp, R) : zero;
        deliver(A.level, i, parent, slot, v, A.out, A.avg, A.avg_f32, A.parent_comb, A.parent_ext, ls0);
    }
    flush(cnt, A.counters, W_SHADOW, trace_flops, trace_visits);
    RR_STAMP(cnt, 7);
}

// bottom-up: the pending events of a level, whose children are all finished, complete their sum
__device__ __forceinline__ void combine_one(const CombArgs& C, int64_t j) {
    const int64_t i = C.pending[j];
    const CombRec c = C.comb[i];
    V3 b = mk(0.0, 0.0, 0.0);  // no transparency in the scene: refracted_color is black, transparency 0
    double transp = 0.0, R = 0.0;
    if (C.comb_ext) {
        const CombExt e = C.comb_ext[i];
        b = mk(e.refr_res[0], e.refr_res[1], e.refr_res[2]);
        transp = e.transp;
        R = e.R;
    }
    const V3 v = shade_sum(mk(c.surf[0], c.surf[1], c.surf[2]), mk(c.refl_res[0], c.refl_res[1], c.refl_res[2]), b,
                           c.refl, transp, R);
    const uint32_t t = (uint32_t)(C.base + i);
    const int64_t oi = C.level == 0 ? (C.lrows > 0 ? tile_to_local_u32(t, (uint32_t)C.hs, (uint32_t)C.lrows) : t) : 0;
    deliver(C.level, i, c.parent, (c.flags & CF_REFRACT_CHILD) ? 1 : 0, v, C.out, C.avg, C.avg_f32, C.parent_comb,
            C.parent_ext, oi);
}
__global__ void __launch_bounds__(256) combine_kernel(CombArgs C) {
    const int64_t n = C.n_dev ? (int64_t)*C.n_dev : C.n;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x)
        combine_one(C, j);
}

// canvas.rs:85-96: r = 0.0; r += p (dy outer, dx inner); r /= aa*aa
template <class T>
__global__ void __launch_bounds__(256) aa_kernel(const double* __restrict__ canvas, T* __restrict__ out,
                                                 int64_t width, int64_t rows, int32_t aa) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= width * rows) return;
    int64_t y = i / width, x = i - y * width;
    const int64_t hs = width * aa;
    const double total = (double)(aa * aa);
    double r = 0.0, g = 0.0, b = 0.0;
    for (int dy = 0; dy < aa; ++dy)
        for (int dx = 0; dx < aa; ++dx) {
            const double* p = canvas + 3 * ((y * aa + dy) * hs + (x * aa + dx));
            r += p[0];
            g += p[1];
            b += p[2];
        }
    out[3 * i + 0] = (T)(r / total);
    out[3 * i + 1] = (T)(g / total);
    out[3 * i + 2] = (T)(b / total);
}

// Scene::is_shadowed for caller-given (point, light position) pairs
template <int G, bool LC>
__global__ void __launch_bounds__(256) shadow_query_kernel(DevScene S, const double* __restrict__ pts,
                                                           const double* __restrict__ lps, int64_t n,
                                                           int32_t* __restrict__ out, unsigned long long* counters) {
    if (LC) stage_culls(S);
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool valid = i < n;
    Counters cnt = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    V3 p = mk(0, 0, 0), l = mk(0, 0, 1);
    if (valid) {
        p = mk(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]);
        l = mk(lps[3 * i], lps[3 * i + 1], lps[3 * i + 2]);
    }
    bool sh = shadowed<G, LC, true>(S, p, l, valid, cnt);
    if (valid) out[i] = sh ? 1 : 0;
    flush(cnt, counters, W_SHADOW);
}

// ------------------------------------------------------------------ host-side launchers
static inline unsigned blocks_for(int64_t n) { return (unsigned)((n + 255) / 256); }
static inline size_t cull_lds(const DevScene& S) {
    return S.lds_culls ? (size_t)S.n_nodes * sizeof(DevCull) + (size_t)S.n_chunks * sizeof(DevChunk) : 0;
}

hipEvent_t KernelProf::get() {
    if (used == pool.size()) {
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        pool.push_back(e);
    }
    return pool[used++];
}

namespace {
struct Span {  // brackets one launch with events when profiling
    KernelProf* p;
    int id;
    hipStream_t st;
    hipEvent_t a = nullptr;
    Span(KernelProf* p_, int id_, hipStream_t st_) : p(p_), id(id_), st(st_) {
        if (p) {
            a = p->get();
            (void)hipEventRecord(a, st);
        }
    }
    ~Span() {
        if (p) {
            hipEvent_t b = p->get();
            (void)hipEventRecord(b, st);
            p->marks.push_back({id, {a, b}});
        }
    }
};
}  // namespace

template <int G, bool LC, bool FUSED, bool RM>
static void launch_shade_rm(const DevScene& S, const LevelArgs& A, hipStream_t st, bool pre, size_t lds) {
    const dim3 grid(blocks_for(A.n)), block(256);
#ifdef RR_QUICK
    if (pre)
        hipLaunchKernelGGL((shade_kernel<G, LC, FUSED, true, false, RM>), grid, block, lds, st, S, A);
    else
        hipLaunchKernelGGL((shade_kernel<G, LC, FUSED, false, false, RM>), grid, block, lds, st, S, A);
#else
    if (S.complex_patterns) {
        if (pre)
            hipLaunchKernelGGL((shade_kernel<G, LC, FUSED, true, true, RM>), grid, block, lds, st, S, A);
        else
            hipLaunchKernelGGL((shade_kernel<G, LC, FUSED, false, true, RM>), grid, block, lds, st, S, A);
    } else {
        if (pre)
            hipLaunchKernelGGL((shade_kernel<G, LC, FUSED, true, false, RM>), grid, block, lds, st, S, A);
        else
            hipLaunchKernelGGL((shade_kernel<G, LC, FUSED, false, false, RM>), grid, block, lds, st, S, A);
    }
#endif
}
// RM (ray-major chunk tests, walk_nodes) for the secondary levels, whose waves are often
// incoherent, and for every level of scenes with groups (a mesh chunk holds many small triangles:
// C4 teapot 1.65 -> 1.35 ms per frame with it at level 0).  Level 0 of flat scenes (camera tiles and
// their shadow rays) runs without it, which keeps the camera kernels' registers (C2 0.172 vs
// 0.177 ms with it).
template <int G, bool LC, bool FUSED>
static void launch_shade(const DevScene& S, const LevelArgs& A, hipStream_t st, bool pre, size_t lds) {
    if (A.level > 0 || G > 0)
        launch_shade_rm<G, LC, FUSED, true>(S, A, st, pre, lds);
    else
        launch_shade_rm<G, LC, FUSED, false>(S, A, st, pre, lds);
}

template <int G, bool LC>
static void launch_level_t(const DevScene& S, const LevelArgs& A, hipStream_t st, KernelProf* prof) {
    const bool pre = S.n_lights <= RR_PRELIT_LIGHTS;
    const size_t shade_lds = cull_lds(S) + (pre ? (size_t)S.n_lights * 6 * 256 * sizeof(double) : 0);
    if (!S.has_transparent && !std::getenv("RRAY_UNFUSED")) {  // trace + shade in one kernel
        Span s(prof, K_TRACE_SHADE, st);
        launch_shade<G, LC, true>(S, A, st, pre, shade_lds);
        return;
    }
    {
        Span s(prof, K_TRACE, st);
        if (A.level > 0)
            hipLaunchKernelGGL((trace_kernel<G, LC, true>), dim3(blocks_for(A.n)), dim3(256), cull_lds(S), st, S, A);
        else
            hipLaunchKernelGGL((trace_kernel<G, LC, false>), dim3(blocks_for(A.n)), dim3(256), cull_lds(S), st, S, A);
    }
    if (S.has_transparent) {
        Span s(prof, K_N1N2, st);
        if (A.level > 0)
            hipLaunchKernelGGL((n1n2_kernel<G, LC, true>), dim3(blocks_for(A.n)), dim3(256), cull_lds(S), st, S, A);
        else
            hipLaunchKernelGGL((n1n2_kernel<G, LC, false>), dim3(blocks_for(A.n)), dim3(256), cull_lds(S), st, S, A);
    }
    {
        Span s(prof, K_SHADE, st);
        launch_shade<G, LC, false>(S, A, st, pre, shade_lds);
    }
}

hipError_t launch_level(const DevScene& S, const LevelArgs& A, hipStream_t st, KernelProf* prof) {
    if (A.n <= 0) return hipSuccess;
    const int g = S.general ? 2 : S.has_groups ? 1 : 0;  // G: flat / groups / general (CSG, 4-entry leaves)
#ifdef RR_QUICK  // experiment builds: only the flat, LDS-culled, simple-pattern kernels (fast compiles)
    if (g != 0 || !S.lds_culls || S.complex_patterns) return hipErrorNotSupported;
    launch_level_t<0, true>(S, A, st, prof);
#else
    if (g == 2) {
        if (S.lds_culls)
            launch_level_t<2, true>(S, A, st, prof);
        else
            launch_level_t<2, false>(S, A, st, prof);
    } else if (g == 1) {
        if (S.lds_culls)
            launch_level_t<1, true>(S, A, st, prof);
        else
            launch_level_t<1, false>(S, A, st, prof);
    } else {
        if (S.lds_culls)
            launch_level_t<0, true>(S, A, st, prof);
        else
            launch_level_t<0, false>(S, A, st, prof);
    }
#endif
    return hipGetLastError();
}

hipError_t launch_combine(const CombArgs& C, hipStream_t st, KernelProf* prof) {
    if (C.n <= 0) return hipSuccess;
    Span s(prof, K_COMBINE, st);
    // grid-stride over the live count: the capacity can be far above it (worst case per level)
    const unsigned grid = std::min<unsigned>(blocks_for(C.n), 256u * 16u);
    hipLaunchKernelGGL(combine_kernel, dim3(grid), dim3(256), 0, st, C);
    return hipGetLastError();
}

template <class T>
static hipError_t launch_aa_t(const double* canvas, T* out, int64_t width, int64_t rows, int32_t aa, hipStream_t st,
                              KernelProf* prof) {
    int64_t n = width * rows;
    if (n == 0) return hipSuccess;
    Span s(prof, K_AA, st);
    hipLaunchKernelGGL((aa_kernel<T>), dim3(blocks_for(n)), dim3(256), 0, st, canvas, out, width, rows, aa);
    return hipGetLastError();
}
hipError_t launch_aa(const double* canvas, double* out, int64_t width, int64_t rows, int32_t aa, hipStream_t st,
                     KernelProf* prof) {
    return launch_aa_t(canvas, out, width, rows, aa, st, prof);
}
hipError_t launch_aa_f32(const double* canvas, float* out, int64_t width, int64_t rows, int32_t aa, hipStream_t st,
                         KernelProf* prof) {
    return launch_aa_t(canvas, out, width, rows, aa, st, prof);
}

template <int G, bool LC>
static void launch_shadow_query_t(const DevScene& S, const double* pts, const double* lps, int64_t n, int32_t* out,
                                  unsigned long long* counters, hipStream_t st) {
    hipLaunchKernelGGL((shadow_query_kernel<G, LC>), dim3(blocks_for(n)), dim3(256), cull_lds(S), st, S, pts, lps, n, out,
                       counters);
}

hipError_t launch_shadow_query(const DevScene& S, const double* pts, const double* lps, int64_t n, int32_t* out,
                               unsigned long long* counters, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const int g = S.general ? 2 : S.has_groups ? 1 : 0;
    if (g == 2) {
        if (S.lds_culls)
            launch_shadow_query_t<2, true>(S, pts, lps, n, out, counters, st);
        else
            launch_shadow_query_t<2, false>(S, pts, lps, n, out, counters, st);
    } else if (g == 1) {
        if (S.lds_culls)
            launch_shadow_query_t<1, true>(S, pts, lps, n, out, counters, st);
        else
            launch_shadow_query_t<1, false>(S, pts, lps, n, out, counters, st);
    } else {
        if (S.lds_culls)
            launch_shadow_query_t<0, true>(S, pts, lps, n, out, counters, st);
        else
            launch_shadow_query_t<0, false>(S, pts, lps, n, out, counters, st);
    }
    return hipGetLastError();
}

}  // namespace rr
