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
#include "render_common.inc"

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
    Counters cnt = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    V3 p = mk(0, 0, 0), l = mk(0, 0, 1);
    if (valid) {
        p = mk(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]);
        l = mk(lps[3 * i], lps[3 * i + 1], lps[3 * i + 2]);
    }
    bool sh = shadowed<G, LC, true, cross_lane_ok(G, false, false)>(S, p, l, valid, cnt);
    if (valid) out[i] = sh ? 1 : 0;
    flush(cnt, counters, W_SHADOW);
}


// One thread per full 8x8 tile of the part: its four corner camera rays exactly as the level-0 lanes compute
// them (level0_px + camera_ray, then f32), and the tile's bundle from them (cam_corner_bundle).  Run once per
// camera / part layout (the context caches the table), so the level-0 walks read their bundle instead of
// building it (~100 VALU per wave).
__global__ void __launch_bounds__(256) tile_bundle_kernel(LevelArgs A, float* __restrict__ out, int64_t n_tiles) {
    const int64_t T = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (T >= n_tiles) return;
    const int corner[4] = {0, 7, 56, 63};
    float o[3] = {0.0f, 0.0f, 0.0f}, dc[4][3];
    for (int j = 0; j < 4; ++j) {
        const Px0 q = level0_px<false>(A, T * 64 + corner[j]);
        const Ray r = camera_ray(A.cam, A.cam_affine, q.px, q.py);
        o[0] = (float)r.o.x;
        o[1] = (float)r.o.y;
        o[2] = (float)r.o.z;
        dc[j][0] = (float)r.d.x;
        dc[j][1] = (float)r.d.y;
        dc[j][2] = (float)r.d.z;
    }
    const Bundle B = cam_corner_bundle(o, dc);
    float* p = out + T * RR_TILE_BUNDLE_FLOATS;
    for (int k = 0; k < 3; ++k) {
        p[k] = B.o[k];
        p[3 + k] = B.a[k];
    }
    p[6] = B.rho;
    p[7] = B.tanT;
    p[8] = B.secT;
    p[9] = __int_as_float(B.ok);
    p[10] = p[11] = 0.0f;
}

// One thread per pixel wave (A.pw): the bundle of the rectangle spanning the wave's samples (the first and last
// pixel's columns, the band's rows) from its four corner rays — every sample ray of the wave lies in the cone of the
// rectangle's corner rays (the argument of the 8x8 tiles).
__global__ void __launch_bounds__(256) pixel_wave_bundle_kernel(LevelArgs A, float* __restrict__ out, int64_t n_waves) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_waves) return;
    const PixelWave pw = pixel_wave(A, (uint32_t)g);
    const uint32_t W = (uint32_t)A.hs / 3u;  // output pixels per row
    const uint32_t p0 = 7u * pw.w, p_end = pw.rb * W - 1u, p1 = p0 + 6u < p_end ? p0 + 6u : p_end;
    const uint32_t c0 = pw.rb == 2u ? p0 >> 1 : p0, c1 = pw.rb == 2u ? p1 >> 1 : p1;
    const uint32_t x0 = 3u * c0, x1 = 3u * c1 + 2u;
    const uint32_t y0 = 6u * pw.band, y1 = y0 + 3u * pw.rb - 1u;
    const uint32_t cx[4] = {x0, x1, x0, x1}, cy[4] = {y0, y0, y1, y1};
    float o[3] = {0.0f, 0.0f, 0.0f}, dc[4][3];
    for (int j = 0; j < 4; ++j) {
        const Ray r = camera_ray(A.cam, A.cam_affine, cx[j], canvas_row(A, cy[j]));
        o[0] = (float)r.o.x;
        o[1] = (float)r.o.y;
        o[2] = (float)r.o.z;
        dc[j][0] = (float)r.d.x;
        dc[j][1] = (float)r.d.y;
        dc[j][2] = (float)r.d.z;
    }
    const Bundle B = cam_corner_bundle(o, dc);
    float* p = out + g * RR_TILE_BUNDLE_FLOATS;
    for (int k = 0; k < 3; ++k) {
        p[k] = B.o[k];
        p[3 + k] = B.a[k];
    }
    p[6] = B.rho;
    p[7] = B.tanT;
    p[8] = B.secT;
    p[9] = __int_as_float(B.ok);
    p[10] = p[11] = 0.0f;
}

hipError_t launch_pixel_wave_bundles(const LevelArgs& A, float* out, int64_t n_waves, hipStream_t st) {
    if (n_waves <= 0) return hipSuccess;
    hipLaunchKernelGGL(pixel_wave_bundle_kernel, dim3(blocks_for(n_waves)), dim3(256), 0, st, A, out, n_waves);
    return hipGetLastError();
}

// A first frame's tile order before any tile has been timed: each tile's cost is guessed from its camera bundle as
// 16 + the number of nodes in the chunks its bundle may reach (the walk's candidates), on the clock-cycle scale the
// counting sort buckets logarithmically (x 64).  Only the launch order depends on it; the frame after re-sorts by
// the measured costs.  One thread per tile (or pixel wave).
__global__ void __launch_bounds__(256) tile_guess_kernel(DevScene S, const float* __restrict__ bundles,
                                                         uint32_t* __restrict__ cost, int64_t n_tiles) {
    const int64_t T = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (T >= n_tiles) return;
    const Bundle B = load_tile_bundle(bundles + T * RR_TILE_BUNDLE_FLOATS);
    uint32_t c = 16u;
    const int nch = S.n_chunks - S.n_free;
    for (int j = 0; j < nch; ++j) {
        const DevChunk ch = S.chunks[j];
        if (!B.ok || bundle_may_hit<false, true>(B, ch.cull)) c += (uint32_t)ch.count;
    }
    cost[T] = c * 64u;
}

hipError_t launch_tile_guess(const DevScene& S, const float* bundles, uint32_t* cost, int64_t n_tiles, hipStream_t st) {
    if (n_tiles <= 0) return hipSuccess;
    hipLaunchKernelGGL(tile_guess_kernel, dim3(blocks_for(n_tiles)), dim3(256), 0, st, S, bundles, cost, n_tiles);
    return hipGetLastError();
}

// Tiles by decreasing cost (a counting sort on 256 buckets: 8 per power of two of the cycle count), so a
// frame's costliest tiles start first and its last waves are its cheapest: the launch's tail, where CUs run
// out of waves, shrinks.  Ties in a bucket land in any order (only timing depends on it).  Three small
// launches over many blocks (the one-block sort took 159 us for C4's 129 600 tiles, most of a cold frame's
// extra cost): per-block LDS histograms added into 256 global counters, an exclusive scan of the 256, then a
// scatter in which each block reserves its run of every bucket with one global atomic per non-empty bucket.
__device__ __forceinline__ int cost_bucket(uint32_t c) {
    if (c == 0) return 255;
    const int e = 31 - __clz(c);
    const int q = e * 8 + (int)((e >= 3 ? c >> (e - 3) : c << (3 - e)) & 7u);
    return 255 - (q > 255 ? 255 : q);
}
constexpr int RR_ORDER_BLOCK = 256, RR_ORDER_PER_THREAD = 16;  // 4096 tiles per block
// the sort's units: single tiles (group 1) or groups of RR_ORDER_GROUP consecutive tiles (a block's four waves),
// whose cost is the sum of their tiles' (saturating)
__device__ __forceinline__ uint32_t group_cost(const uint32_t* cost, int64_t g, int group) {
    if (group == 1) return cost[g];
    uint64_t c = 0;
#pragma unroll
    for (int k = 0; k < RR_ORDER_GROUP; ++k) c += cost[g * RR_ORDER_GROUP + k];
    return c > 0xffffffffull ? 0xffffffffu : (uint32_t)c;
}
__global__ void __launch_bounds__(RR_ORDER_BLOCK) tile_hist_kernel(const uint32_t* __restrict__ cost,
                                                                   uint32_t* __restrict__ hist, int64_t n, int group) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t b0 = (int64_t)blockIdx.x * RR_ORDER_BLOCK * RR_ORDER_PER_THREAD;
    for (int k = 0; k < RR_ORDER_PER_THREAD; ++k) {
        const int64_t i = b0 + (int64_t)k * RR_ORDER_BLOCK + threadIdx.x;
        if (i < n) atomicAdd(&h[cost_bucket(group_cost(cost, i, group))], 1u);
    }
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}
// hist -> exclusive prefix (the first slot of each bucket), in place; one block of 256
__global__ void __launch_bounds__(256) tile_scan_kernel(uint32_t* __restrict__ hist) {
    __shared__ uint32_t v[256];
    const int t = threadIdx.x;
    v[t] = hist[t];
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {  // Hillis-Steele inclusive scan
        const uint32_t a = t >= off ? v[t - off] : 0u;
        __syncthreads();
        v[t] += a;
        __syncthreads();
    }
    hist[t] = t ? v[t - 1] : 0u;
}
__global__ void __launch_bounds__(RR_ORDER_BLOCK) tile_scatter_kernel(const uint32_t* __restrict__ cost,
                                                                      uint32_t* __restrict__ cursor,
                                                                      uint32_t* __restrict__ perm, int64_t n, int group) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t b0 = (int64_t)blockIdx.x * RR_ORDER_BLOCK * RR_ORDER_PER_THREAD;
    int bk[RR_ORDER_PER_THREAD];
#pragma unroll
    for (int k = 0; k < RR_ORDER_PER_THREAD; ++k) {
        const int64_t i = b0 + (int64_t)k * RR_ORDER_BLOCK + threadIdx.x;
        bk[k] = i < n ? cost_bucket(group_cost(cost, i, group)) : -1;
        if (bk[k] >= 0) atomicAdd(&h[bk[k]], 1u);
    }
    __syncthreads();
    // this block's run of each bucket: one global atomic per non-empty bucket
    const uint32_t c = h[threadIdx.x];
    __syncthreads();
    h[threadIdx.x] = c ? atomicAdd(&cursor[threadIdx.x], c) : 0u;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < RR_ORDER_PER_THREAD; ++k) {
        const int64_t i = b0 + (int64_t)k * RR_ORDER_BLOCK + threadIdx.x;
        if (bk[k] >= 0) perm[atomicAdd(&h[bk[k]], 1u)] = (uint32_t)i;
    }
}

// scratch: 256 u32 of device memory for the bucket counters; perm: launch slot -> tile (group 1) or launch block ->
// tile group (group RR_ORDER_GROUP; n_tiles a multiple of it)
hipError_t launch_tile_order(const uint32_t* cost, uint32_t* perm, uint32_t* scratch, int64_t n_tiles, int group,
                             hipStream_t st) {
    if (n_tiles <= 0) return hipSuccess;
    if (group != 1 && group != RR_ORDER_GROUP) return hipErrorInvalidValue;
    n_tiles /= group;  // the sort's units: tiles or tile groups
    const unsigned blocks = (unsigned)((n_tiles + RR_ORDER_BLOCK * RR_ORDER_PER_THREAD - 1) / (RR_ORDER_BLOCK * RR_ORDER_PER_THREAD));
    hipError_t e = hipMemsetAsync(scratch, 0, 256 * sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(tile_hist_kernel, dim3(blocks), dim3(RR_ORDER_BLOCK), 0, st, cost, scratch, n_tiles, group);
    hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(256), 0, st, scratch);
    hipLaunchKernelGGL(tile_scatter_kernel, dim3(blocks), dim3(RR_ORDER_BLOCK), 0, st, cost, scratch, perm, n_tiles, group);
    return hipGetLastError();
}

hipError_t launch_tile_bundles(const DevScene& S, const LevelArgs& A, float* out, int64_t n_tiles, hipStream_t st) {
    (void)S;
    if (n_tiles <= 0) return hipSuccess;
    hipLaunchKernelGGL(tile_bundle_kernel, dim3(blocks_for(n_tiles)), dim3(256), 0, st, A, out, n_tiles);
    return hipGetLastError();
}

hipEvent_t KernelProf::get() {
    if (used == pool.size()) {
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        pool.push_back(e);
    }
    return pool[used++];
}


bool fused_levels(const DevScene& S) { return !S.has_transparent && !std::getenv("RRAY_UNFUSED"); }

hipError_t launch_level(const DevScene& S, const LevelArgs& A, hipStream_t st, KernelProf* prof) {
    if (A.n <= 0) return hipSuccess;
    const int g = S.general ? 2 : S.has_groups ? 1 : 0;  // G: flat / groups / general (CSG, 4-entry leaves)
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
    return hipGetLastError();
}

bool chain_levels(const DevScene& S, int max_children, int max_depth) {
    return fused_levels(S) && max_children > 0 && max_depth > 0 && !std::getenv("RRAY_NO_CHAIN");
}

hipError_t launch_chain(const DevScene& S, const LevelArgs& A, hipStream_t st, KernelProf* prof, bool deep) {
    if (A.n <= 0) return hipSuccess;
    const int g = S.general ? 2 : S.has_groups ? 1 : 0;
    if (g == 2) {
        if (S.lds_culls)
            launch_chain_t<2, true>(S, A, st, prof, deep);
        else
            launch_chain_t<2, false>(S, A, st, prof, deep);
    } else if (g == 1) {
        if (S.lds_culls)
            launch_chain_t<1, true>(S, A, st, prof, deep);
        else
            launch_chain_t<1, false>(S, A, st, prof, deep);
    } else {
        if (S.lds_culls)
            launch_chain_t<0, true>(S, A, st, prof, deep);
        else
            launch_chain_t<0, false>(S, A, st, prof, deep);
    }
    return hipGetLastError();
}

bool tree_levels(const DevScene& S) { return S.has_transparent && !std::getenv("RRAY_NO_TREE"); }

hipError_t launch_tree(const DevScene& S, const LevelArgs& A, hipStream_t st, KernelProf* prof) {
    if (A.n <= 0) return hipSuccess;
    const int g = S.general ? 2 : S.has_groups ? 1 : 0;
    if (g == 2) {
        if (S.lds_culls)
            launch_tree_t<2, true>(S, A, st, prof);
        else
            launch_tree_t<2, false>(S, A, st, prof);
    } else if (g == 1) {
        if (S.lds_culls)
            launch_tree_t<1, true>(S, A, st, prof);
        else
            launch_tree_t<1, false>(S, A, st, prof);
    } else {
        if (S.lds_culls)
            launch_tree_t<0, true>(S, A, st, prof);
        else
            launch_tree_t<0, false>(S, A, st, prof);
    }
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
