// render.hip — wavefront kernels of the MI355X (gfx950) render path.
//
// Camera::render (camera.rs:107-121) -> Scene::color_at (scene.rs:128-136), evaluated level by
// level over HBM-resident queues (wavefront.hpp):
//   trace_kernel   closest hit per pending color_at ray           scene.rs:97-106,130
//   n1n2_kernel    container walk for transparent hits             intersection.rs:61-92
//   shade_kernel   prepare_computations, pattern, children rays    intersection.rs:50-60, scene.rs:281-336
//   shadow_kernel  is_shadowed for every (hit, light, sample)      scene.rs:181-214,234-245
//   finish_kernel  lighting sum per hit                            scene.rs:159-166, light.rs:98-140
//   combine_kernel bottom-up shade_hit sums                        scene.rs:167-177
//   aa_kernel      box average before `as u8`                      canvas.rs:76-96
// Every kernel is one work-item per queue entry; the node loops inside are wave-uniform (scalar
// broadcast loads of the flattened scene) so the f64 VALU does all the work.
#include "device_core.inc"
#include "kernels.hpp"
#include "wavefront.hpp"

namespace rr {

// local sample index of this part -> (px, py) on the supersampled canvas (interleaved row blocks)
__device__ __forceinline__ void local_to_pixel(const LevelArgs& A, int64_t ls, int64_t& px, int64_t& py) {
    int64_t lrow = ls / A.hs;
    px = ls - lrow * A.hs;
    int64_t k = lrow / A.aa, sub = lrow - k * A.aa;
    int64_t bi = k / A.block_rows, kb = k - bi * A.block_rows;
    int64_t y = (bi * A.nparts + A.part) * A.block_rows + kb;
    py = y * A.aa + sub;
}

// Camera::ray_for_pixel (camera.rs:75-93) with the full 4x4 camera inverse (w included)
__device__ Ray camera_ray(const DevCamera& C, int64_t px, int64_t py) {
    double xoffset = ((double)px + 0.5) * C.pixel_size;
    double yoffset = ((double)py + 0.5) * C.pixel_size;
    double wx = C.half_width - xoffset;
    double wy = C.half_height - yoffset;
    const double* M = C.inv;
    double pw[4], ow[4];
    for (int r = 0; r < 4; ++r) {
        pw[r] = M[4 * r] * wx + M[4 * r + 1] * wy + M[4 * r + 2] * -1.0 + M[4 * r + 3] * 1.0;
        ow[r] = M[4 * r] * 0.0 + M[4 * r + 1] * 0.0 + M[4 * r + 2] * 0.0 + M[4 * r + 3] * 1.0;
    }
    double dx = pw[0] - ow[0], dy = pw[1] - ow[1], dz = pw[2] - ow[2], dw = pw[3] - ow[3];
    double mag = sqrt(dx * dx + dy * dy + dz * dz + dw * dw);
    return {mk(ow[0], ow[1], ow[2]), mk(dx / mag, dy / mag, dz / mag)};
}

// the ray of event i at this level
__device__ __forceinline__ Ray event_ray(const LevelArgs& A, int64_t i) {
    if (A.level > 0) {
        const Event& e = A.ev[i];
        return {mk(e.o[0], e.o[1], e.o[2]), mk(e.d[0], e.d[1], e.d[2])};
    }
    if (A.rays0) {
        const double* p = A.rays0 + 6 * (A.base + i);
        return {mk(p[0], p[1], p[2]), mk(p[3], p[4], p[5])};
    }
    int64_t px, py;
    local_to_pixel(A, A.base + i, px, py);
    return camera_ray(A.cam, px, py);
}
// jitter identity of event i: (global sample id, recursion path)
__device__ __forceinline__ void event_key(const LevelArgs& A, int64_t i, uint64_t& sample, uint32_t& path) {
    int64_t ls = A.level > 0 ? (int64_t)A.ev[i].sample : A.base + i;
    path = A.level > 0 ? A.ev[i].path : 1u;
    if (A.rays0) {
        sample = (uint64_t)ls;
    } else {
        int64_t px, py;
        local_to_pixel(A, ls, px, py);
        sample = (uint64_t)(py * A.hs + px);
    }
}

// wave-aggregated queue append: returns this lane's slot (valid only where `want`)
__device__ __forceinline__ int32_t wave_append(unsigned int* counter, bool want) {
    uint64_t mask = __ballot(want);
    if (mask == 0) return -1;
    const int lane = threadIdx.x & 63;
    int leader = __ffsll((long long)mask) - 1;
    unsigned int base = 0;
    if (lane == leader) base = atomicAdd(counter, (unsigned int)__popcll(mask));
    base = __shfl(base, leader, 64);
    uint64_t below = lane == 0 ? 0ull : (mask & ((~0ull) >> (64 - lane)));
    return (int32_t)(base + (unsigned int)__popcll(below));
}

__device__ void flush(Counters& cnt, unsigned long long* counters) {
    uint64_t s;
    const bool l0 = (threadIdx.x & 63) == 0;
    s = wave_sum_u64(cnt.rays);
    if (l0 && s) atomicAdd(counters + C_RAYS, (unsigned long long)s);
    s = wave_sum_u64(cnt.shadow);
    if (l0 && s) atomicAdd(counters + C_SHADOW, (unsigned long long)s);
    s = wave_sum_u64(cnt.shade);
    if (l0 && s) atomicAdd(counters + C_SHADE, (unsigned long long)s);
    s = wave_sum_u64(cnt.n1n2);
    if (l0 && s) atomicAdd(counters + C_N1N2, (unsigned long long)s);
    s = wave_sum_u64(cnt.gtests);
    if (l0 && s) atomicAdd(counters + C_GROUP_TESTS, (unsigned long long)s);
    s = wave_sum_u64(cnt.ghits);
    if (l0 && s) atomicAdd(counters + C_GROUP_HITS, (unsigned long long)s);
    s = wave_sum_u64(cnt.tests);
    if (l0 && s) atomicAdd(counters + C_PRIM_TESTS, (unsigned long long)s);
}

__device__ __forceinline__ bool needs_n1n2(const DevMaterial& m, int rem) {
    // n1/n2 feed refracted_color (rem > 0, transparency != 0) and schlick (reflective > 0 &&
    // transparency > 0); both need transparency != 0.
    return m.transparency != 0.0 && (rem > 0 || m.reflective > 0.0);
}

template <bool G>
__global__ void __launch_bounds__(256) trace_kernel(DevScene S, LevelArgs A) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = i < A.n;
    Counters cnt = {0, 0, 0, 0, 0, 0, 0};
    Ray r = valid ? event_ray(A, i) : Ray{mk(0, 0, 0), mk(0, 0, 1)};
    Hit h;
    trace_closest<G>(S, r, valid, h, cnt);
    if (valid) {
        cnt.rays++;
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
    if (S.has_transparent) {
        int32_t slot = wave_append(A.lcount + LC_N1N2, want);
        if (want) A.n1n2_list[slot] = (int32_t)i;
    }
    flush(cnt, A.counters);
}

template <bool G>
__global__ void __launch_bounds__(256) n1n2_kernel(DevScene S, LevelArgs A) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t cnt_n = (int64_t)A.lcount[LC_N1N2];
    const bool valid = j < cnt_n;
    Counters cnt = {0, 0, 0, 0, 0, 0, 0};
    int64_t i = valid ? A.n1n2_list[j] : 0;
    Ray r = valid ? event_ray(A, i) : Ray{mk(0, 0, 0), mk(0, 0, 1)};
    Hit h;
    h.found = valid;
    h.t = 0.0;
    h.node = -1;
    h.k = 0;
    if (valid) {
        HitRec hr = A.hit[i];
        h.t = hr.t;
        h.u = hr.u;
        h.v = hr.v;
        h.node = hr.node;
        h.k = hr.k;
    }
    double n1 = 1.0, n2 = 1.0;
    n1n2_walk<G>(S, r, h, valid, n1, n2, cnt);
    if (valid) {
        A.n12[2 * i] = n1;
        A.n12[2 * i + 1] = n2;
    }
    flush(cnt, A.counters);
}

__global__ void __launch_bounds__(256) shade_kernel(DevScene S, LevelArgs A) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = i < A.n;
    Counters cnt = {0, 0, 0, 0, 0, 0, 0};
    HitRec hr;
    hr.node = -1;
    if (valid) hr = A.hit[i];
    const bool has_hit = valid && hr.node >= 0;
    int32_t parent = -1, slot = 0;
    if (valid && A.level > 0) {
        parent = A.ev[i].parent;
        slot = A.ev[i].slot;
    }
    CombRec cr;
    cr.surf[0] = cr.surf[1] = cr.surf[2] = 0.0;
    cr.refl_res[0] = cr.refl_res[1] = cr.refl_res[2] = 0.0;
    cr.refr_res[0] = cr.refr_res[1] = cr.refr_res[2] = 0.0;
    cr.refl = 0.0;
    cr.transp = 0.0;
    cr.R = 0.0;
    cr.parent = parent;
    cr.flags = slot ? CF_REFRACT_CHILD : 0;
    bool do_refl = false, do_refr = false;
    Ray rr, refr;
    Comps c;
    uint64_t sample = 0;
    uint32_t path = 1u;
    if (has_hit) {
        cnt.shade++;
        Ray r = event_ray(A, i);
        Hit h;
        h.found = true;
        h.t = hr.t;
        h.u = hr.u;
        h.v = hr.v;
        h.node = hr.node;
        h.k = hr.k;
        prepare(S, r, h, c);  // intersection.rs:50-60
        DevMaterial m = S.mats[S.nodes[hr.node].material];
        if (S.has_transparent && needs_n1n2(m, A.rem)) {
            c.n1 = A.n12[2 * i];
            c.n2 = A.n12[2 * i + 1];
        }
        V3 pcol = pattern_at(S, m.pattern, world_to_object(S, hr.node, c.over));  // material.rs:77-80
        ShadeRec sr;
        sr.over[0] = c.over.x;
        sr.over[1] = c.over.y;
        sr.over[2] = c.over.z;
        sr.eyev[0] = c.eyev.x;
        sr.eyev[1] = c.eyev.y;
        sr.eyev[2] = c.eyev.z;
        sr.normalv[0] = c.normalv.x;
        sr.normalv[1] = c.normalv.y;
        sr.normalv[2] = c.normalv.z;
        sr.pcol[0] = pcol.x;
        sr.pcol[1] = pcol.y;
        sr.pcol[2] = pcol.z;
        sr.material = S.nodes[hr.node].material;
        sr.pad = 0;
        A.sr[i] = sr;
        // reflected_color (scene.rs:281-290) / refracted_color (scene.rs:310-336)
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
        cr.refl = m.reflective;
        cr.transp = m.transparency;
        cr.R = (m.reflective > 0.0 && m.transparency > 0.0) ? schlick(c) : 0.0;
        cr.flags |= CF_HIT;
        if (do_refl || do_refr) event_key(A, i, sample, path);
    }
    if (valid) A.comb[i] = cr;
    // children of this level -> next level queue (wave-aggregated appends keep siblings adjacent)
    int32_t s1 = wave_append(A.lcount + LC_CHILDREN, do_refl);
    if (do_refl) {
        Event e;
        e.o[0] = rr.o.x;
        e.o[1] = rr.o.y;
        e.o[2] = rr.o.z;
        e.d[0] = rr.d.x;
        e.d[1] = rr.d.y;
        e.d[2] = rr.d.z;
        e.sample = A.level > 0 ? A.ev[i].sample : (uint32_t)(A.base + i);
        e.path = path * 2u;
        e.parent = (int32_t)i;
        e.slot = 0;
        A.next[s1] = e;
    }
    int32_t s2 = wave_append(A.lcount + LC_CHILDREN, do_refr);
    if (do_refr) {
        Event e;
        e.o[0] = refr.o.x;
        e.o[1] = refr.o.y;
        e.o[2] = refr.o.z;
        e.d[0] = refr.d.x;
        e.d[1] = refr.d.y;
        e.d[2] = refr.d.z;
        e.sample = A.level > 0 ? A.ev[i].sample : (uint32_t)(A.base + i);
        e.path = path * 2u + 1u;
        e.parent = (int32_t)i;
        e.slot = 1;
        A.next[s2] = e;
    }
    int32_t sl = wave_append(A.lcount + LC_LIT, has_hit);
    if (has_hit) A.lit[sl] = (int32_t)i;
    flush(cnt, A.counters);
}

// one work-item per (lit hit, shadow slot j): j enumerates lights, and level^2 samples for area
// lights (light.rs:47-65 sample_point with the deterministic jitter)
template <bool G>
__global__ void __launch_bounds__(256) shadow_kernel(DevScene S, LevelArgs A) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)A.lcount[LC_LIT] * A.n_sr;
    const bool valid = idx < total;
    Counters cnt = {0, 0, 0, 0, 0, 0, 0};
    V3 p = mk(0, 0, 0), target = mk(0, 0, 1);
    if (valid) {
        int64_t L = idx / A.n_sr;
        int32_t j = (int32_t)(idx - L * A.n_sr);
        int64_t e = A.lit[L];
        const ShadeRec& sr = A.sr[e];
        p = mk(sr.over[0], sr.over[1], sr.over[2]);
        int li = A.sr_light[j];
        DevLight Lt = S.lights[li];
        if (Lt.kind == RR_LIGHT_POINT) {
            target = mk(Lt.position[0], Lt.position[1], Lt.position[2]);
        } else {
            int s = A.sr_s[j];
            int row = s / Lt.level, col = s % Lt.level;
            double ur = 0.5, vr = 0.5;
            if (A.jitter_mode == 0) {
                uint64_t sample;
                uint32_t path;
                event_key(A, e, sample, path);
                ur = jitter(A.seed, sample, path, (uint32_t)li, (uint32_t)s, 0);
                vr = jitter(A.seed, sample, path, (uint32_t)li, (uint32_t)s, 1);
            }
            double uf = ((double)col + ur) / (double)Lt.level;
            double vf = ((double)row + vr) / (double)Lt.level;
            target = vadd(vadd(mk(Lt.corner[0], Lt.corner[1], Lt.corner[2]), vmul(mk(Lt.u[0], Lt.u[1], Lt.u[2]), uf)),
                          vmul(mk(Lt.v[0], Lt.v[1], Lt.v[2]), vf));
        }
    }
    bool sh = shadowed<G>(S, p, target, valid, cnt);
    if (valid) A.sb[idx] = sh ? 1 : 0;
    flush(cnt, A.counters);
}

// shade_hit's light sum (scene.rs:159-166): surface = 0 + L0 + L1 + ...
__global__ void __launch_bounds__(256) finish_kernel(DevScene S, LevelArgs A) {
    const int64_t L = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (L >= (int64_t)A.lcount[LC_LIT]) return;
    const int64_t e = A.lit[L];
    const ShadeRec sr = A.sr[e];
    const DevMaterial m = S.mats[sr.material];
    V3 over = mk(sr.over[0], sr.over[1], sr.over[2]);
    V3 eyev = mk(sr.eyev[0], sr.eyev[1], sr.eyev[2]);
    V3 nrm = mk(sr.normalv[0], sr.normalv[1], sr.normalv[2]);
    V3 pcol = mk(sr.pcol[0], sr.pcol[1], sr.pcol[2]);
    V3 surface = mk(0, 0, 0);
    const uint8_t* bits = A.sb + L * A.n_sr;
    int j = 0;
    for (int li = 0; li < S.n_lights; ++li) {
        DevLight Lt = ldc(S.lights, li);
        double in_shadow;
        if (Lt.kind == RR_LIGHT_POINT) {
            in_shadow = bits[j] ? 1.0 : 0.0;
            j += 1;
        } else {
            int amount = Lt.level * Lt.level, total = 0;
            for (int s = 0; s < amount; ++s) total += bits[j + s];
            in_shadow = (double)total / (double)amount;
            j += amount;
        }
        surface = vadd(surface, lighting(m, Lt, pcol, over, eyev, nrm, in_shadow));
    }
    CombRec& cr = A.comb[e];
    cr.surf[0] = surface.x;
    cr.surf[1] = surface.y;
    cr.surf[2] = surface.z;
}

// shade_hit's final sum (scene.rs:172-177)
__device__ __forceinline__ V3 combine3(const CombRec& c) {
    V3 s = mk(c.surf[0], c.surf[1], c.surf[2]);
    V3 a = mk(c.refl_res[0], c.refl_res[1], c.refl_res[2]);
    V3 b = mk(c.refr_res[0], c.refr_res[1], c.refr_res[2]);
    if (c.refl > 0.0 && c.transp > 0.0) return vadd(vadd(s, vmul(a, c.R)), vmul(b, 1.0 - c.R));
    return vadd(vadd(s, a), b);
}

// bottom-up: this level's color_at values -> the parents' reflected/refracted slots, or the canvas
__global__ void __launch_bounds__(256) combine_kernel(CombArgs C) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C.n) return;
    const CombRec c = C.comb[i];
    V3 v = (c.flags & CF_HIT) ? combine3(c) : mk(0.0, 0.0, 0.0);
    if (C.level == 0) {
        double* o = C.out + 3 * (C.base + i);
        o[0] = v.x;
        o[1] = v.y;
        o[2] = v.z;
        return;
    }
    CombRec& p = C.parent_comb[c.parent];
    if (c.flags & CF_REFRACT_CHILD) {  // refracted_color = color_at(...) * transparency
        double t = p.transp;
        p.refr_res[0] = v.x * t;
        p.refr_res[1] = v.y * t;
        p.refr_res[2] = v.z * t;
    } else {  // reflected_color = color_at(...) * reflective
        double t = p.refl;
        p.refl_res[0] = v.x * t;
        p.refl_res[1] = v.y * t;
        p.refl_res[2] = v.z * t;
    }
}

// canvas.rs:85-96: r = 0.0; r += p (dy outer, dx inner); r /= aa*aa
__global__ void __launch_bounds__(256) aa_kernel(const double* __restrict__ canvas, double* __restrict__ out,
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
    out[3 * i + 0] = r / total;
    out[3 * i + 1] = g / total;
    out[3 * i + 2] = b / total;
}

// Scene::is_shadowed for caller-given (point, light position) pairs
template <bool G>
__global__ void __launch_bounds__(256) shadow_query_kernel(DevScene S, const double* __restrict__ pts,
                                                           const double* __restrict__ lps, int64_t n,
                                                           int32_t* __restrict__ out, unsigned long long* counters) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool valid = i < n;
    Counters cnt = {0, 0, 0, 0, 0, 0, 0};
    V3 p = mk(0, 0, 0), l = mk(0, 0, 1);
    if (valid) {
        p = mk(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]);
        l = mk(lps[3 * i], lps[3 * i + 1], lps[3 * i + 2]);
    }
    bool sh = shadowed<G>(S, p, l, valid, cnt);
    if (valid) out[i] = sh ? 1 : 0;
    flush(cnt, counters);
}

// ------------------------------------------------------------------ host-side launchers
static inline unsigned blocks_for(int64_t n) { return (unsigned)((n + 255) / 256); }

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

template <bool G>
static void launch_level_t(const DevScene& S, const LevelArgs& A, int64_t n_sr_upper, hipStream_t st,
                           KernelProf* prof) {
    {
        Span s(prof, K_TRACE, st);
        hipLaunchKernelGGL(trace_kernel<G>, dim3(blocks_for(A.n)), dim3(256), 0, st, S, A);
    }
    if (S.has_transparent) {
        Span s(prof, K_N1N2, st);
        hipLaunchKernelGGL(n1n2_kernel<G>, dim3(blocks_for(A.n)), dim3(256), 0, st, S, A);
    }
    {
        Span s(prof, K_SHADE, st);
        hipLaunchKernelGGL(shade_kernel, dim3(blocks_for(A.n)), dim3(256), 0, st, S, A);
    }
    if (n_sr_upper > 0) {
        Span s(prof, K_SHADOW, st);
        hipLaunchKernelGGL(shadow_kernel<G>, dim3(blocks_for(n_sr_upper)), dim3(256), 0, st, S, A);
    }
    if (S.n_lights > 0) {
        Span s(prof, K_FINISH, st);
        hipLaunchKernelGGL(finish_kernel, dim3(blocks_for(A.n)), dim3(256), 0, st, S, A);
    }
}

hipError_t launch_level(const DevScene& S, const LevelArgs& A, int64_t n_sr_upper, hipStream_t st,
                        KernelProf* prof) {
    if (A.n <= 0) return hipSuccess;
    if (S.has_groups)
        launch_level_t<true>(S, A, n_sr_upper, st, prof);
    else
        launch_level_t<false>(S, A, n_sr_upper, st, prof);
    return hipGetLastError();
}

hipError_t launch_combine(const CombArgs& C, hipStream_t st, KernelProf* prof) {
    if (C.n <= 0) return hipSuccess;
    Span s(prof, K_COMBINE, st);
    hipLaunchKernelGGL(combine_kernel, dim3(blocks_for(C.n)), dim3(256), 0, st, C);
    return hipGetLastError();
}

hipError_t launch_aa(const double* canvas, double* out, int64_t width, int64_t rows, int32_t aa, hipStream_t st,
                     KernelProf* prof) {
    int64_t n = width * rows;
    if (n == 0) return hipSuccess;
    Span s(prof, K_AA, st);
    hipLaunchKernelGGL(aa_kernel, dim3(blocks_for(n)), dim3(256), 0, st, canvas, out, width, rows, aa);
    return hipGetLastError();
}

hipError_t launch_shadow_query(const DevScene& S, const double* pts, const double* lps, int64_t n, int32_t* out,
                               unsigned long long* counters, hipStream_t st) {
    if (n == 0) return hipSuccess;
    if (S.has_groups)
        hipLaunchKernelGGL(shadow_query_kernel<true>, dim3(blocks_for(n)), dim3(256), 0, st, S, pts, lps, n, out, counters);
    else
        hipLaunchKernelGGL(shadow_query_kernel<false>, dim3(blocks_for(n)), dim3(256), 0, st, S, pts, lps, n, out,
                           counters);
    return hipGetLastError();
}

}  // namespace rr
