// flatten.cpp — flattens the reference's object registry into the HBM layout.
//
// Order: Scene.ids (scene.rs:24-27) with every group's Group.child_ids inlined depth-first.
// That is the order in which Scene::intersect appends intersections before its stable sort
// (scene.rs:97-106; group.rs:80-91 sorts its children's hits first, which a stable sort of the
// concatenation reproduces), so "earliest node index" is the reference's tie-break.
#include "flatten.hpp"

#include <cmath>
#include <cstring>
#include <algorithm>
#include <functional>
#include <limits>

namespace rr {

namespace {

struct Box {
    Tup min, max;
};

void adjust_min_max(Box& b, double x, double y, double z) {  // object.rs:220-227 (f64::min/max == fmin/fmax)
    b.min = point(std::fmin(b.min.x, x), std::fmin(b.min.y, y), std::fmin(b.min.z, z));
    b.max = point(std::fmax(b.max.x, x), std::fmax(b.max.y, y), std::fmax(b.max.z, z));
}

Box apply_transform(const Box& b, const M4& m) {  // object.rs:257-278
    const Tup corners[8] = {point(b.min.x, b.min.y, b.min.z), point(b.min.x, b.min.y, b.max.z),
                            point(b.min.x, b.max.y, b.min.z), point(b.min.x, b.max.y, b.max.z),
                            point(b.max.x, b.min.y, b.min.z), point(b.max.x, b.min.y, b.max.z),
                            point(b.max.x, b.max.y, b.min.z), point(b.max.x, b.max.y, b.max.z)};
    const double inf = std::numeric_limits<double>::infinity();
    Box r{point(inf, inf, inf), point(-inf, -inf, -inf)};
    for (const Tup& c : corners) {
        Tup t = mul(m, c);
        adjust_min_max(r, t.x, t.y, t.z);
    }
    return r;
}

M4 load16(const double* p) {
    M4 m{};
    for (int i = 0; i < 16; ++i) m.m[i] = p[i];
    return m;
}

// inverse = diag(m0, m5, m10) + translation (the off-diagonal products are +-0 and drop out of the
// reference's sums unless the whole sum is zero)
bool is_diag12(const double* m) {
    return m[1] == 0.0 && m[2] == 0.0 && m[4] == 0.0 && m[6] == 0.0 && m[8] == 0.0 && m[9] == 0.0;
}
bool is_identity12(const double* m) {
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 4; ++c)
            if (m[r * 4 + c] != (r == c ? 1.0 : 0.0)) return false;
    return true;
}

// largest singular value of the upper 3x3 of m: sqrt of the largest eigenvalue of A^T A
// (cyclic Jacobi on the symmetric 3x3; converges to full double precision)
double sigma_max(const M4& m) {
    double A[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double s = 0.0;
            for (int k = 0; k < 3; ++k) s += m.get(k, i) * m.get(k, j);
            A[i][j] = s;
        }
    for (int sweep = 0; sweep < 50; ++sweep) {
        double off = std::fabs(A[0][1]) + std::fabs(A[0][2]) + std::fabs(A[1][2]);
        if (off <= 1e-300) break;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                if (A[p][q] == 0.0) continue;
                double theta = (A[q][q] - A[p][p]) / (2.0 * A[p][q]);
                double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
                double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < 3; ++k) {  // A = J^T A J
                    double akp = A[k][p], akq = A[k][q];
                    A[k][p] = c * akp - s * akq;
                    A[k][q] = s * akp + c * akq;
                }
                for (int k = 0; k < 3; ++k) {
                    double apk = A[p][k], aqk = A[q][k];
                    A[p][k] = c * apk - s * aqk;
                    A[q][k] = s * apk + c * aqk;
                }
            }
    }
    double mx = std::fmax(A[0][0], std::fmax(A[1][1], A[2][2]));
    return std::sqrt(std::fmax(mx, 0.0));
}

// bounding sphere (centre in parent space, radius) of node content with local bound (lc, lr)
DevCull make_cull(const M4& fwd, const double lc[3], double lr) {
    DevCull c{};
    const double inf = std::numeric_limits<double>::infinity();
    Tup w = mul(fwd, point(lc[0], lc[1], lc[2]));
    double r = lr * sigma_max(fwd);
    double scale = std::fabs(w.x) + std::fabs(w.y) + std::fabs(w.z) + r;
    // relative 1e-3 + absolute terms: covers the f32 rounding of the centre / radius, the gap
    // between the computed inverse and the exact one, and the f64 test's rounding near tangency
    r = r * 1.001 + 1e-6 * (1.0 + scale);
    if (!std::isfinite(w.x) || !std::isfinite(w.y) || !std::isfinite(w.z) || !std::isfinite(r) || lr == inf) {
        c.c[0] = c.c[1] = c.c[2] = 0.0f;
        c.r = std::numeric_limits<float>::infinity();
        return c;
    }
    c.c[0] = (float)w.x;
    c.c[1] = (float)w.y;
    c.c[2] = (float)w.z;
    c.r = (float)r * 1.0001f;
    return c;
}

uint32_t expand10(uint32_t v) {  // 10 bits -> every third bit
    v &= 0x3ffu;
    v = (v | (v << 16)) & 0x030000FFu;
    v = (v | (v << 8)) & 0x0300F00Fu;
    v = (v | (v << 4)) & 0x030C30C3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

// Stores every sibling list in Morton order of its members' cull centres (unbounded members
// last), keeping each subtree contiguous, and records each node's reference DFS position in
// `rank`.  The kernels break ties on (t, rank), so results do not depend on the storage order;
// the spatial order makes runs of consecutive nodes compact, which the chunk culling needs.
void reorder_spatial(HostScene& hs) {
    const int N = (int)hs.nodes.size();
    if (N == 0) return;
    std::vector<std::vector<int>> kids((size_t)N);
    std::vector<int> top;
    for (int i = 0; i < N; ++i) (hs.nodes[i].parent < 0 ? top : kids[hs.nodes[i].parent]).push_back(i);
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
    for (const DevCull& c : hs.culls)
        if (std::isfinite(c.r))
            for (int k = 0; k < 3; ++k) {
                lo[k] = std::fmin(lo[k], c.c[k]);
                hi[k] = std::fmax(hi[k], c.c[k]);
            }
    std::vector<uint32_t> key((size_t)N, 0xffffffffu);
    for (int i = 0; i < N; ++i) {
        const DevCull& c = hs.culls[i];
        if (!std::isfinite(c.r)) continue;
        uint32_t m = 0;
        for (int k = 0; k < 3; ++k) {
            double ext = hi[k] - lo[k];
            double u = ext > 0 ? (c.c[k] - lo[k]) / ext : 0.0;
            uint32_t q = (uint32_t)std::fmin(1023.0, std::fmax(0.0, std::floor(u * 1024.0)));
            m |= expand10(q) << k;
        }
        key[i] = m;
    }
    auto by_key = [&](int a, int b) { return key[a] < key[b]; };
    // Sibling lists of more than 64 bounded leaves (meshes, sphere fields) are ordered by a recursive
    // median split instead: along the longest axis of the members' centres, at a multiple of 64 near the
    // middle, down to buckets of <= 64 — each bucket becomes one chunk (chunk_break), and a bucket of nearby
    // members has a small bounding sphere.  Morton order sliced every 64 nodes can straddle a cell boundary
    // and join two distant patches in one chunk.
    std::vector<char> bucket_start((size_t)N, 0);
    // bucket size: 64 (one chunk) in general; 16 for scenes that take the general (G = 2) kernels, whose
    // walks reload every candidate's cull from memory (no cross-lane reads): measured example1 32.2 -> 28.9 ms,
    // while the cross-lane walks of the G = 0 / 1 kernels lose with smaller buckets (C4 0.78 -> 0.88 ms at 16)
    const size_t BK = (hs.has_csg || hs.has_quad) ? 16 : 64;
    std::function<void(std::vector<int>&, size_t, size_t)> kd = [&](std::vector<int>& v, size_t b, size_t e) {
        if (e - b <= BK) {
            std::stable_sort(v.begin() + b, v.begin() + e, by_key);
            bucket_start[v[b]] = 1;
            return;
        }
        double mn[3] = {1e300, 1e300, 1e300}, mx[3] = {-1e300, -1e300, -1e300};
        for (size_t q = b; q < e; ++q)
            for (int k = 0; k < 3; ++k) {
                mn[k] = std::fmin(mn[k], hs.culls[v[q]].c[k]);
                mx[k] = std::fmax(mx[k], hs.culls[v[q]].c[k]);
            }
        int ax = 0;
        for (int k = 1; k < 3; ++k)
            if (mx[k] - mn[k] > mx[ax] - mn[ax]) ax = k;
        std::stable_sort(v.begin() + b, v.begin() + e, [&](int a, int c) {
            const float fa = hs.culls[a].c[ax], fc = hs.culls[c].c[ax];
            return fa < fc || (fa == fc && key[a] < key[c]);
        });
        const size_t n = e - b, left = BK * ((n + 2 * BK - 1) / (2 * BK));  // a multiple of BK, about half
        kd(v, b, b + left);
        kd(v, b + left, e);
    };
    auto order = [&](std::vector<int>& v) {
        size_t nb = 0;
        bool leaves = true;
        for (int i : v) {
            if (std::isfinite(hs.culls[i].r)) ++nb;
            leaves = leaves && !is_container(hs.nodes[i].kind);
        }
        std::stable_sort(v.begin(), v.end(), by_key);  // bounded first (unbounded keys are all-ones)
        if (leaves && nb > 64) kd(v, 0, nb);
    };
    order(top);
    // a CSG concatenates left then right and sorts stably (csg.rs:105-113): its subtree keeps the
    // reference order, so the kernel's in-subtree evaluation order is the reference's
    std::vector<char> in_csg((size_t)N, 0);
    for (int i = 0; i < N; ++i)
        for (int a = hs.nodes[i].parent; a >= 0; a = hs.nodes[a].parent)
            if (hs.nodes[a].kind == RR_CSG) {
                in_csg[i] = 1;
                break;
            }
    for (int i = 0; i < N; ++i) {
        if (in_csg[i]) hs.nodes[i].flags |= NF_IN_CSG;
        if (hs.nodes[i].kind != RR_CSG && !in_csg[i]) order(kids[i]);
    }
    std::vector<int> perm;
    perm.reserve((size_t)N);
    std::function<void(int)> emit = [&](int i) {
        perm.push_back(i);
        for (int c : kids[i]) emit(c);
    };
    for (int t : top) emit(t);
    std::vector<int> newidx((size_t)N);
    for (int k = 0; k < N; ++k) newidx[perm[k]] = k;
    std::vector<DevNode> nodes((size_t)N);
    std::vector<DevCull> culls((size_t)N);
    for (int k = 0; k < N; ++k) {
        const int o = perm[k];
        DevNode nd = hs.nodes[o];
        nd.rank = o;
        nd.parent = nd.parent >= 0 ? newidx[nd.parent] : -1;
        nd.skip = k + (hs.nodes[o].skip - o);  // subtree sizes are unchanged
        nodes[k] = nd;
        culls[k] = hs.culls[o];
    }
    for (DevGroup& g : hs.groups)
        for (int j = 0; j < RR_MAX_GROUP_DEPTH; ++j)
            if (g.anc[j] >= 0) g.anc[j] = newidx[g.anc[j]];
    for (int32_t& v : hs.node_of_object)
        if (v >= 0) v = newidx[v];
    hs.nodes.swap(nodes);
    hs.culls.swap(culls);
    hs.chunk_break.assign((size_t)N, 0);
    for (int k = 0; k < N; ++k) hs.chunk_break[k] = bucket_start[perm[k]];
}

// Runs of up to 64 consecutive nodes with a bounding sphere of their culls; unbounded nodes
// (planes, unbounded groups) get a chunk of their own.
// NF_OWN_SAFE (device_core.inc own_node): spheres and planes outside any CSG whose world-to-object transform A
// (ancestors' inverses and the node's, as the walks apply them; linear part A_l, translation A_t) keeps every rounding
// the skip's argument meets far inside its margin (factor 1e3).  The margin: an over point lies EPS = 1e-5 beyond the
// tangent plane at the hit point, at least EPS sigma_min(A_l) in object space, sigma_min(A_l) >= 1 / |F_l|_F (F the
// forward transform).  The roundings against it:
//   * the object-space shadow origin, direction and quadratic: a few ulps of |A_l| |over| + |A_t|, for |over|_inf <= W
//     = 1e5 (own_node checks W at run time); |A_l| <= 1e8 keeps a wrong-side direction component below the plane test's
//     EPS;
//   * the hit point itself: sphere.rs's roots come from b^2 - 4ac, which cancels when the incoming ray's object-space
//     origin q0 is far from the unit sphere, and put the point up to ~4 eps |q0|^2 off the surface along the normal
//     (a camera 2e4 units from a 3e-3 sphere: 2e-3 object units, inside the margin — fuzz seed 2).  |q0|_2 <=
//     sqrt(3) (1.01 + |A_l|_inf T) with T = t |d|_inf of the hit, so the node stores the largest allowed T (float bits
//     in DevNode.aux, unused by spheres and planes) and prepare() compares the hit's T with it.
// Infinity norms throughout.
static void mark_own_safe(HostScene& hs) {
    const double eps = 0x1p-52, W = 1e5, EPS = 1e-5, SAFETY = 1e3;
    for (size_t ni = 0; ni < hs.nodes.size(); ++ni) {
        DevNode& nd = hs.nodes[ni];
        if ((nd.kind != RR_SPHERE && nd.kind != RR_PLANE) || (nd.flags & NF_IN_CSG)) continue;
        M4 fwd = identity(), inv = identity();
        for (int a = (int)ni; a >= 0; a = hs.nodes[a].parent) {
            M4 nfull = identity();
            for (int e = 0; e < 12; ++e) nfull.m[e] = hs.nodes[a].inv[e];
            inv = multiply(inv, nfull);  // the node's inverse first, the root's last: A = inv_node ... inv_root
            fwd = multiply(inverse(nfull), fwd);
        }
        double al = 0.0, at = 0.0, ff = 0.0;
        bool finite = true;
        for (int r = 0; r < 3; ++r) {
            double row = 0.0;
            for (int c = 0; c < 3; ++c) {
                row += std::fabs(inv.m[4 * r + c]);
                ff += fwd.m[4 * r + c] * fwd.m[4 * r + c];
            }
            al = std::fmax(al, row);
            at = std::fmax(at, std::fabs(inv.m[4 * r + 3]));
            for (int c = 0; c < 4; ++c) finite = finite && std::isfinite(inv.m[4 * r + c]) && std::isfinite(fwd.m[4 * r + c]);
        }
        const double fn = std::sqrt(ff);
        if (!finite || !(fn > 0.0) || !(al <= 1e8) || !(al > 0.0)) continue;
        const double sigma_min = 1.0 / fn, margin = EPS * sigma_min;
        if (!(SAFETY * 4.0 * eps * (al * (2.0 * W + 1.0) + at) <= margin)) continue;
        // 4 eps * 3 (1.01 + al T)^2 * SAFETY <= margin
        const double tlim = (std::sqrt(margin / (12.0 * eps * SAFETY)) - 1.01) / al;
        if (!(tlim > 0.0)) continue;
        const float tl = (float)(tlim * (1.0 - 1e-6));
        int32_t bits;
        std::memcpy(&bits, &tl, sizeof bits);
        nd.aux = bits;
        nd.flags |= NF_OWN_SAFE;
    }
}

// Inner balls (render_levels.inc area_in_umbra): for a sphere outside any CSG, a ball that lies inside the set its exact
// test reports — the unit sphere under the world-to-object transform A the walks apply (A_l x + A_t, every ancestor's
// inverse and the node's): centre C = A^-1 (0, 0, 0) = the forward transform of the origin, radius 1 / sigma_max(A_l)
// (|A_l (x - C)| <= sigma_max |x - C|), shrunk by 1e-6 relative and by the f32 rounding of the stored centre.  Other
// nodes get radius 0 (none).
static void mark_inner_balls(HostScene& hs) {
    hs.inner.assign(hs.nodes.size(), DevCull{{0.0f, 0.0f, 0.0f}, 0.0f});
    for (size_t ni = 0; ni < hs.nodes.size(); ++ni) {
        const DevNode& nd = hs.nodes[ni];
        if (nd.kind != RR_SPHERE || (nd.flags & NF_IN_CSG)) continue;
        M4 inv = identity();
        for (int a = (int)ni; a >= 0; a = hs.nodes[a].parent) {
            M4 nfull = identity();
            for (int e = 0; e < 12; ++e) nfull.m[e] = hs.nodes[a].inv[e];
            inv = multiply(inv, nfull);  // the node's inverse first, the root's last
        }
        const M4 fwd = inverse(inv);
        const Tup c = mul(fwd, point(0.0, 0.0, 0.0));
        const double smax = sigma_max(inv);
        // how far the computed centre is from the object-space origin (the inverse's rounding): shrinks the ball
        const Tup oc = mul(inv, c);
        const double res = std::sqrt(oc.x * oc.x + oc.y * oc.y + oc.z * oc.z);
        if (!std::isfinite(c.x) || !std::isfinite(c.y) || !std::isfinite(c.z) || !(smax > 0.0) || !std::isfinite(smax) ||
            !(res < 0.5))
            continue;
        const float cf[3] = {(float)c.x, (float)c.y, (float)c.z};
        const double shift = std::sqrt(((double)cf[0] - c.x) * ((double)cf[0] - c.x) + ((double)cf[1] - c.y) * ((double)cf[1] - c.y) +
                                       ((double)cf[2] - c.z) * ((double)cf[2] - c.z));
        const double scale = std::fabs(c.x) + std::fabs(c.y) + std::fabs(c.z);
        const double r = ((1.0 - res) / smax) * (1.0 - 1e-6) - 2.0 * shift - 1e-9 * (scale + 1.0 / smax);
        if (!(r > 0.0)) continue;
        DevCull& b = hs.inner[ni];
        for (int k = 0; k < 3; ++k) b.c[k] = cf[k];
        b.r = std::nextafter((float)r, 0.0f);  // rounded down
    }
}

void build_chunks(HostScene& hs) {
    hs.chunks.clear();
    const int N = (int)hs.nodes.size();
    for (int i = 0; i < N;) {
        DevChunk ch{};
        ch.start = i;
        if (!std::isfinite(hs.culls[i].r)) {
            ch.count = 1;
            ch.cull = hs.culls[i];
            ++i;
            hs.chunks.push_back(ch);
            continue;
        }
        double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
        // a chunk ends at 64 nodes, before an unbounded node, at a spatial bucket's start, and around a
        // container (a group's cull spans its whole subtree: in a chunk of its own it does not widen its
        // children's chunks)
        auto brk = [&](int m) {
            return (!hs.chunk_break.empty() && hs.chunk_break[m]) || is_container(hs.nodes[m].kind) ||
                   is_container(hs.nodes[m - 1].kind);
        };
        int j = i;
        for (; j < N && j - i < 64 && std::isfinite(hs.culls[j].r) && (j == i || !brk(j)); ++j)
            for (int k = 0; k < 3; ++k) {
                lo[k] = std::fmin(lo[k], (double)hs.culls[j].c[k] - hs.culls[j].r);
                hi[k] = std::fmax(hi[k], (double)hs.culls[j].c[k] + hs.culls[j].r);
            }
        ch.count = j - i;
        float cf[3];
        for (int k = 0; k < 3; ++k) cf[k] = (float)(0.5 * (lo[k] + hi[k]));
        double r = 0.0;
        for (int m = i; m < j; ++m) {
            const DevCull& c = hs.culls[m];
            double dx = (double)c.c[0] - cf[0], dy = (double)c.c[1] - cf[1], dz = (double)c.c[2] - cf[2];
            r = std::fmax(r, std::sqrt(dx * dx + dy * dy + dz * dz) + (double)c.r);
        }
        for (int k = 0; k < 3; ++k) ch.cull.c[k] = cf[k];
        ch.cull.r = (float)(r * (1.0 + 1e-6)) * 1.000001f;
        if (!std::isfinite(ch.cull.r)) ch.cull.r = std::numeric_limits<float>::infinity();
        hs.chunks.push_back(ch);
        i = j;
    }
}

}  // namespace

bool inverse_3x4(const M4& transform, const double* given, double out12[12], M4* full, std::string& err) {
    M4 inv = given ? load16(given) : inverse(transform);
    if (!(inv.get(3, 0) == 0.0 && inv.get(3, 1) == 0.0 && inv.get(3, 2) == 0.0 && inv.get(3, 3) == 1.0)) {
        err = "inverse transform is not affine (row 3 != 0,0,0,1)";
        return false;
    }
    for (int i = 0; i < 12; ++i) out12[i] = inv.m[i];
    if (full) *full = inv;
    return true;
}

int flatten_scene(const rr_scene_desc& d, HostScene& out, std::string& err) {
    out = HostScene();
    const int n = d.n_objects;
    if (n < 0 || (n > 0 && (!d.kind || !d.parent || !d.transform || !d.material))) {
        err = "scene descriptor: missing per-object arrays";
        return RR_E_ARG;
    }
    if (d.n_top < 0 || (d.n_top > 0 && !d.top)) {
        err = "scene descriptor: missing top-level id list";
        return RR_E_ARG;
    }
    // materials
    for (int i = 0; i < d.n_materials; ++i) {
        DevMaterial m{};
        const double* p = d.mat + 7 * (size_t)i;
        m.ambient = p[0];
        m.diffuse = p[1];
        m.specular = p[2];
        m.shininess = p[3];
        m.reflective = p[4];
        m.transparency = p[5];
        m.refractive_index = p[6];
        m.pattern = d.mat_pattern ? d.mat_pattern[i] : -1;
        if (m.pattern < -1 || m.pattern >= d.n_patterns) {
            err = "material references an unknown pattern";
            return RR_E_ARG;
        }
        out.mats.push_back(m);
    }
    // patterns
    for (int i = 0; i < d.n_patterns; ++i) {
        DevPattern p{};
        p.kind = d.pat_kind[i];
        p.a = d.pat_a ? d.pat_a[i] : -1;
        p.b = d.pat_b ? d.pat_b[i] : -1;
        for (int c = 0; c < 3; ++c) p.color[c] = d.pat_color ? d.pat_color[3 * (size_t)i + c] : 0.0;
        p.scale = d.pat_scale ? d.pat_scale[i] : 0.5;
        p.octaves = d.pat_octaves ? d.pat_octaves[i] : 1;
        p.persistence = d.pat_persistence ? d.pat_persistence[i] : 1.0;
        M4 t = d.pat_transform ? load16(d.pat_transform + 16 * (size_t)i) : identity();
        if (!inverse_3x4(t, nullptr, p.inv, nullptr, err)) return RR_E_NONAFFINE;
        p.flags = is_identity12(p.inv) ? NF_IDENT : 0;
        if (p.kind < RR_PAT_TEST || p.kind > RR_PAT_TEXTURE) {
            err = "unknown pattern kind";
            return RR_E_ARG;
        }
        if (p.kind == RR_PAT_TEXTURE) {
            if (p.a < 0 || p.a >= d.n_textures) {
                err = "texture pattern references an unknown texture";
                return RR_E_ARG;
            }
            out.complex_patterns = 1;
            out.pats.push_back(p);
            continue;
        }
        if ((p.kind == RR_PAT_PERTURBED || p.kind == RR_PAT_NOISE) && (p.octaves < 0 || p.octaves > RR_MAX_OCTAVES)) {
            err = "pattern octaves outside [0, RR_MAX_OCTAVES]";
            return RR_E_LIMIT;
        }
        bool leaf = p.kind == RR_PAT_TEST || p.kind == RR_PAT_SOLID;
        bool unary = p.kind == RR_PAT_PERTURBED;
        if (!leaf && (p.a < 0 || p.a >= d.n_patterns || (!unary && (p.b < 0 || p.b >= d.n_patterns)))) {
            err = "pattern child index out of range";
            return RR_E_ARG;
        }
        if (p.kind == RR_PAT_GRADIENT || p.kind == RR_PAT_BLEND || p.kind >= RR_PAT_PERTURBED) out.complex_patterns = 1;
        out.pats.push_back(p);
    }
    // inline Solid leaves: a material whose root is Solid, a select pattern's Solid children
    for (DevPattern& p : out.pats) {
        if (p.kind != RR_PAT_STRIPE && p.kind != RR_PAT_RING && p.kind != RR_PAT_CHECKER) continue;
        if (out.pats[p.a].kind == RR_PAT_SOLID) {
            p.flags |= PF_A_SOLID;
            for (int c = 0; c < 3; ++c) p.ca[c] = out.pats[p.a].color[c];
        }
        if (out.pats[p.b].kind == RR_PAT_SOLID) {
            p.flags |= PF_B_SOLID;
            for (int c = 0; c < 3; ++c) p.cb[c] = out.pats[p.b].color[c];
        }
    }
    for (DevMaterial& m : out.mats) {
        const bool white = m.pattern < 0;  // Material::default: solid white (material.rs:49)
        if (white || out.pats[m.pattern].kind == RR_PAT_SOLID) {
            m.root = 1;
            for (int c = 0; c < 3; ++c) m.color[c] = white ? 1.0 : out.pats[m.pattern].color[c];
        }
    }
    // pattern nesting depth (the kernel evaluates trees with a bounded explicit stack)
    std::function<int(int, int)> pdepth = [&](int i, int lvl) -> int {
        if (lvl > RR_MAX_PATTERN_DEPTH) return lvl;
        const DevPattern& p = out.pats[i];
        if (p.kind == RR_PAT_TEST || p.kind == RR_PAT_SOLID || p.kind == RR_PAT_TEXTURE) return lvl;
        if (p.kind == RR_PAT_PERTURBED) return pdepth(p.a, lvl + 1);
        return std::max(pdepth(p.a, lvl + 1), pdepth(p.b, lvl + 1));
    };
    for (int i = 0; i < d.n_patterns; ++i)
        if (pdepth(i, 1) > RR_MAX_PATTERN_DEPTH) {
            err = "pattern nesting exceeds RR_MAX_PATTERN_DEPTH";
            return RR_E_LIMIT;
        }
    // textures
    if (d.n_textures < 0 || (d.n_textures > 0 && (!d.tex_size || !d.texels))) {
        err = "texture arrays missing";
        return RR_E_ARG;
    }
    for (int i = 0; i < d.n_textures; ++i) {
        int32_t w = d.tex_size[2 * i], h = d.tex_size[2 * i + 1];
        if (w < 1 || h < 1) {
            err = "texture with an empty image";
            return RR_E_ARG;
        }
        DevTexture t{};
        t.offset = out.texels.size();
        t.width = (uint32_t)w;
        t.height = (uint32_t)h;
        const uint8_t* px = d.texels + 4 * t.offset;
        for (size_t k = 0; k < (size_t)w * (size_t)h; ++k)
            out.texels.push_back((uint32_t)px[4 * k] | ((uint32_t)px[4 * k + 1] << 8) | ((uint32_t)px[4 * k + 2] << 16) |
                                 ((uint32_t)px[4 * k + 3] << 24));
        out.textures.push_back(t);
    }
    // lights
    for (int i = 0; i < d.n_lights; ++i) {
        DevLight l{};
        const double* p = d.light + 15 * (size_t)i;
        for (int c = 0; c < 3; ++c) {
            l.position[c] = p[c];
            l.intensity[c] = p[3 + c];
            l.corner[c] = p[6 + c];
            l.u[c] = p[9 + c];
            l.v[c] = p[12 + c];
        }
        l.kind = d.light_kind[i];
        l.level = d.light_level ? d.light_level[i] : 0;
        if (l.kind == RR_LIGHT_AREA && l.level <= 0) {
            err = "area light with level <= 0";
            return RR_E_SCENE;
        }
        if (l.kind == RR_LIGHT_AREA && l.level > RR_MAX_AREA_LEVEL) {  // level^2 cell samples per shading event
            err = "area light level exceeds RR_MAX_AREA_LEVEL";
            return RR_E_LIMIT;
        }
        out.lights.push_back(l);
    }

    // objects: per-object inverses, triangle data, group AABBs (cached like group.rs:54-67)
    std::vector<M4> fwd((size_t)n);
    std::vector<double> inv12((size_t)n * 12);
    std::vector<int> tri_index((size_t)n, -1);
    for (int i = 0; i < n; ++i) {
        fwd[i] = load16(d.transform + 16 * (size_t)i);
        if (!inverse_3x4(fwd[i], d.inverse ? d.inverse + 16 * (size_t)i : nullptr, &inv12[12 * (size_t)i], nullptr,
                         err)) {
            err = "object " + std::to_string(i) + ": " + err;
            return RR_E_NONAFFINE;
        }
        int k = d.kind[i];
        if (k < RR_SPHERE || k > RR_TORUS) {
            err = "unknown object kind";
            return RR_E_ARG;
        }
        if (k == RR_CSG && (d.child_count ? d.child_count[i] : 0) != 2) {
            err = "CSG object " + std::to_string(i) + " needs exactly a left and a right child";
            return RR_E_SCENE;  // csg.rs: get_object(usize::MAX) panics
        }
        if (k == RR_TORUS) {  // torus.rs:23-31: minor radius (major radius 1)
            if (!d.shape) {
                err = "torus without its minor radius (rr_scene_desc.shape)";
                return RR_E_ARG;
            }
            DevShape s{};
            s.minimum = d.shape[3 * (size_t)i];
            s.maximum = 0.0;
            s.closed = 0;
            tri_index[i] = (int)out.shapes.size();
            out.shapes.push_back(s);
            out.has_quad = 1;
        }
        if (k == RR_CYLINDER || k == RR_CONE) {  // cylinder.rs:29-37, cone.rs:30-38
            DevShape s{};
            s.minimum = d.shape ? d.shape[3 * (size_t)i] : -std::numeric_limits<double>::infinity();
            s.maximum = d.shape ? d.shape[3 * (size_t)i + 1] : std::numeric_limits<double>::infinity();
            s.closed = d.shape ? (d.shape[3 * (size_t)i + 2] != 0.0) : 0;
            tri_index[i] = (int)out.shapes.size();
            out.shapes.push_back(s);
            out.has_quad = 1;
        }
        if (k == RR_CUBE) out.has_quad = 1;  // handled by the general kernel variant
        if (!is_container(k) && (d.material[i] < 0 || d.material[i] >= d.n_materials)) {
            err = "object " + std::to_string(i) + " has no valid material";
            return RR_E_ARG;
        }
        if (k == RR_TRIANGLE || k == RR_SMOOTH_TRIANGLE) {
            if (!d.tri) {
                err = "triangle without vertex data";
                return RR_E_ARG;
            }
            const double* p = d.tri + 18 * (size_t)i;
            Tup p1 = point(p[0], p[1], p[2]), p2 = point(p[3], p[4], p[5]), p3 = point(p[6], p[7], p[8]);
            Tup e1 = p2 - p1, e2 = p3 - p1;  // triangle.rs:52-56
            Tup nn = normalize(cross(e2, e1));
            DevTri t{};
            const double pp[3] = {p1.x, p1.y, p1.z}, a1[3] = {e1.x, e1.y, e1.z}, a2[3] = {e2.x, e2.y, e2.z},
                         no[3] = {nn.x, nn.y, nn.z};
            for (int c = 0; c < 3; ++c) {
                t.p1[c] = pp[c];
                t.e1[c] = a1[c];
                t.e2[c] = a2[c];
                t.normal[c] = no[c];
                t.n1[c] = p[9 + c];
                t.n2[c] = p[12 + c];
                t.n3[c] = p[15 + c];
            }
            t.smooth = (k == RR_SMOOTH_TRIANGLE);
            tri_index[i] = (int)out.tris.size();
            out.tris.push_back(t);
        }
    }
    const double inf = std::numeric_limits<double>::infinity();
    std::vector<int> aabb_state((size_t)n, 0);
    std::vector<Box> aabb((size_t)n);
    std::function<Box(int, int)> get_aabb = [&](int id, int lvl) -> Box {
        int k = d.kind[id];
        if (k == RR_SPHERE || k == RR_CUBE) return {point(-1, -1, -1), point(1, 1, 1)};  // sphere.rs / cube.rs
        if (k == RR_PLANE) return {point(-inf, 0.0, -inf), point(inf, 0.0, inf)};  // plane.rs get_aabb
        if (k == RR_CYLINDER || k == RR_CONE) {
            const DevShape& s = out.shapes[tri_index[id]];
            if (k == RR_CYLINDER) return {point(-1, s.minimum, -1), point(1, s.maximum, 1)};  // cylinder.rs
            double limit = std::fmax(std::fabs(s.minimum), std::fabs(s.maximum));             // cone.rs:221-226
            return {point(-limit, s.minimum, -limit), point(limit, s.maximum, limit)};
        }
        if (k == RR_TORUS) {  // torus.rs get_aabb
            const double r = out.shapes[tri_index[id]].minimum;
            return {point(-1.0 - r, -1.0 - r, -r), point(1.0 + r, 1.0 + r, r)};
        }
        if (!is_container(k)) {                                                    // triangle.rs get_aabb
            const double* p = d.tri + 18 * (size_t)id;
            return {point(std::fmin(p[0], std::fmin(p[3], p[6])), std::fmin(p[1], std::fmin(p[4], p[7])),
                          std::fmin(p[2], std::fmin(p[5], p[8]))),
                    point(std::fmax(p[0], std::fmax(p[3], p[6])), std::fmax(p[1], std::fmax(p[4], p[7])),
                          std::fmax(p[2], std::fmax(p[5], p[8])))};
        }
        if (aabb_state[id] == 2) return aabb[id];
        Box b{point(inf, inf, inf), point(-inf, -inf, -inf)};  // group.rs:128-149 (csg.rs: left then right)
        int cs = d.child_start ? d.child_start[id] : 0, cc = d.child_count ? d.child_count[id] : 0;
        for (int j = 0; j < cc && lvl < 64; ++j) {
            int c = d.children[cs + j];
            Box cb = apply_transform(get_aabb(c, lvl + 1), fwd[c]);
            adjust_min_max(b, cb.min.x, cb.min.y, cb.min.z);  // AABB::adjust_aabb (object.rs:237-240)
            adjust_min_max(b, cb.max.x, cb.max.y, cb.max.z);
        }
        aabb[id] = b;
        aabb_state[id] = 2;
        return b;
    };

    // depth-first flattening
    out.node_of_object.assign((size_t)n, -1);
    std::vector<int32_t> anc;
    std::function<int(int, int)> visit = [&](int id, int parent_node) -> int {
        if (id < 0 || id >= n) {
            err = "object id out of range";
            return RR_E_ARG;
        }
        if (out.node_of_object[id] != -1) {
            err = "object " + std::to_string(id) + " appears twice in the scene tree";
            return RR_E_ARG;
        }
        int idx = (int)out.nodes.size();
        out.node_of_object[id] = idx;
        DevNode nd{};
        std::memcpy(nd.inv, &inv12[12 * (size_t)id], sizeof(nd.inv));
        nd.kind = d.kind[id];
        nd.flags = is_identity12(nd.inv) ? NF_IDENT : is_diag12(nd.inv) ? NF_DIAG : 0;
        nd.material = is_container(nd.kind) ? -1 : d.material[id];
        nd.parent = parent_node;
        nd.depth = (int32_t)anc.size();
        nd.aux = tri_index[id];
        if (parent_node >= 0 && d.parent[id] >= 0 && out.node_of_object[d.parent[id]] != parent_node) {
            err = "object parent link disagrees with the group child list";
            return RR_E_ARG;
        }
        out.nodes.push_back(nd);
        if (is_container(nd.kind)) {
            if ((int)anc.size() >= RR_MAX_GROUP_DEPTH) {
                err = "group/CSG nesting exceeds RR_MAX_GROUP_DEPTH";
                return RR_E_LIMIT;
            }
            anc.push_back(idx);
            DevGroup g{};
            Box b = get_aabb(id, 0);
            g.aabb[0] = b.min.x;
            g.aabb[1] = b.min.y;
            g.aabb[2] = b.min.z;
            g.aabb[3] = b.max.x;
            g.aabb[4] = b.max.y;
            g.aabb[5] = b.max.z;
            for (int j = 0; j < RR_MAX_GROUP_DEPTH; ++j) g.anc[j] = j < (int)anc.size() ? anc[j] : -1;
            g.depth = (int32_t)anc.size();
            g.csg_op = nd.kind == RR_CSG ? (d.csg_op ? d.csg_op[id] : RR_CSG_UNION) : 0;
            if (nd.kind == RR_CSG) {
                out.has_csg = 1;
                if (g.csg_op < RR_CSG_UNION || g.csg_op > RR_CSG_DIFFERENCE) {
                    err = "unknown CSG operation";
                    return RR_E_ARG;
                }
            }
            out.nodes[idx].aux = (int)out.groups.size();
            out.groups.push_back(g);
            int cs = d.child_start ? d.child_start[id] : 0, cc = d.child_count ? d.child_count[id] : 0;
            if (cc > 0 && !d.children) {
                err = "group without children array";
                return RR_E_ARG;
            }
            for (int j = 0; j < cc; ++j) {
                int rc = visit(d.children[cs + j], idx);
                if (rc != RR_OK) return rc;
            }
            anc.pop_back();
        } else if (parent_node < 0) {
            out.n_top_leaves++;
        }
        out.nodes[idx].skip = (int)out.nodes.size();
        return RR_OK;
    };
    for (int i = 0; i < d.n_top; ++i) {
        int rc = visit(d.top[i], -1);
        if (rc != RR_OK) return rc;
    }
    for (const DevNode& nd : out.nodes) {
        if (is_container(nd.kind)) continue;
        const DevMaterial& m = out.mats[nd.material];
        if (m.transparency != 0.0) out.has_transparent = 1;
        if (m.transparency != 0.0 || m.reflective != 0.0) out.has_secondary = 1;  // scene.rs:281-336
        // children one shade_hit can queue: reflected (reflective != 0) + refracted (transparency != 0)
        const int32_t kids = (m.reflective != 0.0 ? 1 : 0) + (m.transparency != 0.0 ? 1 : 0);
        out.max_children = std::max(out.max_children, kids);
    }
    // culling bounds (parent space) per node
    std::vector<int> obj_of_node(out.nodes.size(), -1);
    for (int i = 0; i < n; ++i)
        if (out.node_of_object[i] >= 0) obj_of_node[out.node_of_object[i]] = i;
    out.culls.resize(out.nodes.size());
    for (size_t ni = 0; ni < out.nodes.size(); ++ni) {
        const int id = obj_of_node[ni];
        const DevNode& nd = out.nodes[ni];
        double lc[3] = {0.0, 0.0, 0.0};
        double lr = inf;
        if (nd.kind == RR_SPHERE) {
            lr = 1.0;
        } else if (nd.kind == RR_TRIANGLE || nd.kind == RR_SMOOTH_TRIANGLE) {
            const double* p = d.tri + 18 * (size_t)id;
            for (int k = 0; k < 3; ++k) lc[k] = (p[k] + p[3 + k] + p[6 + k]) / 3.0;
            lr = 0.0;
            for (int v = 0; v < 3; ++v) {
                double dx = p[3 * v] - lc[0], dy = p[3 * v + 1] - lc[1], dz = p[3 * v + 2] - lc[2];
                lr = std::fmax(lr, std::sqrt(dx * dx + dy * dy + dz * dz));
            }
            lr = lr * 1.001 + 1e-9;
        } else if (nd.kind != RR_PLANE) {  // cube, cylinder, cone: their AABB; group, CSG: the cached AABB
            double bb[6];
            if (is_container(nd.kind)) {
                for (int k = 0; k < 6; ++k) bb[k] = out.groups[nd.aux].aabb[k];
            } else {
                Box bx = get_aabb(id, 0);
                const double v6[6] = {bx.min.x, bx.min.y, bx.min.z, bx.max.x, bx.max.y, bx.max.z};
                for (int k = 0; k < 6; ++k) bb[k] = v6[k];
            }
            const double* b = bb;
            bool finite = true;
            for (int k = 0; k < 6; ++k) finite = finite && std::isfinite(b[k]);
            if (finite && b[0] <= b[3] && b[1] <= b[4] && b[2] <= b[5]) {
                for (int k = 0; k < 3; ++k) lc[k] = 0.5 * (b[k] + b[3 + k]);
                double hx = 0.5 * (b[3] - b[0]), hy = 0.5 * (b[4] - b[1]), hz = 0.5 * (b[5] - b[2]);
                lr = std::sqrt(hx * hx + hy * hy + hz * hz) * 1.001 + 1e-9;
            } else if (finite) {
                lr = 0.0;  // empty group: nothing inside can be hit; a tiny sphere is still conservative
            }
        }
        // world-space bound of the set the kernel's test accepts: the kernel applies the ancestors'
        // and the node's stored inverses, so map back through their inverses (root-first product)
        M4 world = identity();
        std::vector<int> chain;
        for (int a = (int)ni; a >= 0; a = out.nodes[a].parent) chain.push_back(a);
        for (int k = (int)chain.size() - 1; k >= 0; --k) {
            M4 nfull = identity();
            for (int e = 0; e < 12; ++e) nfull.m[e] = out.nodes[chain[k]].inv[e];
            world = multiply(world, inverse(nfull));
        }
        out.culls[ni] = make_cull(world, lc, lr);
    }
    // CSG filtering needs left.includes(leaf) for every CSG above a leaf (csg.rs:86-88): leaves compare
    // ids, groups ask all children (group.rs:151-159), a CSG only its two direct children (csg.rs:160-162)
    if (out.has_csg) {
        const int N = (int)out.nodes.size();
        std::vector<std::vector<int>> kids((size_t)N);
        for (int i = 0; i < N; ++i)
            if (out.nodes[i].parent >= 0) kids[out.nodes[i].parent].push_back(i);
        std::function<bool(int, int)> includes = [&](int c, int leaf) -> bool {
            const DevNode& cn = out.nodes[c];
            if (cn.kind == RR_GROUP) {
                for (int k : kids[c])
                    if (includes(k, leaf)) return true;
                return false;
            }
            if (cn.kind == RR_CSG) return (kids[c].size() > 0 && kids[c][0] == leaf) || (kids[c].size() > 1 && kids[c][1] == leaf);
            return c == leaf;
        };
        for (int i = 0; i < N; ++i) {
            DevNode& nd = out.nodes[i];
            if (is_container(nd.kind) || nd.parent < 0) continue;
            const DevGroup& g = out.groups[out.nodes[nd.parent].aux];
            for (int dd = 0; dd < g.depth; ++dd) {
                const int c = g.anc[dd];
                if (out.nodes[c].kind == RR_CSG && !kids[c].empty() && includes(kids[c][0], i))
                    nd.flags |= NF_CSG_LHIT0 << dd;
            }
        }
        for (const DevNode& nd : out.nodes)  // bounded per-ray entry buffer for a CSG subtree
            if (nd.kind == RR_CSG) {
                int entries = 0;
                const int self = (int)(&nd - out.nodes.data());
                for (int j = self + 1; j < nd.skip; ++j)
                    if (!is_container(out.nodes[j].kind))
                        entries += (out.nodes[j].kind == RR_CYLINDER || out.nodes[j].kind == RR_CONE ||
                                    out.nodes[j].kind == RR_TORUS)
                                       ? 4
                                       : 2;
                if (entries > RR_MAX_CSG_ENTRIES) {
                    err = "a CSG subtree can produce more than RR_MAX_CSG_ENTRIES intersections";
                    return RR_E_LIMIT;
                }
            }
    }
    reorder_spatial(out);
    build_chunks(out);
    // identity-transform triangles carry their Möller-Trumbore data in the (unused) inverse slots, after
    // every use of the stored inverses above (culls); the kernels and rr_scene_inspect know NF_TRI_INLINE
    int n_tri = 0, n_inline = 0;
    for (DevNode& nd : out.nodes) {
        if (nd.kind != RR_TRIANGLE && nd.kind != RR_SMOOTH_TRIANGLE) continue;
        ++n_tri;
        if (!(nd.flags & NF_IDENT)) continue;
        const DevTri& t = out.tris[nd.aux];
        for (int c = 0; c < 3; ++c) {
            nd.inv[c] = t.p1[c];
            nd.inv[3 + c] = t.e1[c];
            nd.inv[6 + c] = t.e2[c];
        }
        nd.inv[9] = nd.inv[10] = nd.inv[11] = 0.0;
        nd.flags |= NF_TRI_INLINE;
        ++n_inline;
    }
    out.tri_inline = n_tri > 0 && n_inline == n_tri ? 1 : 0;
    mark_own_safe(out);
    mark_inner_balls(out);
    for (DevChunk& ch : out.chunks) {  // runs of one kind (DevChunk.run)
        ch.run = CR_NONE;
        const DevNode& a = out.nodes[ch.start];
        bool mesh = a.parent >= 0, spheres = true;
        for (int m = ch.start; m < ch.start + ch.count; ++m) {
            const DevNode& nd = out.nodes[m];
            mesh = mesh && (nd.kind == RR_TRIANGLE || nd.kind == RR_SMOOTH_TRIANGLE) && (nd.flags & NF_TRI_INLINE) &&
                   !(nd.flags & NF_IN_CSG) && nd.parent == a.parent;
            spheres = spheres && nd.kind == RR_SPHERE && nd.parent < 0 && (nd.flags & NF_DIAG) && !(nd.flags & NF_IDENT) &&
                      !(nd.flags & NF_IN_CSG);
        }
        if (mesh) {
            ch.run = a.parent;
        } else if (spheres) {
            ch.run = CR_SPHERE_DIAG;
        }
    }
    return RR_OK;
}

}  // namespace rr
