// rray_oracle.cpp — TEST INFRASTRUCTURE ONLY (see rray_oracle.h).
//
// CPU restatement of davelpz/rray's render path, op for op, for parity checks.
// Every function cites the reference file:line it restates (paths relative to
// /root/reference/src).  Compile with -O2 -ffp-contract=off (no FMA contraction,
// matching rustc); never with -ffast-math.
#include "rray_oracle.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

namespace {

const double EPSILON = 0.00001;  // main.rs:10

// ---------------------------------------------------------------- tuple.rs
struct Tuple {
    double x, y, z, w;
};
inline Tuple point(double x, double y, double z) { return {x, y, z, 1.0}; }   // tuple.rs:48
inline Tuple vector(double x, double y, double z) { return {x, y, z, 0.0}; }  // tuple.rs:53
inline Tuple add(const Tuple& a, const Tuple& b) { return {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
inline Tuple sub(const Tuple& a, const Tuple& b) { return {a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; }
inline Tuple neg(const Tuple& a) { return {-a.x, -a.y, -a.z, -a.w}; }
inline Tuple mul(const Tuple& a, double s) { return {a.x * s, a.y * s, a.z * s, a.w * s}; }
inline Tuple divs(const Tuple& a, double s) { return {a.x / s, a.y / s, a.z / s, a.w / s}; }
// tuple.rs:85-87: powi(2) == x*x (LLVM expands the constant powi; compiler_builtins agrees)
inline double magnitude(const Tuple& a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w); }
inline Tuple normalize(const Tuple& a) {  // tuple.rs:95-98
    double m = magnitude(a);
    return {a.x / m, a.y / m, a.z / m, a.w / m};
}
inline double dot(const Tuple& a, const Tuple& b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
inline Tuple cross(const Tuple& a, const Tuple& b) {  // tuple.rs:106-112
    return vector(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
inline Tuple reflect(const Tuple& v, const Tuple& n) { return sub(v, mul(n, 2.0 * dot(v, n))); }  // tuple.rs:115-117

// ---------------------------------------------------------------- color.rs
struct Color {
    double r, g, b;
};
inline Color cadd(const Color& a, const Color& b) { return {a.r + b.r, a.g + b.g, a.b + b.b}; }
inline Color csub(const Color& a, const Color& b) { return {a.r - b.r, a.g - b.g, a.b - b.b}; }
inline Color cmul(const Color& a, double s) { return {a.r * s, a.g * s, a.b * s}; }
inline Color cprod(const Color& a, const Color& b) { return {a.r * b.r, a.g * b.g, a.b * b.b}; }
const Color BLACK = {0.0, 0.0, 0.0};

// ---------------------------------------------------------------- matrix.rs
// Dynamic-size matrix: the cofactor inverse recurses through 3x3 and 2x2 submatrices.
struct Matrix {
    int rows = 4, cols = 4;
    std::vector<double> data;
    Matrix() : data(16, 0.0) {}
    Matrix(int r, int c) : rows(r), cols(c), data((size_t)r * c, 0.0) {}
    double get(int r, int c) const { return data[(size_t)r * cols + c]; }
    void set(int r, int c, double v) { data[(size_t)r * cols + c] = v; }
};
Matrix identity4() {  // matrix.rs identity
    Matrix m(4, 4);
    for (int i = 0; i < 4; ++i) m.set(i, i, 1.0);
    return m;
}
Matrix mat_multiply(const Matrix& a, const Matrix& b) {  // matrix.rs:205-216: sum from 0.0, k ascending
    Matrix r(a.rows, b.cols);
    for (int i = 0; i < a.rows; ++i)
        for (int j = 0; j < b.cols; ++j) {
            double sum = 0.0;
            for (int k = 0; k < a.cols; ++k) sum += a.get(i, k) * b.get(k, j);
            r.set(i, j, sum);
        }
    return r;
}
Tuple mul_tuple(const Matrix& m, const Tuple& t) {  // matrix.rs:234-240 (left-to-right 4-term sums)
    double x = m.get(0, 0) * t.x + m.get(0, 1) * t.y + m.get(0, 2) * t.z + m.get(0, 3) * t.w;
    double y = m.get(1, 0) * t.x + m.get(1, 1) * t.y + m.get(1, 2) * t.z + m.get(1, 3) * t.w;
    double z = m.get(2, 0) * t.x + m.get(2, 1) * t.y + m.get(2, 2) * t.z + m.get(2, 3) * t.w;
    double w = m.get(3, 0) * t.x + m.get(3, 1) * t.y + m.get(3, 2) * t.z + m.get(3, 3) * t.w;
    return {x, y, z, w};
}
Matrix transpose(const Matrix& m) {
    Matrix r(m.cols, m.rows);
    for (int i = 0; i < m.rows; ++i)
        for (int j = 0; j < m.cols; ++j) r.set(j, i, m.get(i, j));
    return r;
}
double determinant(const Matrix& m);
Matrix submatrix(const Matrix& m, int row, int col) {  // matrix.rs:300-320
    Matrix r(m.rows - 1, m.cols - 1);
    int rr = 0;
    for (int i = 0; i < m.rows; ++i) {
        if (i == row) continue;
        int cc = 0;
        for (int j = 0; j < m.cols; ++j) {
            if (j == col) continue;
            r.set(rr, cc, m.get(i, j));
            ++cc;
        }
        ++rr;
    }
    return r;
}
double cofactor(const Matrix& m, int row, int col) {  // matrix.rs:330-345
    double minor = determinant(submatrix(m, row, col));
    return ((row + col) % 2 == 0) ? minor : -minor;
}
double determinant(const Matrix& m) {  // matrix.rs:285-296
    if (m.rows == 2 && m.cols == 2) return m.get(0, 0) * m.get(1, 1) - m.get(0, 1) * m.get(1, 0);
    double det = 0.0;
    for (int i = 0; i < m.cols; ++i) det += m.get(0, i) * cofactor(m, 0, i);
    return det;
}
Matrix inverse(const Matrix& m) {  // matrix.rs:389-412 (the cache does not change values)
    double det = determinant(m);
    Matrix r(m.rows, m.cols);
    for (int i = 0; i < m.rows; ++i)
        for (int j = 0; j < m.cols; ++j) {
            double c = cofactor(m, i, j);
            r.set(j, i, c / det);
        }
    return r;
}
Matrix translate(double x, double y, double z) {  // matrix.rs:430-436
    Matrix m = identity4();
    m.set(0, 3, x);
    m.set(1, 3, y);
    m.set(2, 3, z);
    return m;
}
Matrix scale(double x, double y, double z) {  // matrix.rs:447-453
    Matrix m = identity4();
    m.set(0, 0, x);
    m.set(1, 1, y);
    m.set(2, 2, z);
    return m;
}
Matrix rotate(int axis, double r) {  // matrix.rs:463-510 (glibc sin/cos, as Rust's f64::sin/cos)
    Matrix m = identity4();
    if (axis == 0) {
        m.set(1, 1, std::cos(r));
        m.set(1, 2, -std::sin(r));
        m.set(2, 1, std::sin(r));
        m.set(2, 2, std::cos(r));
    } else if (axis == 1) {
        m.set(0, 0, std::cos(r));
        m.set(0, 2, std::sin(r));
        m.set(2, 0, -std::sin(r));
        m.set(2, 2, std::cos(r));
    } else {
        m.set(0, 0, std::cos(r));
        m.set(0, 1, -std::sin(r));
        m.set(1, 0, std::sin(r));
        m.set(1, 1, std::cos(r));
    }
    return m;
}
Matrix shear(double xy, double xz, double yx, double yz, double zx, double zy) {  // matrix.rs:521-530
    Matrix m = identity4();
    m.set(0, 1, xy);
    m.set(0, 2, xz);
    m.set(1, 0, yx);
    m.set(1, 2, yz);
    m.set(2, 0, zx);
    m.set(2, 1, zy);
    return m;
}
Matrix view_transform(Tuple from, Tuple to, Tuple up) {  // matrix.rs:582-603
    Tuple forward = normalize(sub(to, from));
    Tuple left = cross(forward, normalize(up));
    Tuple true_up = cross(left, forward);
    Matrix o(4, 4);
    o.set(0, 0, left.x);
    o.set(0, 1, left.y);
    o.set(0, 2, left.z);
    o.set(1, 0, true_up.x);
    o.set(1, 1, true_up.y);
    o.set(1, 2, true_up.z);
    o.set(2, 0, -forward.x);
    o.set(2, 1, -forward.y);
    o.set(2, 2, -forward.z);
    o.set(3, 0, 0.0);
    o.set(3, 1, 0.0);
    o.set(3, 2, 0.0);
    o.set(3, 3, 1.0);
    return mat_multiply(o, translate(-from.x, -from.y, -from.z));
}
Matrix from16(const double* m) {
    Matrix r(4, 4);
    for (int i = 0; i < 16; ++i) r.data[i] = m[i];
    return r;
}
void to16(const Matrix& m, double* out) {
    for (int i = 0; i < 16; ++i) out[i] = m.data[i];
}

// ---------------------------------------------------------------- ray.rs
struct Ray {
    Tuple origin, direction;
};
inline Tuple position(const Ray& r, double t) { return add(r.origin, mul(r.direction, t)); }  // ray.rs:38-40
inline Ray transform_ray(const Ray& r, const Matrix& m) {                                      // ray.rs:54-59
    return {mul_tuple(m, r.origin), mul_tuple(m, r.direction)};
}

// ---------------------------------------------------------------- pattern.rs / material.rs
struct Pattern {
    int kind = ORC_PAT_SOLID;
    Color color = {1.0, 1.0, 1.0};
    int a = -1, b = -1;
    double scale = 0.5;
    int64_t octaves = 0;       // perturbed / noise (usize)
    double persistence = 0.0;
    Matrix transform = identity4();
    Matrix inv = identity4();
};
struct Material {  // material.rs:35-58
    int pattern = -1;  // -1 = Pattern::solid(white, identity)
    double ambient = 0.1, diffuse = 0.9, specular = 0.9, shininess = 200.0;
    double reflective = 0.0, transparency = 0.0, refractive_index = 1.0;
};

// ---------------------------------------------------------------- light.rs
struct Light {  // light.rs:10-45
    bool area = false;
    Color intensity;
    Tuple position;  // area: centre = corner + u*0.5 + v*0.5
    Tuple corner, u, v;
    int level = 0;
};

// ---------------------------------------------------------------- object.rs
struct AABB {
    Tuple min, max;
};
struct Object {
    int id = 0, kind = ORC_SPHERE, parent = -1;
    Matrix transform = identity4();
    Matrix inv = identity4();
    Matrix inv_t = identity4();  // inverse().transpose()
    Material material;
    std::vector<int> children;
    Tuple p1{}, p2{}, p3{}, n1{}, n2{}, n3{}, e1{}, e2{}, normal{};
    double minimum = -INFINITY, maximum = INFINITY;  // cylinder / cone
    bool closed = false;
    int csg_op = 0;  // CSG: children[0] = left, children[1] = right
    bool aabb_valid = false;
    AABB aabb{};
};

struct Intersection {  // intersection.rs:11-17
    double t;
    int object;
    double u, v;
};
inline bool ix_eq(const Intersection& a, const Intersection& b) {  // #[derive(PartialEq)]
    return a.t == b.t && a.object == b.object && a.u == b.u && a.v == b.v;
}

struct Computations {  // computations.rs:13-25
    double t;
    int object;
    Tuple point, eyev, normalv;
    bool inside;
    Tuple over_point, under_point, reflectv;
    double n1, n2;
};

struct Ctx {  // per-sample context for the deterministic jitter + counters
    uint64_t seed = 0;
    int jitter_mode = 0;
    uint64_t sample = 0;
    orc_stats st{};
    bool nan = false;
};

uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

}  // namespace

// Deterministic stand-in for thread_rng (light.rs:57-59), shared bit for bit with the HIP kernels
// (device_core.inc jitter_base / jitter_value): a 64-bit mix of (seed, global sample id, recursion
// path) per shading event, then a 32-bit lowbias32 mix per value of (light, cell sample, u/v).
extern "C" double orc_jitter(uint64_t seed, uint64_t sample, uint32_t path, uint32_t light, uint32_t s, uint32_t which) {
    const uint32_t base = (uint32_t)(splitmix64(seed ^ splitmix64(sample ^ ((uint64_t)path << 40))) >> 32);
    uint32_t x = base ^ ((light << 21) | (s << 1) | which);
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return (double)x * (1.0 / 4294967296.0);
}

struct Texture {  // texture.rs:6-11 (RgbaImage after to_rgba8)
    uint32_t width = 0, height = 0;
    std::vector<uint8_t> rgba;
};

struct orc_world {
    std::vector<Object> objects;  // object/db.rs registry: index == id
    std::vector<Texture> textures;
    std::vector<int> ids;         // Scene.ids (scene.rs:24-27)
    std::vector<Light> lights;
    std::vector<Pattern> patterns;
    Ctx ctx;  // context used by the single-ray query API
    bool dirty = true;  // group AABB caches need (re)building (group.rs:54-67 invalidation)
    // DIAGNOSTIC ONLY (never the reference's semantics): 1 = the specular power of an integer shininess
    // n in [0, 512] correctly rounded (x^n in binary128, then rounded once) instead of libm pow.  libm's
    // pow (what the reference's f64::powf calls) is within 0.52 ulp, not always correctly rounded; the
    // fuzz test uses this mode to tell a last-ulp pow difference from a walk error.
    int pow_mode = 0;
};

namespace {

const Pattern& default_pattern() {
    static Pattern p;  // solid white, identity (material.rs:49)
    return p;
}
const Pattern& pat(const orc_world* w, int i) { return i < 0 ? default_pattern() : w->patterns[i]; }

// object.rs:102-109 — parent first, then this object's inverse
Tuple world_to_object(const orc_world* w, int id, const Tuple& p) {
    const Object& o = w->objects[id];
    Tuple pt = p;
    if (o.parent >= 0) pt = world_to_object(w, o.parent, pt);
    return mul_tuple(o.inv, pt);
}
// object.rs:129-138 — inverse-transpose, w=0, normalize, then the parent
Tuple normal_to_world(const orc_world* w, int id, const Tuple& n) {
    const Object& o = w->objects[id];
    Tuple nn = mul_tuple(o.inv_t, n);
    nn.w = 0.0;
    nn = normalize(nn);
    if (o.parent >= 0) nn = normal_to_world(w, o.parent, nn);
    return nn;
}

// ---------------------------------------------------------------- roots 0.0.8 (crates.io "roots")
// torus.rs calls roots::find_roots_quartic; the crate is a third-party dependency (Cargo.toml:18,
// roots = "0.0.8") not vendored in the reference.  Restated from its published analytical solvers
// (src/analytical/{linear,quadratic,biquadratic,cubic,cubic_depressed,cubic_normalized,quartic,
// quartic_depressed}.rs): Roots<F> keeps its roots ascending, and add_new_root drops a value equal
// to one already present.  Parity of this restatement is pinned only through the reference's own
// rendered example1.png (tests/test_oracle_png.py).
namespace rootsq {
struct Roots {
    int n = 0;
    double v[4];
};
Roots add_new_root(Roots r, double x) {
    int pos = 0;
    for (int i = 0; i < r.n; ++i) {
        if (r.v[i] == x) return r;
        if (r.v[i] > x) break;
        pos++;
    }
    if (r.n >= 4) return r;
    for (int i = r.n; i > pos; --i) r.v[i] = r.v[i - 1];
    r.v[pos] = x;
    r.n++;
    return r;
}
Roots one(double x) {
    Roots r;
    r.n = 1;
    r.v[0] = x;
    return r;
}
const double FRAC_PI_3 = 1.04719755119659774615421446109316763;
const double TWO_THIRD_PI = 2.0 * FRAC_PI_3;

Roots linear(double a1, double a0) {  // linear.rs
    if (a1 == 0.0) return a0 == 0.0 ? one(0.0) : Roots{};
    return one(-a0 / a1);
}
Roots quadratic(double a2, double a1, double a0) {  // quadratic.rs
    if (a2 == 0.0) return linear(a1, a0);
    double discriminant = a1 * a1 - 4.0 * a2 * a0;
    if (discriminant < 0.0) return Roots{};
    double a2x2 = 2.0 * a2;
    if (discriminant == 0.0) return one(-a1 / a2x2);
    double sq = std::sqrt(discriminant);
    double same_sign, diff_sign;
    if (a1 < 0.0) {
        same_sign = -a1 + sq;
        diff_sign = -a1 - sq;
    } else {
        same_sign = -a1 - sq;
        diff_sign = -a1 + sq;
    }
    double x1, x2;
    if (std::fabs(same_sign) > std::fabs(a2x2)) {
        double a0x2 = 2.0 * a0;
        if (std::fabs(diff_sign) > std::fabs(a2x2)) {
            x1 = a0x2 / same_sign;
            x2 = a0x2 / diff_sign;
        } else {
            x1 = a0x2 / same_sign;
            x2 = same_sign / a2x2;
        }
    } else {
        x1 = diff_sign / a2x2;
        x2 = same_sign / a2x2;
    }
    Roots r;
    r.n = 2;
    if (x1 < x2) {
        r.v[0] = x1;
        r.v[1] = x2;
    } else {
        r.v[0] = x2;
        r.v[1] = x1;
    }
    return r;
}
Roots biquadratic(double a4, double a2, double a0) {  // biquadratic.rs
    if (a4 == 0.0) return quadratic(a2, 0.0, a0);
    Roots out;
    Roots q = quadratic(a4, a2, a0);
    for (int i = 0; i < q.n; ++i) {
        double x = q.v[i];
        if (x > 0.0) {
            double s = std::sqrt(x);
            out = add_new_root(add_new_root(out, -s), s);
        } else if (x == 0.0) {
            out = add_new_root(out, 0.0);
        }
    }
    return out;
}
Roots cubic_normalized(double a2, double a1, double a0) {  // cubic_normalized.rs: x^3 + a2 x^2 + a1 x + a0
    double q = (3.0 * a1 - a2 * a2) / 9.0;
    double r = (9.0 * a2 * a1 - 27.0 * a0 - 2.0 * a2 * a2 * a2) / 54.0;
    double q3 = q * q * q;
    double d = q3 + r * r;
    double a2_div_3 = a2 / 3.0;
    if (d < 0.0) {
        double phi_3 = std::acos(r / std::sqrt(-q3)) / 3.0;
        double sqrt_q_2 = 2.0 * std::sqrt(-q);
        Roots out = one(sqrt_q_2 * std::cos(phi_3) - a2_div_3);
        out = add_new_root(out, sqrt_q_2 * std::cos(phi_3 - TWO_THIRD_PI) - a2_div_3);
        return add_new_root(out, sqrt_q_2 * std::cos(phi_3 + TWO_THIRD_PI) - a2_div_3);
    }
    double sqrt_d = std::sqrt(d);
    double s = std::cbrt(r + sqrt_d);
    double t = std::cbrt(r - sqrt_d);
    if (s == t) {
        if (s + t == 0.0) return one(s + t - a2_div_3);
        return add_new_root(one(s + t - a2_div_3), -(s + t) / 2.0 - a2_div_3);
    }
    return one(s + t - a2_div_3);
}
Roots cubic_depressed(double a1, double a0) {  // cubic_depressed.rs: x^3 + a1 x + a0
    if (a1 == 0.0) return one(-std::cbrt(a0));
    if (a0 == 0.0) return add_new_root(quadratic(1.0, 0.0, a1), 0.0);
    double d = a0 * a0 / 4.0 + a1 * a1 * a1 / 27.0;
    if (d < 0.0) {
        double a = std::sqrt(-4.0 * a1 / 3.0);
        double phi = std::acos(-4.0 * a0 / (a * a * a)) / 3.0;
        Roots out = one(a * std::cos(phi));
        out = add_new_root(out, a * std::cos(phi + TWO_THIRD_PI));
        return add_new_root(out, a * std::cos(phi - TWO_THIRD_PI));
    }
    double sqrt_d = std::sqrt(d);
    double a0_div_2 = a0 / 2.0;
    double x1 = std::cbrt(sqrt_d - a0_div_2) - std::cbrt(sqrt_d + a0_div_2);
    if (d == 0.0) return add_new_root(one(x1), std::cbrt(a0_div_2));
    return one(x1);
}
Roots cubic(double a3, double a2, double a1, double a0) {  // cubic.rs
    if (a3 == 0.0) return quadratic(a2, a1, a0);
    if (a2 == 0.0) return cubic_depressed(a1 / a3, a0 / a3);
    if (a3 == 1.0) return cubic_normalized(a2, a1, a0);
    double d = 18.0 * a3 * a2 * a1 * a0 - 4.0 * a2 * a2 * a2 * a0 + a2 * a2 * a1 * a1 - 4.0 * a3 * a1 * a1 * a1 -
               27.0 * a3 * a3 * a0 * a0;
    double d0 = a2 * a2 - 3.0 * a3 * a1;
    double d1 = 2.0 * a2 * a2 * a2 - 9.0 * a3 * a2 * a1 + 27.0 * a3 * a3 * a0;
    if (d < 0.0) {  // one real root
        double sq = std::sqrt(-27.0 * a3 * a3 * d);
        double c = std::cbrt((d1 < 0.0 ? d1 - sq : d1 + sq) / 2.0);
        return one(-(a2 + c + d0 / c) / (3.0 * a3));
    }
    if (d == 0.0) {
        if (d0 == 0.0) return one(-a2 / (a3 * 3.0));  // triple root
        return add_new_root(one((9.0 * a3 * a0 - a2 * a1) / (d0 * 2.0)),
                            (4.0 * a3 * a2 * a1 - 9.0 * a3 * a3 * a0 - a2 * a2 * a2) / (a3 * d0));
    }
    // three real roots through the complex cube root of (d1 + i sqrt(27 a3^2 d)) / 2
    double c3_img = std::sqrt(27.0 * a3 * a3 * d) / 2.0;
    double c3_real = d1 / 2.0;
    double c3_module = std::sqrt(c3_img * c3_img + c3_real * c3_real);
    double c3_phase = 2.0 * std::atan(c3_img / (c3_real + c3_module));
    double c_module = std::cbrt(c3_module);
    double c_phase = c3_phase / 3.0;
    double c_real = c_module * std::cos(c_phase);
    double c_img = c_module * std::sin(c_phase);
    double x0_real = -(a2 + c_real + (d0 * c_real) / (c_module * c_module)) / (3.0 * a3);
    double e_real = -1.0 / 2.0;
    double e_img = std::sqrt(3.0) / 2.0;
    double c1_real = c_real * e_real - c_img * e_img;
    double c1_img = c_real * e_img + c_img * e_real;
    double x1_real = -(a2 + c1_real + (d0 * c1_real) / (c1_real * c1_real + c1_img * c1_img)) / (3.0 * a3);
    double c2_real = c1_real * e_real - c1_img * e_img;
    double c2_img = c1_real * e_img + c1_img * e_real;
    double x2_real = -(a2 + c2_real + (d0 * c2_real) / (c2_real * c2_real + c2_img * c2_img)) / (3.0 * a3);
    return add_new_root(add_new_root(one(x0_real), x1_real), x2_real);
}
Roots quartic_depressed(double a2, double a1, double a0) {  // quartic_depressed.rs: x^4 + a2 x^2 + a1 x + a0
    if (a1 == 0.0) return biquadratic(1.0, a2, a0);
    if (a0 == 0.0) return add_new_root(cubic_normalized(0.0, a2, a1), 0.0);
    // resolvent y^3 + 5/2 a2 y^2 + (2 a2^2 - a0) y + (a2^3 - a2 a0 - a1^2 / 4) / 2, largest root
    double a2_pow_2 = a2 * a2;
    double a1_div_2 = a1 / 2.0;
    double b2 = a2 * 5.0 / 2.0;
    double b1 = 2.0 * a2_pow_2 - a0;
    double b0 = (a2_pow_2 * a2 - a2 * a0 - a1_div_2 * a1_div_2) / 2.0;
    Roots res = cubic_normalized(b2, b1, b0);
    double y = res.v[res.n - 1];
    double a2_plus_2y = a2 + 2.0 * y;
    if (!(a2_plus_2y > 0.0)) return Roots{};
    double sqrt_a2_plus_2y = std::sqrt(a2_plus_2y);
    double q0a = a2 + y - a1_div_2 / sqrt_a2_plus_2y;
    double q0b = a2 + y + a1_div_2 / sqrt_a2_plus_2y;
    Roots out = quadratic(1.0, sqrt_a2_plus_2y, q0a);
    Roots more = quadratic(1.0, -sqrt_a2_plus_2y, q0b);
    for (int i = 0; i < more.n; ++i) out = add_new_root(out, more.v[i]);
    return out;
}
// quartic.rs: depressed quartic y^4 + p y^2 + q y + r with x = y - a3 / (4 a4)
Roots via_depressed_quartic(double a4, double a3, double a2, double a1, double a0, double pp, double rr, double dd) {
    double a4_pow_2 = a4 * a4;
    double a4_pow_3 = a4_pow_2 * a4;
    double a4_pow_4 = a4_pow_2 * a4_pow_2;
    double p = pp / (8.0 * a4_pow_2);
    double q = rr / (8.0 * a4_pow_3);
    double r = (dd + 16.0 * a4_pow_2 * (12.0 * a0 * a4 - 3.0 * a1 * a3 + a2 * a2)) / (256.0 * a4_pow_4);
    Roots dep = quartic_depressed(p, q, r);
    Roots out;
    for (int i = 0; i < dep.n; ++i) out = add_new_root(out, dep.v[i] - a3 / (4.0 * a4));
    return out;
}
// quartic.rs: the discriminant (partially factored) and P, R, Delta0, D of the nature-of-roots table
// classify the equation first; only the cases with real roots go through Ferrari's resolvent.
Roots quartic(double a4, double a3, double a2, double a1, double a0) {
    if (a4 == 0.0) return cubic(a3, a2, a1, a0);
    if (a0 == 0.0) return add_new_root(cubic(a4, a3, a2, a1), 0.0);
    if (a1 == 0.0 && a3 == 0.0) return biquadratic(a4, a2, a0);
    double discriminant =
        a4 * a0 * a4 * (256.0 * a4 * a0 * a0 + a1 * (144.0 * a2 * a1 - 192.0 * a3 * a0)) +
        a4 * a0 * a2 * a2 * (16.0 * a2 * a2 - 80.0 * a3 * a1 - 128.0 * a4 * a0) +
        (a3 * a3 *
         (a4 * a0 * (144.0 * a2 * a0 - 6.0 * a1 * a1) +
          (a0 * (18.0 * a3 * a2 * a1 - 27.0 * a3 * a3 * a0 - 4.0 * a2 * a2 * a2) + a1 * a1 * (a2 * a2 - 4.0 * a3 * a1)))) +
        a4 * a1 * a1 * (18.0 * a3 * a2 * a1 - 27.0 * a4 * a1 * a1 - 4.0 * a2 * a2 * a2);
    double pp = 8.0 * a4 * a2 - 3.0 * a3 * a3;
    double rr = a3 * a3 * a3 + 8.0 * a4 * a4 * a1 - 4.0 * a4 * a3 * a2;
    double delta0 = a2 * a2 - 3.0 * a3 * a1 + 12.0 * a4 * a0;
    double dd = 64.0 * a4 * a4 * a4 * a0 - 16.0 * a4 * a4 * a2 * a2 + 16.0 * a4 * a3 * a3 * a2 -
                16.0 * a4 * a4 * a3 * a1 - 3.0 * a3 * a3 * a3 * a3;
    if (discriminant == 0.0) {
        bool triple_root = delta0 == 0.0;
        bool quadruple_root = triple_root && dd == 0.0;
        bool no_roots = dd == 0.0 && pp > 0.0 && rr == 0.0;
        if (quadruple_root) return one(-a3 / (4.0 * a4));
        if (triple_root) {
            double x0 = (-72.0 * a4 * a4 * a0 + 10.0 * a4 * a2 * a2 - 3.0 * a3 * a3 * a2) /
                        (9.0 * (8.0 * a4 * a4 * a1 - 4.0 * a4 * a3 * a2 + a3 * a3 * a3));
            return add_new_root(one(x0), -(a3 / a4 + 3.0 * x0));
        }
        if (no_roots) return Roots{};
        return via_depressed_quartic(a4, a3, a2, a1, a0, pp, rr, dd);
    }
    bool no_roots = discriminant > 0.0 && (pp > 0.0 || dd > 0.0);
    if (no_roots) return Roots{};  // two pairs of complex conjugate roots
    return via_depressed_quartic(a4, a3, a2, a1, a0, pp, rr, dd);
}
}  // namespace rootsq

Tuple local_normal_at(const Object& o, const Tuple& lp, const Intersection& hit) {
    switch (o.kind) {
        case ORC_SPHERE: return sub(lp, point(0.0, 0.0, 0.0));  // sphere.rs:80-82
        case ORC_PLANE: return vector(0.0, 1.0, 0.0);           // plane.rs:59-61
        case ORC_TRIANGLE: return o.normal;                      // triangle.rs:96-98
        case ORC_SMOOTH_TRIANGLE:                                // smooth_triangle.rs:99-101
            return add(add(mul(o.n2, hit.u), mul(o.n3, hit.v)), mul(o.n1, 1.0 - hit.u - hit.v));
        case ORC_CUBE: {  // cube.rs:81-90
            double maxc = std::fmax(std::fmax(std::fabs(lp.x), std::fabs(lp.y)), std::fabs(lp.z));
            if (maxc == std::fabs(lp.x)) return vector(lp.x, 0.0, 0.0);
            if (maxc == std::fabs(lp.y)) return vector(0.0, lp.y, 0.0);
            return vector(0.0, 0.0, lp.z);
        }
        case ORC_CYLINDER: {  // cylinder.rs:113-124
            double dist = lp.x * lp.x + lp.z * lp.z;
            if (dist < 1.0 && lp.y >= o.maximum - EPSILON) return vector(0.0, 1.0, 0.0);
            if (dist < 1.0 && lp.y <= o.minimum + EPSILON) return vector(0.0, -1.0, 0.0);
            return vector(lp.x, 0.0, lp.z);
        }
        case ORC_CONE: {  // cone.rs:137-155
            double dist = lp.x * lp.x + lp.z * lp.z;
            if (dist < 1.0 && lp.y >= o.maximum - EPSILON) return vector(0.0, 1.0, 0.0);
            if (dist < 1.0 && lp.y <= o.minimum + EPSILON) return vector(0.0, -1.0, 0.0);
            double y = std::sqrt(dist);
            if (lp.y > 0.0) y = -y;
            return vector(lp.x, y, lp.z);
        }
        case ORC_TORUS: {  // torus.rs:97-107
            double sum_squared = lp.x * lp.x + lp.y * lp.y + lp.z * lp.z;
            double param_squared = 1.0 + o.minimum * o.minimum;
            Tuple n = vector(4.0 * lp.x * (sum_squared - param_squared), 4.0 * lp.y * (sum_squared - param_squared),
                             4.0 * lp.z * (sum_squared - param_squared + 2.0));
            return normalize(n);
        }
        default: return vector(0, 0, 0);  // group.rs: panics ("Groups do not have normals")
    }
}
Tuple normal_at(const orc_world* w, int id, const Tuple& wp, const Intersection& hit) {  // object.rs:52-56
    Tuple lp = world_to_object(w, id, wp);
    Tuple ln = local_normal_at(w->objects[id], lp, hit);
    return normal_to_world(w, id, ln);
}

// object.rs:178-218
void check_axis(double origin, double direction, double mn, double mx, double& tmin, double& tmax) {
    double tmin_num = mn - origin;
    double tmax_num = mx - origin;
    if (std::fabs(direction) >= EPSILON) {
        tmin = tmin_num / direction;
        tmax = tmax_num / direction;
    } else {
        tmin = tmin_num * INFINITY;
        tmax = tmax_num * INFINITY;
    }
    if (tmin > tmax) std::swap(tmin, tmax);
}
bool aabb_intersect(const AABB& b, const Ray& r) {
    double xmin, xmax, ymin, ymax, zmin, zmax;
    check_axis(r.origin.x, r.direction.x, b.min.x, b.max.x, xmin, xmax);
    check_axis(r.origin.y, r.direction.y, b.min.y, b.max.y, ymin, ymax);
    check_axis(r.origin.z, r.direction.z, b.min.z, b.max.z, zmin, zmax);
    // Rust f64::max/min ignore NaN operands == C fmax/fmin
    double tmin = std::fmax(xmin, std::fmax(ymin, zmin));
    double tmax = std::fmin(xmax, std::fmin(ymax, zmax));
    return tmin <= tmax;
}
void adjust_min_max(AABB& b, double x, double y, double z) {  // object.rs:220-227
    b.min = point(std::fmin(b.min.x, x), std::fmin(b.min.y, y), std::fmin(b.min.z, z));
    b.max = point(std::fmax(b.max.x, x), std::fmax(b.max.y, y), std::fmax(b.max.z, z));
}
AABB apply_transform(const AABB& b, const Matrix& m) {  // object.rs:257-278
    Tuple corners[8] = {point(b.min.x, b.min.y, b.min.z), point(b.min.x, b.min.y, b.max.z),
                        point(b.min.x, b.max.y, b.min.z), point(b.min.x, b.max.y, b.max.z),
                        point(b.max.x, b.min.y, b.min.z), point(b.max.x, b.min.y, b.max.z),
                        point(b.max.x, b.max.y, b.min.z), point(b.max.x, b.max.y, b.max.z)};
    AABB r{point(INFINITY, INFINITY, INFINITY), point(-INFINITY, -INFINITY, -INFINITY)};
    for (auto& c : corners) {
        Tuple t = mul_tuple(m, c);
        adjust_min_max(r, t.x, t.y, t.z);
    }
    return r;
}
AABB get_aabb(orc_world* w, int id) {
    Object& o = w->objects[id];
    switch (o.kind) {
        case ORC_SPHERE: return {point(-1, -1, -1), point(1, 1, 1)};                       // sphere.rs get_aabb
        case ORC_PLANE: return {point(-INFINITY, 0.0, -INFINITY), point(INFINITY, 0.0, INFINITY)};  // plane.rs
        case ORC_TRIANGLE:
        case ORC_SMOOTH_TRIANGLE:  // triangle.rs get_aabb
            return {point(std::fmin(o.p1.x, std::fmin(o.p2.x, o.p3.x)), std::fmin(o.p1.y, std::fmin(o.p2.y, o.p3.y)),
                          std::fmin(o.p1.z, std::fmin(o.p2.z, o.p3.z))),
                    point(std::fmax(o.p1.x, std::fmax(o.p2.x, o.p3.x)), std::fmax(o.p1.y, std::fmax(o.p2.y, o.p3.y)),
                          std::fmax(o.p1.z, std::fmax(o.p2.z, o.p3.z)))};
        case ORC_CUBE: return {point(-1, -1, -1), point(1, 1, 1)};                   // cube.rs get_aabb
        case ORC_CYLINDER: return {point(-1, o.minimum, -1), point(1, o.maximum, 1)};  // cylinder.rs get_aabb
        case ORC_CONE: {                                                          // cone.rs:221-226
            double limit = std::fmax(std::fabs(o.minimum), std::fabs(o.maximum));
            return {point(-limit, o.minimum, -limit), point(limit, o.maximum, limit)};
        }
        case ORC_TORUS: {  // torus.rs get_aabb
            double r = o.minimum;
            return {point(-1.0 - r, -1.0 - r, -r), point(1.0 + r, 1.0 + r, r)};
        }
        case ORC_CSG:  // csg.rs get_aabb (cached): left then right, transformed
        case ORC_GROUP: {  // group.rs:128-149 (cached)
            if (o.aabb_valid) return o.aabb;
            AABB b{point(INFINITY, INFINITY, INFINITY), point(-INFINITY, -INFINITY, -INFINITY)};
            for (int c : o.children) {
                AABB cb = apply_transform(get_aabb(w, c), w->objects[c].transform);
                adjust_min_max(b, cb.min.x, cb.min.y, cb.min.z);  // adjust_aabb: object.rs:237-240
                adjust_min_max(b, cb.max.x, cb.max.y, cb.max.z);
            }
            Object& oo = w->objects[id];
            oo.aabb = b;
            oo.aabb_valid = true;
            return b;
        }
    }
    return {};
}

void sort_xs(std::vector<Intersection>& xs, Ctx& ctx) {
    // Vec::sort_by(partial_cmp().unwrap()) is a stable sort that panics on a NaN comparison; a list of
    // fewer than two entries is never compared
    if (xs.size() >= 2)
        for (auto& x : xs)
            if (std::isnan(x.t)) {
                ctx.nan = true;
                ctx.st.nan_sorts++;
                break;
            }
    std::stable_sort(xs.begin(), xs.end(), [](const Intersection& a, const Intersection& b) { return a.t < b.t; });
}

void intersect_obj(const orc_world* w, int id, const Ray& r, std::vector<Intersection>& xs, Ctx& ctx);

// Object::includes: leaves compare ids, groups ask every child (group.rs:151-159), a CSG only
// compares its two direct children (csg.rs:160-162)
bool includes(const orc_world* w, int id, int object_id) {
    const Object& o = w->objects[id];
    if (o.kind == ORC_GROUP) {
        for (int c : o.children)
            if (includes(w, c, object_id)) return true;
        return false;
    }
    if (o.kind == ORC_CSG)
        return (o.children.size() > 0 && object_id == o.children[0]) ||
               (o.children.size() > 1 && object_id == o.children[1]);
    return o.id == object_id;
}
bool csg_allowed(int op, bool lhit, bool inl, bool inr) {  // csg.rs:67-80
    switch (op) {
        case ORC_CSG_UNION: return (lhit && !inr) || (!lhit && !inl);
        case ORC_CSG_INTERSECTION: return (lhit && inr) || (!lhit && inl);
        default: return (lhit && !inr) || (!lhit && inl);  // difference
    }
}
void csg_filter(const orc_world* w, const Object& o, const std::vector<Intersection>& xs,
                std::vector<Intersection>& out) {  // csg.rs:82-101
    bool inl = false, inr = false;
    const int left = o.children.empty() ? -1 : o.children[0];
    for (const Intersection& i : xs) {
        bool lhit = left >= 0 && includes(w, left, i.object);
        if (csg_allowed(o.csg_op, lhit, inl, inr)) out.push_back(i);
        if (lhit)
            inl = !inl;
        else
            inr = !inr;
    }
}

void local_intersect(const orc_world* w, int id, const Ray& ray, std::vector<Intersection>& xs, Ctx& ctx) {
    const Object& o = w->objects[id];
    switch (o.kind) {
        case ORC_SPHERE: {  // sphere.rs:64-78
            ctx.st.sphere_tests++;
            Tuple s2r = sub(ray.origin, point(0.0, 0.0, 0.0));
            double a = dot(ray.direction, ray.direction);
            double b = 2.0 * dot(ray.direction, s2r);
            double c = dot(s2r, s2r) - 1.0;
            double disc = b * b - 4.0 * a * c;
            if (disc < 0.0) return;
            double t1 = (-b - std::sqrt(disc)) / (2.0 * a);
            double t2 = (-b + std::sqrt(disc)) / (2.0 * a);
            xs.push_back({t1, o.id, 0.0, 0.0});
            xs.push_back({t2, o.id, 0.0, 0.0});
            return;
        }
        case ORC_PLANE: {  // plane.rs:51-58
            ctx.st.plane_tests++;
            if (std::fabs(ray.direction.y) < EPSILON) return;
            double t = -ray.origin.y / ray.direction.y;
            xs.push_back({t, o.id, 0.0, 0.0});
            return;
        }
        case ORC_TRIANGLE:
        case ORC_SMOOTH_TRIANGLE: {  // triangle.rs:72-94, smooth_triangle.rs:75-97
            ctx.st.tri_tests++;
            Tuple dce2 = cross(ray.direction, o.e2);
            double det = dot(o.e1, dce2);
            if (std::fabs(det) < EPSILON) return;
            double f = 1.0 / det;
            Tuple p1o = sub(ray.origin, o.p1);
            double u = f * dot(p1o, dce2);
            if (u < 0.0 || u > 1.0) return;
            Tuple oce1 = cross(p1o, o.e1);
            double v = f * dot(ray.direction, oce1);
            if (v < 0.0 || (u + v) > 1.0) return;
            double t = f * dot(o.e2, oce1);
            xs.push_back({t, o.id, u, v});
            return;
        }
        case ORC_CUBE: {  // cube.rs:64-78
            ctx.st.cube_tests++;
            double xtmin, xtmax, ytmin, ytmax, ztmin, ztmax;
            check_axis(ray.origin.x, ray.direction.x, -1.0, 1.0, xtmin, xtmax);  // cube.rs:49-61
            check_axis(ray.origin.y, ray.direction.y, -1.0, 1.0, ytmin, ytmax);
            check_axis(ray.origin.z, ray.direction.z, -1.0, 1.0, ztmin, ztmax);
            double tmin = std::fmax(std::fmax(xtmin, ytmin), ztmin);
            double tmax = std::fmin(std::fmin(xtmax, ytmax), ztmax);
            if (tmin > tmax) return;
            xs.push_back({tmin, o.id, 0.0, 0.0});
            xs.push_back({tmax, o.id, 0.0, 0.0});
            return;
        }
        case ORC_CYLINDER: {  // cylinder.rs:85-111
            ctx.st.cyl_tests++;
            const Tuple& d = ray.direction;
            const Tuple& og = ray.origin;
            double a = d.x * d.x + d.z * d.z;
            if (std::fabs(a) > EPSILON) {
                double b = 2.0 * og.x * d.x + 2.0 * og.z * d.z;
                double c2 = og.x * og.x + og.z * og.z - 1.0;
                double disc = b * b - 4.0 * a * c2;
                if (disc < 0.0) return;  // returns vec![] — no caps either
                double t0 = (-b - std::sqrt(disc)) / (2.0 * a);
                double t1 = (-b + std::sqrt(disc)) / (2.0 * a);
                if (t0 > t1) std::swap(t0, t1);
                double y0 = og.y + t0 * d.y;
                if (o.minimum < y0 && y0 < o.maximum) xs.push_back({t0, o.id, 0.0, 0.0});
                double y1 = og.y + t1 * d.y;
                if (o.minimum < y1 && y1 < o.maximum) xs.push_back({t1, o.id, 0.0, 0.0});
            }
            // intersect_caps (cylinder.rs:48-73), check_cap (cylinder.rs:40-46)
            if (!o.closed || std::fabs(d.y) < EPSILON) return;
            for (double lim : {o.minimum, o.maximum}) {
                double t = (lim - og.y) / d.y;
                double x = og.x + t * d.x, z = og.z + t * d.z;
                if ((x * x + z * z) <= 1.0) xs.push_back({t, o.id, 0.0, 0.0});
            }
            return;
        }
        case ORC_CONE: {  // cone.rs:75-135
            ctx.st.cone_tests++;
            const Tuple& d = ray.direction;
            const Tuple& og = ray.origin;
            auto caps = [&]() {  // cone.rs:46-73, check_cap cone.rs:36-44
                if (!o.closed || std::fabs(d.y) < EPSILON) return;
                for (double lim : {o.minimum, o.maximum}) {
                    double t = (lim - og.y) / d.y;
                    double x = og.x + t * d.x, y = og.y + t * d.y, z = og.z + t * d.z;
                    if ((x * x + z * z) <= y * y) xs.push_back({t, o.id, 0.0, 0.0});
                }
            };
            double a = d.x * d.x - d.y * d.y + d.z * d.z;
            double b = 2.0 * og.x * d.x - 2.0 * og.y * d.y + 2.0 * og.z * d.z;
            if (std::fabs(a) < EPSILON && std::fabs(b) < EPSILON) {
                caps();
                return;
            }
            double c2 = og.x * og.x - og.y * og.y + og.z * og.z;
            if (std::fabs(a) < EPSILON) {
                double t = -c2 / (2.0 * b);
                double y = og.y + t * d.y;
                if (o.minimum < y && y < o.maximum) {
                    xs.push_back({t, o.id, 0.0, 0.0});
                    return;  // cone.rs:101-103: returns without the caps
                }
            }
            double disc = b * b - 4.0 * a * c2;
            if (disc < 0.0) return;
            double t0 = (-b - std::sqrt(disc)) / (2.0 * a);
            double t1 = (-b + std::sqrt(disc)) / (2.0 * a);
            if (t0 > t1) std::swap(t0, t1);
            double y0 = og.y + t0 * d.y;
            if (o.minimum < y0 && y0 < o.maximum) xs.push_back({t0, o.id, 0.0, 0.0});
            double y1 = og.y + t1 * d.y;
            if (o.minimum < y1 && y1 < o.maximum) xs.push_back({t1, o.id, 0.0, 0.0});
            caps();
            return;
        }
        case ORC_TORUS: {  // torus.rs:37-95
            ctx.st.torus_tests++;
            const Tuple& og = ray.origin;
            const Tuple& d = ray.direction;
            double r = o.minimum;
            double r_sq = r * r;
            double sum_d_sq = d.x * d.x + d.y * d.y + d.z * d.z;
            double e = og.x * og.x + og.y * og.y + og.z * og.z - r_sq + 1.0;
            double f = dot(og, d);
            const double four = 4.0;
            double a4 = sum_d_sq * sum_d_sq;
            double a3 = 4.0 * sum_d_sq * f;
            double a2 = 2.0 * sum_d_sq * e + 4.0 * f * f - four * (d.x * d.x + d.y * d.y);
            double a1 = 4.0 * e * f - 2.0 * four * (og.x * d.x + og.y * d.y);
            double a0 = e * e - four * (og.x * og.x + og.y * og.y);
            rootsq::Roots rs = rootsq::quartic(a4, a3, a2, a1, a0);
            for (int i = 0; i < rs.n; ++i)
                if (rs.v[i] > 0.0) xs.push_back({rs.v[i], o.id, 0.0, 0.0});
            return;
        }
        case ORC_CSG: {  // csg.rs:105-113: left.intersect ++ right.intersect, sort, filter
            ctx.st.csg_tests++;
            std::vector<Intersection> cx;
            if (o.children.size() >= 1) intersect_obj(w, o.children[0], ray, cx, ctx);
            if (o.children.size() >= 2) intersect_obj(w, o.children[1], ray, cx, ctx);
            sort_xs(cx, ctx);
            csg_filter(w, o, cx, xs);
            return;
        }
        case ORC_GROUP: {  // group.rs:80-91
            ctx.st.group_tests++;
            std::vector<Intersection> gx;
            if (aabb_intersect(w->objects[id].aabb, ray)) {
                ctx.st.group_hits++;
                for (int c : o.children) intersect_obj(w, c, ray, gx, ctx);
                sort_xs(gx, ctx);
            }
            xs.insert(xs.end(), gx.begin(), gx.end());
            return;
        }
    }
}
// object.rs:45-48: transform the ray by the inverse, then local_intersect
void intersect_obj(const orc_world* w, int id, const Ray& r, std::vector<Intersection>& xs, Ctx& ctx) {
    Ray tr = transform_ray(r, w->objects[id].inv);
    local_intersect(w, id, tr, xs, ctx);
}

// scene.rs:97-106
std::vector<Intersection> scene_intersect(const orc_world* w, const Ray& r, Ctx& ctx) {
    ctx.st.rays++;
    std::vector<Intersection> xs;
    for (int id : w->ids) intersect_obj(w, id, r, xs, ctx);
    sort_xs(xs, ctx);
    return xs;
}

// intersection.rs:50-95
Computations prepare_computations(const orc_world* w, const Intersection& self, const Ray& r,
                                  const std::vector<Intersection>& xs) {
    Computations c;
    c.t = self.t;
    c.object = self.object;
    c.point = position(r, self.t);
    c.eyev = neg(r.direction);
    Tuple n = normal_at(w, self.object, c.point, self);
    c.inside = dot(n, c.eyev) < 0.0;
    c.normalv = c.inside ? neg(n) : n;
    c.over_point = add(c.point, mul(c.normalv, EPSILON));
    c.under_point = sub(c.point, mul(c.normalv, EPSILON));
    c.reflectv = reflect(r.direction, c.normalv);
    c.n1 = 1.0;
    c.n2 = 1.0;
    std::vector<int> containers;
    for (const Intersection& i : xs) {
        if (ix_eq(i, self)) {
            c.n1 = containers.empty() ? 1.0 : w->objects[containers.back()].material.refractive_index;
        }
        auto it = std::find(containers.begin(), containers.end(), i.object);
        if (it != containers.end())
            containers.erase(it);
        else
            containers.push_back(i.object);
        if (ix_eq(i, self)) {
            c.n2 = containers.empty() ? 1.0 : w->objects[containers.back()].material.refractive_index;
        }
    }
    return c;
}

// computations.rs:39-54
double schlick(const Computations& c) {
    double cos = dot(c.eyev, c.normalv);
    if (c.n1 > c.n2) {
        double n = c.n1 / c.n2;
        double sin2_t = n * n * (1.0 - cos * cos);
        if (sin2_t > 1.0) return 1.0;
        double cos_t = std::sqrt(1.0 - sin2_t);
        cos = cos_t;
    }
    double q = (c.n1 - c.n2) / (c.n1 + c.n2);
    double r0 = q * q;
    double m = 1.0 - cos;
    double m2 = m * m;
    double m5 = m * (m2 * m2);  // powi(5): x * (x^2)^2 (LLVM ExpandPowI / __powidf2 order)
    return r0 + (1.0 - r0) * m5;
}

// saturating `as i32` (Rust semantics)
int32_t sat_i32(double v) {
    if (std::isnan(v)) return 0;
    if (v >= 2147483647.0) return 2147483647;
    if (v <= -2147483648.0) return (int32_t)-2147483648LL;
    return (int32_t)v;
}

// pattern.rs:145-215
// ---------------------------------------------------------------- noise.rs
// fastnoise-lite 1.1.1 (crate feature "f64"), NoiseType::Perlin with the defaults noise.rs keeps:
// seed 1337, frequency 0.01 (an f32, widened to f64 when the coordinates are scaled), no fractal,
// no domain rotation.  Lattice coordinates are f64 (FastFloor), the fractional parts are cast to
// f32 and everything after is f32 arithmetic; get_noise_3d returns the f32 noise.
namespace fnl {
const int32_t PRIME_X = 501125321, PRIME_Y = 1136930381, PRIME_Z = 1720413743;
const float GRADIENTS_3D[256] = {
    0, 1, 1, 0, 0, -1, 1, 0, 0, 1, -1, 0, 0, -1, -1, 0, 1, 0, 1, 0, -1, 0, 1, 0, 1, 0, -1, 0, -1, 0, -1, 0,
    1, 1, 0, 0, -1, 1, 0, 0, 1, -1, 0, 0, -1, -1, 0, 0, 0, 1, 1, 0, 0, -1, 1, 0, 0, 1, -1, 0, 0, -1, -1, 0,
    1, 0, 1, 0, -1, 0, 1, 0, 1, 0, -1, 0, -1, 0, -1, 0, 1, 1, 0, 0, -1, 1, 0, 0, 1, -1, 0, 0, -1, -1, 0, 0,
    0, 1, 1, 0, 0, -1, 1, 0, 0, 1, -1, 0, 0, -1, -1, 0, 1, 0, 1, 0, -1, 0, 1, 0, 1, 0, -1, 0, -1, 0, -1, 0,
    1, 1, 0, 0, -1, 1, 0, 0, 1, -1, 0, 0, -1, -1, 0, 0, 0, 1, 1, 0, 0, -1, 1, 0, 0, 1, -1, 0, 0, -1, -1, 0,
    1, 0, 1, 0, -1, 0, 1, 0, 1, 0, -1, 0, -1, 0, -1, 0, 1, 1, 0, 0, -1, 1, 0, 0, 1, -1, 0, 0, -1, -1, 0, 0,
    0, 1, 1, 0, 0, -1, 1, 0, 0, 1, -1, 0, 0, -1, -1, 0, 1, 0, 1, 0, -1, 0, 1, 0, 1, 0, -1, 0, -1, 0, -1, 0,
    1, 1, 0, 0, -1, 1, 0, 0, 1, -1, 0, 0, -1, -1, 0, 0, 1, 1, 0, 0, 0, -1, 1, 0, -1, 1, 0, 0, 0, -1, -1, 0};
int32_t as_i32(double f) {  // Rust `as i32`: truncate, saturate, NaN -> 0
    if (f != f) return 0;
    if (f >= 2147483647.0) return 2147483647;
    if (f <= -2147483648.0) return INT32_MIN;
    return (int32_t)f;
}
int32_t fast_floor(double f) { return f >= 0 ? as_i32(f) : (int32_t)((uint32_t)as_i32(f) - 1u); }
int32_t wmul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
int32_t wadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
float interp_quintic(float t) { return t * t * t * (t * (t * 6.0f - 15.0f) + 10.0f); }
float lerp(float a, float b, float t) { return a + t * (b - a); }
float grad_coord(int32_t seed, int32_t xp, int32_t yp, int32_t zp, float xd, float yd, float zd) {
    int32_t hash = wmul(seed ^ xp ^ yp ^ zp, 0x27d4eb2d);
    hash ^= hash >> 15;  // arithmetic shift (i32)
    hash &= 63 << 2;
    return xd * GRADIENTS_3D[hash] + yd * GRADIENTS_3D[hash | 1] + zd * GRADIENTS_3D[hash | 2];
}
float single_perlin(int32_t seed, double x, double y, double z) {
    int32_t x0 = fast_floor(x), y0 = fast_floor(y), z0 = fast_floor(z);
    float xd0 = (float)(x - (double)x0), yd0 = (float)(y - (double)y0), zd0 = (float)(z - (double)z0);
    float xd1 = xd0 - 1.0f, yd1 = yd0 - 1.0f, zd1 = zd0 - 1.0f;
    float xs = interp_quintic(xd0), ys = interp_quintic(yd0), zs = interp_quintic(zd0);
    x0 = wmul(x0, PRIME_X);
    y0 = wmul(y0, PRIME_Y);
    z0 = wmul(z0, PRIME_Z);
    int32_t x1 = wadd(x0, PRIME_X), y1 = wadd(y0, PRIME_Y), z1 = wadd(z0, PRIME_Z);
    float xf00 = lerp(grad_coord(seed, x0, y0, z0, xd0, yd0, zd0), grad_coord(seed, x1, y0, z0, xd1, yd0, zd0), xs);
    float xf10 = lerp(grad_coord(seed, x0, y1, z0, xd0, yd1, zd0), grad_coord(seed, x1, y1, z0, xd1, yd1, zd0), xs);
    float xf01 = lerp(grad_coord(seed, x0, y0, z1, xd0, yd0, zd1), grad_coord(seed, x1, y0, z1, xd1, yd0, zd1), xs);
    float xf11 = lerp(grad_coord(seed, x0, y1, z1, xd0, yd1, zd1), grad_coord(seed, x1, y1, z1, xd1, yd1, zd1), xs);
    float yf0 = lerp(xf00, xf10, ys);
    float yf1 = lerp(xf01, xf11, ys);
    return lerp(yf0, yf1, zs) * 0.964921414852142333984375f;
}
float get_noise_3d(double x, double y, double z) {
    const double freq = (double)0.01f;  // frequency: f32, `as Float` when scaling the coordinates
    return single_perlin(1337, x * freq, y * freq, z * freq);
}
}  // namespace fnl

// noise.rs:11-29
double octave_perlin(double x, double y, double z, int64_t octaves, double persistence) {
    double total = 0.0, frequency = 1.0, amplitude = 1.0, max_value = 0.0;
    for (int64_t i = 0; i < octaves; ++i) {
        total += (double)fnl::get_noise_3d(x * frequency, y * frequency, z * frequency) * amplitude;
        max_value += amplitude;
        amplitude *= persistence;
        frequency *= 2.0;
    }
    return total / max_value;
}

double rust_clamp(double x, double lo, double hi) {  // f64::clamp: NaN passes through
    if (x < lo) x = lo;
    if (x > hi) x = hi;
    return x;
}
uint32_t as_u32(double f) {  // `as u32`: truncate, saturate, NaN -> 0
    if (!(f > 0.0)) return 0;
    if (f >= 4294967295.0) return 4294967295u;
    return (uint32_t)f;
}

// texture.rs:31-55
void texture_color(const Texture& t, double u, double v, uint8_t out[4]) {
    u = rust_clamp(u, 0.0, 1.0);
    v = rust_clamp(v, 0.0, 1.0);
    uint32_t x = std::min(as_u32(u * (double)t.width), t.width - 1);
    uint32_t y = std::min(as_u32(v * (double)t.height), t.height - 1);
    y = t.height - y - 1;  // v = 0 is the bottom row
    const uint8_t* px = &t.rgba[4 * ((size_t)y * t.width + x)];
    for (int k = 0; k < 4; ++k) out[k] = px[k];
}
Color sample_texture(const Texture& t, double u, double v) {
    uint8_t c[4];
    texture_color(t, u, v, c);
    return Color{(double)c[0] / 255.0, (double)c[1] / 255.0, (double)c[2] / 255.0};
}

// Object::uv_mapping: sphere.rs:126-132, plane.rs:105-113, cube.rs:132-175, cylinder.rs:181-197,
// cone.rs:232-257, triangle.rs:148-170 (smooth_triangle.rs:151-173 is the same); groups and CSG keep
// the trait default (0, 0) (object.rs:70-72).
void uv_mapping(const Object& o, const Tuple& p, double& u, double& v) {
    const double PI = 3.141592653589793;
    switch (o.kind) {
        case ORC_SPHERE: {
            double theta = std::atan2(p.z, p.x);
            double phi = std::acos(p.y / std::sqrt(p.x * p.x + p.y * p.y + p.z * p.z));
            u = (theta + PI) / (2.0 * PI);
            v = 1.0 - (phi / PI);
            return;
        }
        case ORC_PLANE: {
            u = std::fmod(p.x, 1.0);
            v = std::fmod(p.z, 1.0);
            if (u < 0.0) u = 1.0 + u;
            if (v < 0.0) v = 1.0 + v;
            return;
        }
        case ORC_CUBE: {
            double ax = std::fabs(p.x), ay = std::fabs(p.y), az = std::fabs(p.z);
            if (ax >= ay && ax >= az) {
                u = p.x > 0.0 ? (p.z + 1.0) * 0.5 : (1.0 - p.z) * 0.5;
                v = (p.y + 1.0) * 0.5;
            } else if (ay >= ax && ay >= az) {
                u = (p.x + 1.0) * 0.5;
                v = p.y > 0.0 ? (1.0 - p.z) * 0.5 : (p.z + 1.0) * 0.5;
            } else {
                u = p.z > 0.0 ? (p.x + 1.0) * 0.5 : (1.0 - p.x) * 0.5;
                v = (p.y + 1.0) * 0.5;
            }
            return;
        }
        case ORC_CYLINDER: {
            if (o.closed && (p.y <= o.minimum || p.y >= o.maximum)) {
                u = (p.x + 1.0) / 2.0;
                v = (p.z + 1.0) / 2.0;
                return;
            }
            double theta = std::atan2(p.z, p.x);
            u = (theta + PI) / (2.0 * PI);
            v = std::fmod(p.y, 1.0);
            if (v < 0.0) v = 1.0 + v;
            return;
        }
        case ORC_CONE: {
            double dmin = std::fabs(p.y - o.minimum), dmax = std::fabs(p.y - o.maximum);
            if (o.closed && (dmin <= EPSILON || dmax <= EPSILON)) {
                double radius = std::fabs(p.y);
                u = (p.x / radius + 1.0) / 2.0;
                v = (p.z / radius + 1.0) / 2.0;
                return;
            }
            double theta = (std::atan2(p.z, p.x) + PI) / (2.0 * PI);
            u = (p.y - o.minimum) / (o.maximum - o.minimum);
            v = theta;
            return;
        }
        case ORC_TRIANGLE:
        case ORC_SMOOTH_TRIANGLE: {
            Tuple v0 = sub(o.p2, o.p1), v1 = sub(o.p3, o.p1), v2 = sub(p, o.p1);
            double d00 = dot(v0, v0), d01 = dot(v0, v1), d11 = dot(v1, v1), d20 = dot(v2, v0), d21 = dot(v2, v1);
            double denom = d00 * d11 - d01 * d01;
            u = (d11 * d20 - d01 * d21) / denom;
            v = (d00 * d21 - d01 * d20) / denom;
            return;
        }
        case ORC_TORUS: {  // torus.rs:150-161
            u = (std::atan2(p.y, p.x) + PI) / (2.0 * PI);
            double dist_to_center = std::sqrt(p.x * p.x + p.y * p.y) - 1.0;
            v = (std::atan2(p.z, dist_to_center) + PI) / (2.0 * PI);
            return;
        }
        default:
            u = 0.0;
            v = 0.0;
    }
}

Color pattern_at(const orc_world* w, int pidx, const Tuple& object_point, int shape) {
    const Pattern& p = pat(w, pidx);
    Tuple pp = mul_tuple(p.inv, object_point);
    switch (p.kind) {
        case ORC_PAT_TEST: return {pp.x, pp.y, pp.z};
        case ORC_PAT_SOLID: return p.color;
        case ORC_PAT_STRIPE:
            return (sat_i32(std::floor(pp.x)) % 2 == 0) ? pattern_at(w, p.a, pp, shape) : pattern_at(w, p.b, pp, shape);
        case ORC_PAT_GRADIENT: {
            Color a = pattern_at(w, p.a, pp, shape);
            Color b = pattern_at(w, p.b, pp, shape);
            Color distance = csub(b, a);
            double fraction = pp.x - std::floor(pp.x);
            return cadd(a, cmul(distance, fraction));
        }
        case ORC_PAT_RING:
            return (sat_i32(std::floor(std::sqrt(pp.x * pp.x + pp.z * pp.z))) % 2 == 0) ? pattern_at(w, p.a, pp, shape)
                                                                                           : pattern_at(w, p.b, pp, shape);
        case ORC_PAT_CHECKER:
            return (sat_i32(std::floor(pp.x) + std::floor(pp.y) + std::floor(pp.z)) % 2 == 0) ? pattern_at(w, p.a, pp, shape)
                                                                                              : pattern_at(w, p.b, pp, shape);
        case ORC_PAT_BLEND: {
            Color a = pattern_at(w, p.a, pp, shape);
            Color b = pattern_at(w, p.b, pp, shape);
            return cadd(cmul(a, 1.0 - p.scale), cmul(b, p.scale));
        }
        case ORC_PAT_PERTURBED: {  // pattern.rs:187-199
            double nx = octave_perlin(pp.x, pp.y, pp.z, p.octaves, p.persistence) * p.scale;
            double ny = octave_perlin(pp.x, pp.y, pp.z + 1.0, p.octaves, p.persistence) * p.scale;
            double nz = octave_perlin(pp.x, pp.y, pp.z + 2.0, p.octaves, p.persistence) * p.scale;
            Tuple np = {pp.x + nx, pp.y + ny, pp.z + nz, pp.w};
            return pattern_at(w, p.a, np, shape);
        }
        case ORC_PAT_NOISE: {  // pattern.rs:200-208
            double n = octave_perlin(pp.x, pp.y, pp.z, p.octaves, p.persistence);
            n = n * p.scale;
            if (n <= 0.0) return cmul(pattern_at(w, p.a, pp, shape), -n);
            return cmul(pattern_at(w, p.b, pp, shape), n);
        }
        case ORC_PAT_TEXTURE: {  // pattern.rs:209-213: uv of the shape being shaded
            double u = 0.0, v = 0.0;
            if (shape >= 0) uv_mapping(w->objects[shape], pp, u, v);
            return sample_texture(w->textures[p.a], u, v);
        }
    }
    return BLACK;
}
// material.rs:77-80
Color pattern_at_object(const orc_world* w, int shape, const Tuple& wp) {
    Tuple op = world_to_object(w, shape, wp);
    return pattern_at(w, w->objects[shape].material.pattern, op, shape);
}

// light.rs:98-140
Color lighting(const orc_world* w, int obj, const Light& light, const Tuple& point, const Tuple& eyev,
               const Tuple& normalv, double in_shadow) {
    const Material& m = w->objects[obj].material;
    Color color = pattern_at_object(w, obj, point);
    Color eff = cprod(color, light.intensity);
    Tuple lightv = normalize(sub(light.position, point));
    Color ambient = cmul(eff, m.ambient);
    double ldn = dot(lightv, normalv);
    Color diffuse, specular;
    if (ldn < 0.0) {
        diffuse = BLACK;
        specular = BLACK;
    } else {
        diffuse = cmul(cmul(eff, m.diffuse), ldn);
        Tuple reflectv = reflect(neg(lightv), normalv);
        double rde = dot(reflectv, eyev);
        if (rde <= 0.0) {
            specular = BLACK;
        } else {
            double factor;
            if (w->pow_mode == 1 && m.shininess >= 0.0 && m.shininess <= 512.0 && m.shininess == std::floor(m.shininess)) {
                __float128 x = rde, r = 1;  // exact squaring chain: 113-bit products, one final rounding
                for (unsigned n = (unsigned)m.shininess; n; n >>= 1) {
                    if (n & 1u) r *= x;
                    x *= x;
                }
                factor = (double)r;
            } else {
                factor = std::pow(rde, m.shininess);
            }
            specular = cmul(cmul(light.intensity, m.specular), factor);
        }
    }
    Color ds = cmul(cadd(diffuse, specular), 1.0 - in_shadow);
    return cadd(ambient, ds);
}

// light.rs:47-65 (jitter replaced by the shared counter hash)
Tuple sample_point(const Light& l, int sample, int amount, const Ctx& ctx, uint32_t path, uint32_t light_idx) {
    if (!l.area) return l.position;
    int row = sample / amount;
    int col = sample % amount;
    double ur, vr;
    if (ctx.jitter_mode == 1) {
        ur = 0.5;
        vr = 0.5;
    } else {
        ur = orc_jitter(ctx.seed, ctx.sample, path, light_idx, (uint32_t)sample, 0);
        vr = orc_jitter(ctx.seed, ctx.sample, path, light_idx, (uint32_t)sample, 1);
    }
    double uf = ((double)col + ur) / (double)amount;
    double vf = ((double)row + vr) / (double)amount;
    return add(add(l.corner, mul(l.u, uf)), mul(l.v, vf));
}

// scene.rs:249-259
const Intersection* hit(const std::vector<Intersection>& xs) {
    const Intersection* result = nullptr;
    double t = 1.7976931348623157e308;  // f64::MAX
    for (const auto& x : xs)
        if (x.t >= 0.0 && x.t < t) {
            t = x.t;
            result = &x;
        }
    return result;
}

// scene.rs:234-245
bool is_shadowed(const orc_world* w, const Tuple& p, const Tuple& light_pos, Ctx& ctx) {
    Tuple v = sub(light_pos, p);
    double distance = magnitude(v);
    Tuple direction = normalize(v);
    Ray r{p, direction};
    ctx.st.shadow_rays++;
    std::vector<Intersection> xs = scene_intersect(w, r, ctx);
    const Intersection* h = hit(xs);
    return h ? (h->t < distance) : false;
}

Color color_at(const orc_world* w, const Ray& r, int remaining, Ctx& ctx, uint32_t path);

// scene.rs:181-214
Color shade_hit_light(const orc_world* w, const Computations& c, const Light& light, uint32_t li, Ctx& ctx,
                      uint32_t path) {
    if (!light.area) {
        bool sh = is_shadowed(w, c.over_point, light.position, ctx);
        return lighting(w, c.object, light, c.over_point, c.eyev, c.normalv, sh ? 1.0 : 0.0);
    }
    int total = 0;
    int amount = light.level * light.level;
    for (int s = 0; s < amount; ++s) {
        Tuple lp = sample_point(light, s, light.level, ctx, path, li);
        if (is_shadowed(w, c.over_point, lp, ctx)) total += 1;
    }
    double shadowed = (double)total / (double)amount;
    return lighting(w, c.object, light, c.over_point, c.eyev, c.normalv, shadowed);
}

// scene.rs:281-290
Color reflected_color(const orc_world* w, const Computations& c, int remaining, Ctx& ctx, uint32_t path) {
    const Material& m = w->objects[c.object].material;
    if (remaining <= 0 || m.reflective == 0.0) return BLACK;
    Ray rr{c.over_point, c.reflectv};
    Color col = color_at(w, rr, remaining - 1, ctx, path * 2u);
    return cmul(col, m.reflective);
}

// scene.rs:310-336
Color refracted_color(const orc_world* w, const Computations& c, int remaining, Ctx& ctx, uint32_t path) {
    const Material& m = w->objects[c.object].material;
    if (remaining <= 0 || m.transparency == 0.0) return BLACK;
    double n_ratio = c.n1 / c.n2;
    double cos_i = dot(c.eyev, c.normalv);
    double sin2_t = (n_ratio * n_ratio) * (1.0 - cos_i * cos_i);
    if (sin2_t > 1.0) return BLACK;
    double cos_t = std::sqrt(1.0 - sin2_t);
    Tuple direction = sub(mul(c.normalv, n_ratio * cos_i - cos_t), mul(c.eyev, n_ratio));
    Ray rr{c.under_point, direction};
    return cmul(color_at(w, rr, remaining - 1, ctx, path * 2u + 1u), m.transparency);
}

// scene.rs:159-178
Color shade_hit(const orc_world* w, const Computations& c, int remaining, Ctx& ctx, uint32_t path) {
    ctx.st.shade_events++;
    Color surface = BLACK;
    for (size_t li = 0; li < w->lights.size(); ++li)
        surface = cadd(surface, shade_hit_light(w, c, w->lights[li], (uint32_t)li, ctx, path));
    Color reflected = reflected_color(w, c, remaining, ctx, path);
    Color refracted = refracted_color(w, c, remaining, ctx, path);
    const Material& m = w->objects[c.object].material;
    if (m.reflective > 0.0 && m.transparency > 0.0) {
        double R = schlick(c);
        return cadd(cadd(surface, cmul(reflected, R)), cmul(refracted, 1.0 - R));
    }
    return cadd(cadd(surface, reflected), refracted);
}

// scene.rs:128-136
Color color_at(const orc_world* w, const Ray& r, int remaining, Ctx& ctx, uint32_t path) {
    std::vector<Intersection> xs = scene_intersect(w, r, ctx);
    for (const Intersection& x : xs)
        if (x.t >= 0.0) {
            Computations c = prepare_computations(w, x, r, xs);
            return shade_hit(w, c, remaining, ctx, path);
        }
    return BLACK;
}

Tuple tp(const double* p, double w) { return {p[0], p[1], p[2], w}; }
void out3(const Color& c, double* o) {
    o[0] = c.r;
    o[1] = c.g;
    o[2] = c.b;
}
void out4(const Tuple& t, double* o) {
    o[0] = t.x;
    o[1] = t.y;
    o[2] = t.z;
    o[3] = t.w;
}

// caches the derived data the reference computes lazily (inverse cache, AABB cache)
void finalize(orc_world* w) {
    if (!w->dirty) return;
    w->dirty = false;
    for (auto& o : w->objects)
        if (o.kind == ORC_GROUP || o.kind == ORC_CSG) o.aabb_valid = false;
    for (size_t i = 0; i < w->objects.size(); ++i)
        if (w->objects[i].kind == ORC_GROUP || w->objects[i].kind == ORC_CSG) get_aabb(w, (int)i);
}

std::vector<Intersection> xs_from(int n, const double* t, const int* obj, const double* u, const double* v) {
    std::vector<Intersection> xs;
    for (int i = 0; i < n; ++i) xs.push_back({t[i], obj[i], u ? u[i] : 0.0, v ? v[i] : 0.0});
    return xs;
}

}  // namespace

// =============================================================== C API
extern "C" {

void orc_mat_identity(double out[16]) { to16(identity4(), out); }
void orc_mat_translate(double x, double y, double z, double out[16]) { to16(translate(x, y, z), out); }
void orc_mat_scale(double x, double y, double z, double out[16]) { to16(scale(x, y, z), out); }
void orc_mat_rotate(int axis, double r, double out[16]) { to16(rotate(axis, r), out); }
void orc_mat_shear(double xy, double xz, double yx, double yz, double zx, double zy, double out[16]) {
    to16(shear(xy, xz, yx, yz, zx, zy), out);
}
void orc_mat_multiply(const double a[16], const double b[16], double out[16]) {
    to16(mat_multiply(from16(a), from16(b)), out);
}
void orc_mat_inverse(const double a[16], double out[16]) { to16(inverse(from16(a)), out); }
double orc_mat_determinant(const double a[16]) { return determinant(from16(a)); }
void orc_mat_view_transform(const double f[3], const double t[3], const double u[3], double out[16]) {
    to16(view_transform(tp(f, 1.0), tp(t, 1.0), tp(u, 0.0)), out);
}
void orc_mat_multiply_tuple(const double m[16], const double t[4], double out[4]) {
    out4(mul_tuple(from16(m), {t[0], t[1], t[2], t[3]}), out);
}

orc_world* orc_world_new(void) { return new orc_world(); }
void orc_world_free(orc_world* w) { delete w; }

int orc_add_object(orc_world* w, int kind, int parent) {
    Object o;
    o.id = (int)w->objects.size();  // db.rs:60-66 get_next_id
    o.kind = kind;
    o.parent = parent;
    w->objects.push_back(o);
    if (parent >= 0)
        w->objects[parent].children.push_back(o.id);  // group.rs:69-76 add_child
    else
        w->ids.push_back(o.id);  // scene.rs:66-71 add_object
    w->dirty = true;
    return o.id;
}
static void set_tri(Object& o, Tuple p1, Tuple p2, Tuple p3) {  // triangle.rs:52-68
    o.p1 = p1;
    o.p2 = p2;
    o.p3 = p3;
    o.e1 = sub(p2, p1);
    o.e2 = sub(p3, p1);
    o.normal = normalize(cross(o.e2, o.e1));
}
int orc_add_triangle(orc_world* w, int parent, const double p1[3], const double p2[3], const double p3[3]) {
    int id = orc_add_object(w, ORC_TRIANGLE, parent);
    set_tri(w->objects[id], tp(p1, 1), tp(p2, 1), tp(p3, 1));
    return id;
}
int orc_add_smooth_triangle(orc_world* w, int parent, const double p1[3], const double p2[3], const double p3[3],
                            const double n1[3], const double n2[3], const double n3[3]) {
    int id = orc_add_object(w, ORC_SMOOTH_TRIANGLE, parent);
    Object& o = w->objects[id];
    set_tri(o, tp(p1, 1), tp(p2, 1), tp(p3, 1));
    o.n1 = tp(n1, 0);
    o.n2 = tp(n2, 0);
    o.n3 = tp(n3, 0);
    return id;
}
void orc_set_shape_params(orc_world* w, int id, double minimum, double maximum, int closed) {
    Object& o = w->objects[id];
    o.minimum = minimum;
    o.maximum = maximum;
    o.closed = closed != 0;
    w->dirty = true;
}
void orc_set_csg_op(orc_world* w, int id, int op) {
    w->objects[id].csg_op = op;
    w->dirty = true;
}
void orc_get_shape_params(orc_world* w, int id, double out[3]) {
    const Object& o = w->objects[id];
    out[0] = o.minimum;
    out[1] = o.maximum;
    out[2] = o.closed ? 1.0 : 0.0;
}
int orc_get_csg_op(orc_world* w, int id) { return w->objects[id].csg_op; }
int orc_csg_allowed(int op, int lhit, int inl, int inr) { return csg_allowed(op, lhit != 0, inl != 0, inr != 0) ? 1 : 0; }
int orc_csg_filter(orc_world* w, int csg, int n, const double* t, const int* obj, int* keep_index) {
    std::vector<Intersection> xs, out;
    for (int i = 0; i < n; ++i) xs.push_back({t[i], obj[i], (double)i, 0.0});  // u carries the index
    csg_filter(w, w->objects[csg], xs, out);
    for (size_t k = 0; k < out.size(); ++k) keep_index[k] = (int)out[k].u;
    return (int)out.size();
}
void orc_set_transform(orc_world* w, int id, const double m[16]) {
    Object& o = w->objects[id];
    o.transform = from16(m);
    o.inv = inverse(o.transform);
    o.inv_t = transpose(o.inv);
    w->dirty = true;
}
void orc_set_material(orc_world* w, int id, const double m7[7], int pattern) {
    Material& m = w->objects[id].material;
    m.ambient = m7[0];
    m.diffuse = m7[1];
    m.specular = m7[2];
    m.shininess = m7[3];
    m.reflective = m7[4];
    m.transparency = m7[5];
    m.refractive_index = m7[6];
    m.pattern = pattern;
}
int orc_pattern_new(orc_world* w, int kind, const double color[3], int a, int b, double sc, const double m[16]) {
    Pattern p;
    p.kind = kind;
    if (color) p.color = {color[0], color[1], color[2]};
    p.a = a;
    p.b = b;
    p.scale = sc;
    if (m) p.transform = from16(m);
    p.inv = inverse(p.transform);
    w->patterns.push_back(p);
    return (int)w->patterns.size() - 1;
}
void orc_pattern_set_noise(orc_world* w, int pattern, int64_t octaves, double persistence) {
    w->patterns[pattern].octaves = octaves;
    w->patterns[pattern].persistence = persistence;
}
double orc_noise_3d(double x, double y, double z) { return (double)fnl::get_noise_3d(x, y, z); }
double orc_octave_perlin(double x, double y, double z, int64_t octaves, double persistence) {
    return octave_perlin(x, y, z, octaves, persistence);
}
int orc_add_point_light(orc_world* w, const double pos[3], const double color[3]) {
    Light l;
    l.area = false;
    l.position = tp(pos, 1.0);
    l.intensity = {color[0], color[1], color[2]};
    w->lights.push_back(l);
    return (int)w->lights.size() - 1;
}
int orc_add_area_light(orc_world* w, const double corner[3], const double u[3], const double v[3],
                       const double color[3], int level) {
    Light l;  // light.rs:41-45
    l.area = true;
    l.corner = tp(corner, 1.0);
    l.u = tp(u, 0.0);
    l.v = tp(v, 0.0);
    l.level = level;
    l.intensity = {color[0], color[1], color[2]};
    l.position = add(add(l.corner, mul(l.u, 0.5)), mul(l.v, 0.5));
    w->lights.push_back(l);
    return (int)w->lights.size() - 1;
}
void orc_remove_light(orc_world* w, int index) { w->lights.erase(w->lights.begin() + index); }
int orc_num_children(orc_world* w, int id) { return (int)w->objects[id].children.size(); }
int orc_num_objects(orc_world* w) { return (int)w->objects.size(); }
int orc_num_patterns(orc_world* w) { return (int)w->patterns.size(); }
void orc_pattern_info(orc_world* w, int id, int32_t ints[3], double dbl[2], int64_t* octaves) {
    const Pattern& p = w->patterns[id];
    ints[0] = p.kind;
    ints[1] = p.a;
    ints[2] = p.b;
    dbl[0] = p.scale;
    dbl[1] = p.persistence;
    *octaves = p.octaves;
}
void orc_get_inverse(orc_world* w, int id, double out[16]) { to16(w->objects[id].inv, out); }

void orc_set_pow_mode(orc_world* w, int mode) { w->pow_mode = mode; }

void orc_set_context(orc_world* w, uint64_t seed, int jitter_mode, uint64_t sample) {
    w->ctx.seed = seed;
    w->ctx.jitter_mode = jitter_mode;
    w->ctx.sample = sample;
}
void orc_get_stats(orc_world* w, orc_stats* out) { *out = w->ctx.st; }

int orc_intersect(orc_world* w, const double o[3], const double d[3], int max, double* t, int* obj, double* u,
                  double* v) {
    finalize(w);
    Ray r{tp(o, 1.0), tp(d, 0.0)};
    std::vector<Intersection> xs = scene_intersect(w, r, w->ctx);
    int n = (int)xs.size();
    for (int i = 0; i < n && i < max; ++i) {
        t[i] = xs[i].t;
        obj[i] = xs[i].object;
        if (u) u[i] = xs[i].u;
        if (v) v[i] = xs[i].v;
    }
    return n;
}
int orc_local_intersect(orc_world* w, int id, const double o[4], const double d[4], int max, double* t, int* obj,
                        double* u, double* v) {
    finalize(w);
    Ray r{{o[0], o[1], o[2], o[3]}, {d[0], d[1], d[2], d[3]}};
    std::vector<Intersection> xs;
    local_intersect(w, id, r, xs, w->ctx);
    int n = (int)xs.size();
    for (int i = 0; i < n && i < max; ++i) {
        t[i] = xs[i].t;
        obj[i] = xs[i].object;
        if (u) u[i] = xs[i].u;
        if (v) v[i] = xs[i].v;
    }
    return n;
}
void orc_color_at(orc_world* w, const double o[3], const double d[3], int remaining, double out[3]) {
    finalize(w);
    Ray r{tp(o, 1.0), tp(d, 0.0)};
    out3(color_at(w, r, remaining, w->ctx, 1u), out);
}
void orc_shade(orc_world* w, const double o[3], const double d[3], int n, const double* t, const int* obj,
               const double* u, const double* v, int hit_i, int remaining, int what, double out[3]) {
    finalize(w);
    Ray r{tp(o, 1.0), tp(d, 0.0)};
    std::vector<Intersection> xs = xs_from(n, t, obj, u, v);
    Computations c = prepare_computations(w, xs[hit_i], r, xs);
    Color res = BLACK;
    if (what == 0)
        res = shade_hit(w, c, remaining, w->ctx, 1u);
    else if (what == 1)
        res = reflected_color(w, c, remaining, w->ctx, 1u);
    else
        res = refracted_color(w, c, remaining, w->ctx, 1u);
    out3(res, out);
}
void orc_prepare_computations(orc_world* w, const double o[3], const double d[3], int n, const double* t,
                              const int* obj, const double* u, const double* v, int hit_i, double out[27]) {
    finalize(w);
    Ray r{tp(o, 1.0), tp(d, 0.0)};
    std::vector<Intersection> xs = xs_from(n, t, obj, u, v);
    Computations c = prepare_computations(w, xs[hit_i], r, xs);
    out[0] = c.t;
    out4(c.point, out + 1);
    out4(c.eyev, out + 5);
    out4(c.normalv, out + 9);
    out[13] = c.inside ? 1.0 : 0.0;
    out4(c.over_point, out + 14);
    out4(c.under_point, out + 18);
    // reflectv packed as 3 (w is always 0 for a reflected direction); n1, n2, schlick
    out[22] = c.reflectv.x;
    out[23] = c.reflectv.y;
    out[24] = c.reflectv.z;
    out[25] = c.n1;
    out[26] = c.n2;
    // schlick is exposed through orc_shade-free path: recompute on demand
}
int orc_is_shadowed(orc_world* w, const double p[3], const double lp[3]) {
    finalize(w);
    return is_shadowed(w, tp(p, 1.0), tp(lp, 1.0), w->ctx) ? 1 : 0;
}
void orc_lighting(orc_world* w, int obj, int light, const double p[3], const double e[3], const double n[3],
                  double in_shadow, double out[3]) {
    finalize(w);
    out3(lighting(w, obj, w->lights[light], tp(p, 1.0), tp(e, 0.0), tp(n, 0.0), in_shadow), out);
}
void orc_pattern_at(orc_world* w, int pattern, const double p[3], double out[3]) {
    out3(pattern_at(w, pattern, tp(p, 1.0), -1), out);
}
int orc_add_texture(orc_world* w, int width, int height, const uint8_t* rgba) {
    Texture t;
    t.width = (uint32_t)width;
    t.height = (uint32_t)height;
    t.rgba.assign(rgba, rgba + 4 * (size_t)width * (size_t)height);
    w->textures.push_back(std::move(t));
    return (int)w->textures.size() - 1;
}
void orc_texture_color(orc_world* w, int tex, double u, double v, uint8_t out[4]) {
    texture_color(w->textures[tex], u, v, out);
}
static int roots_out(const rootsq::Roots& r, double out[4]) {
    for (int i = 0; i < r.n; ++i) out[i] = r.v[i];
    return r.n;
}
int orc_find_roots_quartic(double a4, double a3, double a2, double a1, double a0, double out[4]) {
    return roots_out(rootsq::quartic(a4, a3, a2, a1, a0), out);
}
int orc_find_roots_cubic(double a3, double a2, double a1, double a0, double out[4]) {
    return roots_out(rootsq::cubic(a3, a2, a1, a0), out);
}
int orc_find_roots_quadratic(double a2, double a1, double a0, double out[4]) {
    return roots_out(rootsq::quadratic(a2, a1, a0), out);
}
void orc_uv_mapping(orc_world* w, int obj, const double p[3], double out[2]) {
    uv_mapping(w->objects[obj], tp(p, 1.0), out[0], out[1]);
}
void orc_normal_at(orc_world* w, int obj, const double p[3], double u, double v, double out[4]) {
    finalize(w);
    Intersection h{0.0, obj, u, v};
    out4(normal_at(w, obj, tp(p, 1.0), h), out);
}
void orc_world_to_object(orc_world* w, int obj, const double p[3], double out[4]) {
    out4(world_to_object(w, obj, tp(p, 1.0)), out);
}
void orc_normal_to_world(orc_world* w, int obj, const double n[3], double out[4]) {
    out4(normal_to_world(w, obj, tp(n, 0.0)), out);
}
void orc_group_aabb(orc_world* w, int id, double out[6]) {
    finalize(w);
    AABB b = get_aabb(w, id);
    out[0] = b.min.x;
    out[1] = b.min.y;
    out[2] = b.min.z;
    out[3] = b.max.x;
    out[4] = b.max.y;
    out[5] = b.max.z;
}

// camera.rs:41-63
void orc_camera_new(int64_t hsize, int64_t vsize, double fov, const double transform[16], orc_camera* c) {
    double half_view = std::tan(fov / 2.0);
    double aspect = (double)hsize / (double)vsize;
    double hw, hh;
    if (aspect >= 1.0) {
        hw = half_view;
        hh = half_view / aspect;
    } else {
        hw = half_view * aspect;
        hh = half_view;
    }
    c->hsize = hsize;
    c->vsize = vsize;
    c->field_of_view = fov;
    c->half_width = hw;
    c->half_height = hh;
    c->pixel_size = (hw * 2.0) / (double)hsize;
    if (transform)
        std::memcpy(c->transform, transform, sizeof(double) * 16);
    else
        to16(identity4(), c->transform);
}
// camera.rs:75-93
void orc_ray_for_pixel(const orc_camera* c, int64_t px, int64_t py, double o[4], double d[4]) {
    double xoffset = ((double)px + 0.5) * c->pixel_size;
    double yoffset = ((double)py + 0.5) * c->pixel_size;
    double wx = c->half_width - xoffset;
    double wy = c->half_height - yoffset;
    Matrix inv = inverse(from16(c->transform));
    Tuple pixel = mul_tuple(inv, point(wx, wy, -1.0));
    Tuple origin = mul_tuple(inv, point(0.0, 0.0, 0.0));
    Tuple direction = normalize(sub(pixel, origin));
    out4(origin, o);
    out4(direction, d);
}

// camera.rs:107-121 + 134-136 (rows y, x fastest).  Multi-threaded over rows (rayon par_bridge
// analogue); results do not depend on thread count.
int orc_render(orc_world* w, const orc_camera* c, int max_depth, uint64_t seed, int jitter_mode, int threads,
               int band, int band_stride, int band_phase, double* canvas, orc_stats* stats) {
    finalize(w);
    if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
    if (band <= 0) band = 1;
    if (band_stride <= 0) band_stride = 1;
    Matrix inv = inverse(from16(c->transform));
    std::vector<int64_t> rows;
    for (int64_t y = 0; y < c->vsize; ++y)
        if ((y / band) % band_stride == band_phase) rows.push_back(y);
    std::atomic<size_t> next{0};
    std::vector<orc_stats> st((size_t)threads);
    std::atomic<int> nan{0};
    auto worker = [&](int tid) {
        Ctx ctx;
        ctx.seed = seed;
        ctx.jitter_mode = jitter_mode;
        for (;;) {
            size_t ri = next.fetch_add(1);
            if (ri >= rows.size()) break;
            int64_t y = rows[ri];
            for (int64_t x = 0; x < c->hsize; ++x) {
                double xoffset = ((double)x + 0.5) * c->pixel_size;
                double yoffset = ((double)y + 0.5) * c->pixel_size;
                double wx = c->half_width - xoffset;
                double wy = c->half_height - yoffset;
                Tuple pixel = mul_tuple(inv, point(wx, wy, -1.0));
                Tuple origin = mul_tuple(inv, point(0.0, 0.0, 0.0));
                Ray r{origin, normalize(sub(pixel, origin))};
                ctx.sample = (uint64_t)(y * c->hsize + x);
                Color col = color_at(w, r, max_depth, ctx, 1u);
                double* px = canvas + 3 * (size_t)(y * c->hsize + x);
                px[0] = col.r;
                px[1] = col.g;
                px[2] = col.b;
            }
        }
        st[(size_t)tid] = ctx.st;
        if (ctx.nan) nan = 1;
    };
    std::vector<std::thread> pool;
    for (int i = 0; i < threads; ++i) pool.emplace_back(worker, i);
    for (auto& t : pool) t.join();
    if (stats) {
        orc_stats s{};
        for (auto& x : st) {
            s.rays += x.rays;
            s.shadow_rays += x.shadow_rays;
            s.sphere_tests += x.sphere_tests;
            s.plane_tests += x.plane_tests;
            s.tri_tests += x.tri_tests;
            s.group_tests += x.group_tests;
            s.group_hits += x.group_hits;
            s.cube_tests += x.cube_tests;
            s.cyl_tests += x.cyl_tests;
            s.cone_tests += x.cone_tests;
            s.csg_tests += x.csg_tests;
            s.shade_events += x.shade_events;
            s.nan_sorts += x.nan_sorts;
            s.torus_tests += x.torus_tests;
        }
        *stats = s;
    }
    return nan ? -1 : 0;
}

// canvas.rs:76-105 (before quantisation)
void orc_aa_average(const double* canvas, int64_t hsize, int64_t vsize, int aa, double* out) {
    double total = (double)(aa * aa);
    int64_t W = hsize / aa;
    for (int64_t y = 0; y < vsize; y += aa)
        for (int64_t x = 0; x < hsize; x += aa) {
            double r = 0.0, g = 0.0, b = 0.0;
            for (int dy = 0; dy < aa; ++dy)
                for (int dx = 0; dx < aa; ++dx) {
                    const double* p = canvas + 3 * (size_t)((y + dy) * hsize + (x + dx));
                    r += p[0];
                    g += p[1];
                    b += p[2];
                }
            double* o = out + 3 * (size_t)((y / aa) * W + (x / aa));
            o[0] = r / total;
            o[1] = g / total;
            o[2] = b / total;
        }
}
static uint8_t sat_u8(double v) {  // Rust `as u8`: NaN -> 0, saturate, truncate
    if (std::isnan(v) || v <= 0.0) return 0;
    if (v >= 255.0) return 255;
    return (uint8_t)v;
}
void orc_quantize(const double* avg, int64_t n, uint8_t* rgba) {
    for (int64_t i = 0; i < n; ++i) {
        rgba[4 * i + 0] = sat_u8(avg[3 * i + 0] * 255.0);
        rgba[4 * i + 1] = sat_u8(avg[3 * i + 1] * 255.0);
        rgba[4 * i + 2] = sat_u8(avg[3 * i + 2] * 255.0);
        rgba[4 * i + 3] = 255;
    }
}

}  // extern "C"

// =============================================================== OBJ (load_obj.rs + tobj 4.0.2)
// tobj (LoadOptions::default(): triangulate=false, single_index=false) semantics restated:
//  * `v`/`vn` components parsed as f32 (correctly rounded strtof), widened with `as f64`;
//  * `o`/`g` start a new model when faces are pending; models without faces are not emitted;
//  * faces keep their arity; face_arities is EMPTY when every face of a model is a triangle
//    (tobj 4.0.2 Mesh docs), in which case load_obj.rs:get_faces yields no faces at all.
// Parity for all-triangle meshes is unpinned (tobj not buildable here); teapot*.obj contain quads.
namespace {
struct ObjModel {
    std::vector<std::vector<long>> fv, fn;  // per face: position / normal indices (0-based)
    bool has_normals = false;
};
long obj_index(const std::string& s, size_t n) {
    long i = std::strtol(s.c_str(), nullptr, 10);
    return i < 0 ? (long)n + i : i - 1;
}
}  // namespace

extern "C" int orc_load_obj(orc_world* w, const char* path, int parent, const double mat7[7], int pattern) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return -1;
    std::stringstream ss;
    ss << f.rdbuf();
    std::string text = ss.str();
    for (auto& ch : text)
        if (ch == '\r') ch = '\n';
    std::vector<float> pos, nrm;
    std::vector<ObjModel> models;
    ObjModel cur;
    std::istringstream in(text);
    std::string line;
    while (std::getline(in, line)) {
        std::istringstream ls(line);
        std::string tag;
        if (!(ls >> tag)) continue;
        if (tag == "v" || tag == "vn") {
            std::string a, b, c;
            ls >> a >> b >> c;
            std::vector<float>& dst = (tag == "v") ? pos : nrm;
            dst.push_back(std::strtof(a.c_str(), nullptr));
            dst.push_back(std::strtof(b.c_str(), nullptr));
            dst.push_back(std::strtof(c.c_str(), nullptr));
        } else if (tag == "f") {
            std::vector<long> fv, fn;
            std::string tok;
            while (ls >> tok) {
                size_t s1 = tok.find('/');
                fv.push_back(obj_index(tok.substr(0, s1), pos.size() / 3));
                if (s1 != std::string::npos) {
                    size_t s2 = tok.find('/', s1 + 1);
                    if (s2 != std::string::npos && s2 + 1 < tok.size())
                        fn.push_back(obj_index(tok.substr(s2 + 1), nrm.size() / 3));
                }
            }
            if (fv.size() < 3) continue;  // points/lines ignored by default
            if (!fn.empty()) cur.has_normals = true;
            cur.fv.push_back(fv);
            cur.fn.push_back(fn);
        } else if (tag == "o" || tag == "g") {
            if (!cur.fv.empty()) models.push_back(cur);
            cur = ObjModel();
        }
    }
    if (!cur.fv.empty()) models.push_back(cur);
    if (models.empty()) return -2;  // load_obj.rs:130 panics "No models found"
    auto make_group = [&](const ObjModel& m, int par) -> int {  // load_obj.rs:100-122
        int g = orc_add_object(w, ORC_GROUP, par);
        bool all_tri = true;
        for (auto& fv : m.fv)
            if (fv.size() != 3) all_tri = false;
        if (all_tri) return g;  // face_arities empty -> get_faces() returns nothing
        for (size_t fi = 0; fi < m.fv.size(); ++fi) {
            const auto& fv = m.fv[fi];
            auto P = [&](size_t k) {
                long i = fv[k];
                double p[3] = {(double)pos[3 * i], (double)pos[3 * i + 1], (double)pos[3 * i + 2]};
                return std::vector<double>(p, p + 3);
            };
            for (size_t i = 1; i + 1 < fv.size(); ++i) {  // fan: (v0, vi, vi+1), load_obj.rs:57-76
                auto a = P(0), b = P(i), c = P(i + 1);
                int t;
                if (m.has_normals) {
                    const auto& fn = m.fn[fi];
                    auto N = [&](size_t k) {
                        long j = fn[k];
                        double n[3] = {(double)nrm[3 * j], (double)nrm[3 * j + 1], (double)nrm[3 * j + 2]};
                        return std::vector<double>(n, n + 3);
                    };
                    auto na = N(0), nb = N(i), nc = N(i + 1);
                    t = orc_add_smooth_triangle(w, g, a.data(), b.data(), c.data(), na.data(), nb.data(), nc.data());
                } else {
                    t = orc_add_triangle(w, g, a.data(), b.data(), c.data());
                }
                orc_set_material(w, t, mat7, pattern);  // material.clone() per triangle
            }
        }
        return g;
    };
    if (models.size() == 1) return make_group(models[0], parent);
    int master = orc_add_object(w, ORC_GROUP, parent);
    for (auto& m : models) make_group(m, master);
    return master;
}
