// rr_math.hpp — host-side f64 math with the reference's exact operation order.
//
// Restates src/tuple.rs:28-118 and src/matrix.rs:205-412,430-603: left-to-right sums,
// w-inclusive dot/magnitude, recursive cofactor inverse.  Compiled with -ffp-contract=off
// (rustc never fuses a*b+c), so results are bit-identical to the reference.
#pragma once
#include <cmath>

namespace rr {

struct Tup {
    double x, y, z, w;
};
inline Tup point(double x, double y, double z) { return {x, y, z, 1.0}; }
inline Tup vec(double x, double y, double z) { return {x, y, z, 0.0}; }
inline Tup operator+(const Tup& a, const Tup& b) { return {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
inline Tup operator-(const Tup& a, const Tup& b) { return {a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; }
inline Tup operator*(const Tup& a, double s) { return {a.x * s, a.y * s, a.z * s, a.w * s}; }
inline double dot(const Tup& a, const Tup& b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
inline double magnitude(const Tup& a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w); }
inline Tup normalize(const Tup& a) {
    double m = magnitude(a);
    return {a.x / m, a.y / m, a.z / m, a.w / m};
}
inline Tup cross(const Tup& a, const Tup& b) {
    return vec(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

// Square matrix of order N (2..4), row-major, as Matrix{rows, cols, data} (matrix.rs:20-25).
template <int N>
struct Mat {
    double m[N * N];
    double get(int r, int c) const { return m[r * N + c]; }
    void set(int r, int c, double v) { m[r * N + c] = v; }
};
using M4 = Mat<4>;

template <int N>
inline Mat<N - 1> submatrix(const Mat<N>& a, int row, int col) {  // matrix.rs:300-320
    Mat<N - 1> r{};
    int rr = 0;
    for (int i = 0; i < N; ++i) {
        if (i == row) continue;
        int cc = 0;
        for (int j = 0; j < N; ++j) {
            if (j == col) continue;
            r.set(rr, cc, a.get(i, j));
            ++cc;
        }
        ++rr;
    }
    return r;
}
inline double determinant(const Mat<2>& a) { return a.get(0, 0) * a.get(1, 1) - a.get(0, 1) * a.get(1, 0); }
template <int N>
inline double determinant(const Mat<N>& a);
template <int N>
inline double cofactor(const Mat<N>& a, int row, int col) {  // matrix.rs:330-345
    double minor = determinant(submatrix(a, row, col));
    return ((row + col) % 2 == 0) ? minor : -minor;
}
template <int N>
inline double determinant(const Mat<N>& a) {  // matrix.rs:285-296 (sum from 0.0)
    double det = 0.0;
    for (int i = 0; i < N; ++i) det += a.get(0, i) * cofactor(a, 0, i);
    return det;
}
inline M4 inverse(const M4& a) {  // matrix.rs:389-412
    double det = determinant(a);
    M4 r{};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double c = cofactor(a, i, j);
            r.set(j, i, c / det);
        }
    return r;
}
inline M4 identity() {
    M4 r{};
    for (int i = 0; i < 4; ++i) r.set(i, i, 1.0);
    return r;
}
inline M4 multiply(const M4& a, const M4& b) {  // matrix.rs:205-216
    M4 r{};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double sum = 0.0;
            for (int k = 0; k < 4; ++k) sum += a.get(i, k) * b.get(k, j);
            r.set(i, j, sum);
        }
    return r;
}
inline Tup mul(const M4& a, const Tup& t) {  // matrix.rs:234-240
    return {a.get(0, 0) * t.x + a.get(0, 1) * t.y + a.get(0, 2) * t.z + a.get(0, 3) * t.w,
            a.get(1, 0) * t.x + a.get(1, 1) * t.y + a.get(1, 2) * t.z + a.get(1, 3) * t.w,
            a.get(2, 0) * t.x + a.get(2, 1) * t.y + a.get(2, 2) * t.z + a.get(2, 3) * t.w,
            a.get(3, 0) * t.x + a.get(3, 1) * t.y + a.get(3, 2) * t.z + a.get(3, 3) * t.w};
}
inline M4 translate(double x, double y, double z) {
    M4 r = identity();
    r.set(0, 3, x);
    r.set(1, 3, y);
    r.set(2, 3, z);
    return r;
}
inline M4 scale(double x, double y, double z) {
    M4 r = identity();
    r.set(0, 0, x);
    r.set(1, 1, y);
    r.set(2, 2, z);
    return r;
}
inline M4 rotate(int axis, double a) {  // matrix.rs:463-510
    M4 r = identity();
    int i = axis == 0 ? 1 : 0, j = axis == 2 ? 1 : 2;
    if (axis == 1) {  // rotate_y: (0,0)=cos (0,2)=sin (2,0)=-sin (2,2)=cos
        r.set(0, 0, std::cos(a));
        r.set(0, 2, std::sin(a));
        r.set(2, 0, -std::sin(a));
        r.set(2, 2, std::cos(a));
    } else {  // rotate_x on (1,2), rotate_z on (0,1): (i,i)=cos (i,j)=-sin (j,i)=sin (j,j)=cos
        r.set(i, i, std::cos(a));
        r.set(i, j, -std::sin(a));
        r.set(j, i, std::sin(a));
        r.set(j, j, std::cos(a));
    }
    return r;
}
inline M4 shear(double xy, double xz, double yx, double yz, double zx, double zy) {
    M4 r = identity();
    r.set(0, 1, xy);
    r.set(0, 2, xz);
    r.set(1, 0, yx);
    r.set(1, 2, yz);
    r.set(2, 0, zx);
    r.set(2, 1, zy);
    return r;
}
inline M4 view_transform(Tup from, Tup to, Tup up) {  // matrix.rs:582-603
    Tup forward = normalize(to - from);
    Tup left = cross(forward, normalize(up));
    Tup true_up = cross(left, forward);
    M4 o{};
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
    return multiply(o, translate(-from.x, -from.y, -from.z));
}

}  // namespace rr
