// pt_funcs.hpp — the RayMarchingShape implicit functions (host + device).
//
// Heart, Sine, Star, DupinCyclide, HuntsSurface and Cushion
// (src/world/shapes/ray_marching.rs:121-520) are polynomials of degree <= 6 in
// (x, y, z).  Each is written ONCE, as a template over the number type, in the
// reference's operation order:
//   * double  — the value the reference computes (march steps, f at a point);
//   * P<D>    — exact polynomial arithmetic in the step index j along
//               p(j) = p0 + j*c, giving the coefficients of g(j) = f(p(j))
//               (degree <= 6) for the skipping march's sign proof;
//   * DM      — magnitude arithmetic with forward-mode gradients: every
//               operation on absolute values, so the result bounds |f| (the
//               rounding-error scale M) and |df/dx_k| (the drift of the
//               accumulated step points) over a block.
// Gradients (normals), the bounds and the uv are plain double code, again in
// the reference's order.
#pragma once
#include <cmath>
#include <cstdint>

#ifndef PT_HD
#define PT_HD __host__ __device__ __forceinline__
#endif

namespace pt {
namespace march {

enum FuncKind : int32_t { F_HEART = 0, F_SINE = 1, F_STAR = 2, F_DUPIN = 3, F_HUNTS = 4, F_CUSHION = 5 };

// Per-shape constants of a function, precomputed on the host exactly as the
// reference computes them inside shape_func (pure functions of the JSON
// parameters, so the values are identical).
struct FParams {
    int32_t func, pad;
    double k[4];  // Sine/Star: a | Dupin: a, b*b, c*d, d*d
    double radius;  // sphere_radius of the bound (not used by the Heart)
};

// ---------------------------------------------------------------- P<D>
template <int D>
struct P {
    double c[D + 1];
};
PT_HD constexpr int pmax(int a, int b) { return a > b ? a : b; }

template <int A, int B>
PT_HD P<pmax(A, B)> operator+(const P<A> &x, const P<B> &y) {
    P<pmax(A, B)> r;
#pragma unroll
    for (int i = 0; i <= pmax(A, B); i++) r.c[i] = (i <= A ? x.c[i] : 0.0) + (i <= B ? y.c[i] : 0.0);
    return r;
}
template <int A, int B>
PT_HD P<pmax(A, B)> operator-(const P<A> &x, const P<B> &y) {
    P<pmax(A, B)> r;
#pragma unroll
    for (int i = 0; i <= pmax(A, B); i++) r.c[i] = (i <= A ? x.c[i] : 0.0) - (i <= B ? y.c[i] : 0.0);
    return r;
}
template <int A, int B>
PT_HD P<A + B> operator*(const P<A> &x, const P<B> &y) {
    P<A + B> r;
#pragma unroll
    for (int i = 0; i <= A + B; i++) r.c[i] = 0.0;
#pragma unroll
    for (int i = 0; i <= A; i++)
#pragma unroll
        for (int j = 0; j <= B; j++) r.c[i + j] += x.c[i] * y.c[j];
    return r;
}
template <int A>
PT_HD P<A> operator*(double k, const P<A> &x) {
    P<A> r;
#pragma unroll
    for (int i = 0; i <= A; i++) r.c[i] = k * x.c[i];
    return r;
}
template <int A>
PT_HD P<A> operator*(const P<A> &x, double k) {
    return k * x;
}
template <int A>
PT_HD P<A> operator-(const P<A> &x, double k) {
    P<A> r = x;
    r.c[0] = r.c[0] - k;
    return r;
}
template <int A>
PT_HD P<A> operator+(const P<A> &x, double k) {
    P<A> r = x;
    r.c[0] = r.c[0] + k;
    return r;
}
template <int A>
PT_HD P<6> widen6(const P<A> &x) {
    P<6> r;
#pragma unroll
    for (int i = 0; i <= 6; i++) r.c[i] = i <= A ? x.c[i] : 0.0;
    return r;
}
PT_HD P<6> widen6(const P<6> &x) { return x; }

// ---------------------------------------------------------------- DM
// Magnitude + gradient-magnitude dual: (|v|, |dv/dx|, |dv/dy|, |dv/dz|) bounds.
struct DM {
    double v, gx, gy, gz;
};
PT_HD DM operator+(const DM &a, const DM &b) { return {a.v + b.v, a.gx + b.gx, a.gy + b.gy, a.gz + b.gz}; }
PT_HD DM operator-(const DM &a, const DM &b) { return a + b; }
PT_HD DM operator*(const DM &a, const DM &b) {
    return {a.v * b.v, a.v * b.gx + b.v * a.gx, a.v * b.gy + b.v * a.gy, a.v * b.gz + b.v * a.gz};
}
PT_HD DM operator*(double k, const DM &a) {
    const double m = fabs(k);
    return {m * a.v, m * a.gx, m * a.gy, m * a.gz};
}
PT_HD DM operator*(const DM &a, double k) { return k * a; }
PT_HD DM operator-(const DM &a, double k) { return {a.v + fabs(k), a.gx, a.gy, a.gz}; }
PT_HD DM operator+(const DM &a, double k) { return {a.v + fabs(k), a.gx, a.gy, a.gz}; }

// ------------------------------------------------------- the functions
// Heart::shape_func (ray_marching.rs:147-155)
template <class T>
PT_HD auto f_heart(const T &x, const T &y, const T &z) {
    auto x2 = x * x;
    auto y2 = y * y;
    auto z2 = z * z;
    auto z3 = z2 * z;
    auto a = x2 + (9.0 / 4.0) * y2 + z2 - 1.0;
    return a * a * a - x2 * z3 - (9.0 / 80.0) * y2 * z3;
}
// Sine::shape_func (:202-210)
template <class T>
PT_HD auto f_sine(const FParams &F, const T &x, const T &y, const T &z) {
    const double a = F.k[0];
    return a * a * (x - y - z) * (x + y - z) * (x - y + z) * (x + y + z) + 4.0 * x * x * y * y * z * z;
}
// Star::shape_func (:258-264)
template <class T>
PT_HD auto f_star(const FParams &F, const T &x, const T &y, const T &z) {
    auto x2 = x * x;
    auto y2 = y * y;
    auto z2 = z * z;
    auto c = x2 + y2 + z2 - 1.0;
    return F.k[0] * (x2 * y2 + x2 * z2 + y2 * z2) + (c * c * c);
}
// DupinCyclide::shape_func (:339-344): k = a, b*b, c*d, d*d
template <class T>
PT_HD auto f_dupin(const FParams &F, const T &x, const T &y, const T &z) {
    const double b2 = F.k[1];
    auto e = x * x + y * y + z * z + b2 - F.k[3];
    auto f = F.k[0] * x - F.k[2];
    return e * e - 4.0 * (f * f + b2 * y * y);
}
// HuntsSurface::shape_func (:399-406)
template <class T>
PT_HD auto f_hunts(const T &x, const T &y, const T &z) {
    auto x2 = x * x;
    auto y2 = y * y;
    auto z2 = z * z;
    auto a = x2 + y2 + z2 - 13.0;
    auto b = 3.0 * x2 + y2 - 4.0 * z2 - 12.0;
    return 4.0 * a * a * a + 27.0 * b * b;
}
// Cushion::shape_func (:456-472)
template <class T>
PT_HD auto f_cushion(const T &x, const T &y, const T &z) {
    auto x2 = x * x;
    auto y2 = y * y;
    auto z2 = z * z;
    auto a = x2 - z;
    return z2 * x2 - z2 * z2 - 2.0 * z * x2 + 2.0 * z * z2 + x2 - z2 - a * a - y2 * y2 - 2.0 * x2 * y2 - y2 * z2 +
           2.0 * y2 * z + y2;
}

// f at a point, the reference's f64 value
PT_HD double shape_f(const FParams &F, double x, double y, double z) {
    switch (F.func) {
    case F_SINE: return f_sine(F, x, y, z);
    case F_STAR: return f_star(F, x, y, z);
    case F_DUPIN: return f_dupin(F, x, y, z);
    case F_HUNTS: return f_hunts(x, y, z);
    case F_CUSHION: return f_cushion(x, y, z);
    default: return f_heart(x, y, z);
    }
}

// g(j) = f(p0 + j*c): coefficients g[0..6] (degree <= 6 for every function)
PT_HD void shape_poly(const FParams &F, double x0, double y0, double z0, double cx, double cy, double cz,
                      double *g) {
    const P<1> x{{x0, cx}}, y{{y0, cy}}, z{{z0, cz}};
    P<6> r;
    switch (F.func) {
    case F_SINE: r = widen6(f_sine(F, x, y, z)); break;
    case F_STAR: r = widen6(f_star(F, x, y, z)); break;
    case F_DUPIN: r = widen6(f_dupin(F, x, y, z)); break;
    case F_HUNTS: r = widen6(f_hunts(x, y, z)); break;
    case F_CUSHION: r = widen6(f_cushion(x, y, z)); break;
    default: r = widen6(f_heart(x, y, z)); break;
    }
#pragma unroll
    for (int k = 0; k < 7; k++) g[k] = r.c[k];
}

// magnitude bound of f and of its gradient over the box |x| <= xm, ...
PT_HD DM shape_mag(const FParams &F, double xm, double ym, double zm) {
    const DM x{xm, 1.0, 0.0, 0.0}, y{ym, 0.0, 1.0, 0.0}, z{zm, 0.0, 0.0, 1.0};
    switch (F.func) {
    case F_SINE: return f_sine(F, x, y, z);
    case F_STAR: return f_star(F, x, y, z);
    case F_DUPIN: return f_dupin(F, x, y, z);
    case F_HUNTS: return f_hunts(x, y, z);
    case F_CUSHION: return f_cushion(x, y, z);
    default: return f_heart(x, y, z);
    }
}

// ShapeFunction::gradient (the normal), reference order
PT_HD void shape_gradient(const FParams &F, double px, double py, double pz, double *n) {
    switch (F.func) {
    case F_SINE: {  // :227-238
        double x2 = px * px, y2 = py * py, z2 = pz * pz;
        double a2 = F.k[0] * F.k[0];
        n[0] = 4.0 * px * (a2 * (x2 - y2 - z2) + 2.0 * y2 * z2);
        n[1] = 8.0 * x2 * py * z2 - 4.0 * a2 * py * (x2 - y2 + z2);
        n[2] = 8.0 * x2 * y2 * pz - 4.0 * a2 * pz * (x2 + y2 - z2);
        return;
    }
    case F_STAR: {  // :279-289
        double x2 = px * px, y2 = py * py, z2 = pz * pz;
        double c = x2 + y2 + z2 - 1.0;
        const double a = F.k[0];
        n[0] = 2.0 * a * px * (y2 + z2) + 6.0 * px * c * c;
        n[1] = 2.0 * a * py * (x2 + z2) + 6.0 * py * c * c;
        n[2] = 2.0 * a * pz * (x2 + y2) + 6.0 * pz * c * c;
        return;
    }
    case F_DUPIN: {  // :359-367: e = 4 (x.x + y.y + z.z + b2 - d*d)
        const double b2 = F.k[1];
        double e = 4.0 * (px * px + py * py + pz * pz + b2 - F.k[3]);
        n[0] = e * px - 8.0 * F.k[0] * (F.k[0] * px - F.k[2]);
        n[1] = e * py - 8.0 * b2 * py;
        n[2] = e * pz;
        return;
    }
    case F_HUNTS: {  // :421-433 (b as the reference writes it here: 4 (z2 + 3))
        double x2 = px * px, y2 = py * py, z2 = pz * pz;
        double a = x2 + y2 + z2 - 13.0;
        double b = 3.0 * x2 + y2 - 4.0 * (z2 + 3.0);
        n[0] = 24.0 * px * a * a + 324.0 * px * b;
        n[1] = 12.0 * py * (2.0 * a * a + 9.0 * b);
        n[2] = 24.0 * pz * (a * a - 18.0 * b);
        return;
    }
    case F_CUSHION: {  // :487-496
        double x2 = px * px, y2 = py * py, z2 = pz * pz;
        n[0] = 2.0 * px * (-2.0 * x2 - 2.0 * y2 + z2 + 1.0);
        n[1] = -2.0 * py * (2.0 * x2 + 2.0 * y2 + z2 - 2.0 * pz - 1.0);
        n[2] = 2.0 * pz * (x2 - 2.0 * z2 + 3.0 * pz - 2.0) - 2.0 * py * (pz - 1.0);
        return;
    }
    default: {  // Heart :157-168 (the 27/40 coefficient kept as in the reference)
        double a = px * px + (9.0 / 4.0) * py * py + pz * pz - 1.0;
        a = 3.0 * a * a;
        double z2 = pz * pz;
        double z3 = z2 * pz;
        n[0] = 2.0 * px * (a - z3);
        n[1] = (9.0 / 2.0) * py * (a - 0.05 * z3);
        n[2] = 2.0 * pz * (a - pz * (1.5 * px * px + (27.0 / 40.0) * py * py));
        return;
    }
    }
}

// solve_quadratic_equation (algebra/equation.rs:5-15) on (a, half_b, c), then
// the (max(x1, 0), max(x2, 0)) interval; false on a miss.
PT_HD bool bound_interval(double a, double hb, double c, double *start, double *end) {
    double disc = hb * hb - a * c;
    if (disc < 0.0) return false;
    double x1, x2;
    if (disc == 0.0) {
        x1 = -hb;
        x2 = -hb;
    } else {
        double sq = sqrt(disc);
        x1 = (-hb - sq) / a;
        x2 = (-hb + sq) / a;
    }
    if (x1 < 0.0 && x2 < 0.0) return false;
    *start = fmax(x1, 0.0);
    *end = fmax(x2, 0.0);
    return true;
}

// ShapeFunction::intersect_bound: the Heart's fixed ellipsoid (:135-145, the
// JSON sphere_radius ignored), the others' sphere of sphere_radius.
PT_HD bool shape_bound(const FParams &F, double ox, double oy, double oz, double dx, double dy, double dz,
                       double *start, double *end) {
    if (F.func == F_HEART) {
        const double rx = 1.45, ry = 1.45 / 2.05, rz = 1.45;
        double oox = ox / rx, ooy = oy / ry, ooz = oz / rz;
        double ddx = dx / rx, ddy = dy / ry, ddz = dz / rz;
        return bound_interval(ddx * ddx + ddy * ddy + ddz * ddz, ddx * oox + ddy * ooy + ddz * ooz,
                              oox * oox + ooy * ooy + ooz * ooz - 1.0, start, end);
    }
    const double r = F.radius;
    return bound_interval(dx * dx + dy * dy + dz * dz, dx * ox + dy * oy + dz * oz,
                          ox * ox + oy * oy + oz * oz - r * r, start, end);
}

// Compile-time function kind: FK >= 0 instantiates one function (a scene
// whose marched shapes are all Hearts runs the Heart-only build: no dispatch,
// no unused constants in registers); FK = F_ANY dispatches on F.func.
constexpr int F_ANY = -1;
// F_NONE: the scene has no ray-marched shape (the bounce build for large BVHs without one, C5): the helpers
// below are never reached at run time and compile to nothing
constexpr int F_NONE = -2;

template <int FK>
PT_HD double shape_f_k(const FParams &F, double x, double y, double z) {
    if constexpr (FK == F_NONE) return 0.0;
    else if constexpr (FK == F_HEART) return f_heart(x, y, z);
    else return shape_f(F, x, y, z);
}
template <int FK>
PT_HD void shape_poly_k(const FParams &F, double x0, double y0, double z0, double cx, double cy, double cz,
                        double *g) {
    if constexpr (FK == F_HEART) {
        const P<1> x{{x0, cx}}, y{{y0, cy}}, z{{z0, cz}};
        const P<6> r = f_heart(x, y, z);
#pragma unroll
        for (int k = 0; k < 7; k++) g[k] = r.c[k];
    } else {
        shape_poly(F, x0, y0, z0, cx, cy, cz, g);
    }
}
template <int FK>
PT_HD DM shape_mag_k(const FParams &F, double xm, double ym, double zm) {
    if constexpr (FK == F_HEART) {
        const DM x{xm, 1.0, 0.0, 0.0}, y{ym, 0.0, 1.0, 0.0}, z{zm, 0.0, 0.0, 1.0};
        return f_heart(x, y, z);
    } else {
        return shape_mag(F, xm, ym, zm);
    }
}
template <int FK>
PT_HD bool shape_bound_k(const FParams &F, double ox, double oy, double oz, double dx, double dy, double dz,
                         double *start, double *end) {
    if constexpr (FK == F_NONE) {
        *start = *end = 0.0;
        return false;
    } else if constexpr (FK == F_HEART) {
        FParams H{};
        H.func = F_HEART;
        return shape_bound(H, ox, oy, oz, dx, dy, dz, start, end);
    } else {
        return shape_bound(F, ox, oy, oz, dx, dy, dz, start, end);
    }
}
template <int FK>
PT_HD void shape_gradient_k(const FParams &F, double px, double py, double pz, double *n) {
    if constexpr (FK == F_NONE) {
        n[0] = n[1] = n[2] = 0.0;
    } else if constexpr (FK == F_HEART) {
        FParams H{};
        H.func = F_HEART;
        shape_gradient(H, px, py, pz, n);
    } else {
        shape_gradient(F, px, py, pz, n);
    }
}

}  // namespace march
}  // namespace pt
