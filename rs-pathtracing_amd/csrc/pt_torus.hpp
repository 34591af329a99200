// pt_torus.hpp — Torus::ray_intersect (src/world/shapes/mod.rs:429-476) and
// the quartic solver it calls, solve_quantic_equation
// (src/algebra/equation.rs:17-67), host + device.
//
// The solver runs on num::Complex<f64> (crate `num` 0.4, Cargo.toml; no
// Cargo.lock, so the num-complex release is unpinned): every operation below
// restates num-complex 0.4's published arithmetic — Mul / Div of two complex
// numbers with the textbook formulas (Div through norm_sqr = c*c + d*d),
// real-on-complex operations componentwise, and the special-cased sqrt / cbrt
// (real and imaginary axes in closed form, otherwise from_polar of
// (hypot, atan2)).  Signed zeros matter there (is_sign_positive picks the
// branch of the root), and the expressions keep them as Rust computes them.
// Compiled with -ffp-contract=off like the rest of the path.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#ifndef PT_HD
#define PT_HD __host__ __device__ __forceinline__
#endif

namespace pt {
namespace torus {

struct Cx {
    double re, im;
};
PT_HD Cx cx(double re, double im) { return Cx{re, im}; }
PT_HD Cx real(double x) { return Cx{x, 0.0}; }  // From<f64>
PT_HD Cx add(Cx a, Cx b) { return cx(a.re + b.re, a.im + b.im); }
PT_HD Cx sub(Cx a, Cx b) { return cx(a.re - b.re, a.im - b.im); }
PT_HD Cx neg(Cx a) { return cx(-a.re, -a.im); }
PT_HD Cx mul(Cx a, Cx b) { return cx(a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re); }
PT_HD Cx div(Cx a, Cx b) {
    const double ns = b.re * b.re + b.im * b.im;
    const double re = a.re * b.re + a.im * b.im;
    const double im = a.im * b.re - a.re * b.im;
    return cx(re / ns, im / ns);
}
PT_HD Cx rmul(double k, Cx a) { return cx(k * a.re, k * a.im); }  // f64 * Complex
PT_HD Cx divr(Cx a, double k) { return cx(a.re / k, a.im / k); }  // Complex / f64
PT_HD Cx addr(Cx a, double k) { return cx(a.re + k, a.im); }      // Complex + f64
PT_HD bool sign_pos(double x) { return !std::signbit(x); }          // f64::is_sign_positive

// Complex::from_polar(r, theta), to_polar = (hypot(re, im), atan2(im, re))
PT_HD Cx from_polar(double r, double th) { return cx(r * cos(th), r * sin(th)); }

PT_HD Cx csqrt(Cx z) {
    if (z.im == 0.0) {
        if (sign_pos(z.re)) return cx(sqrt(z.re), z.im);
        const double im = sqrt(-z.re);
        return sign_pos(z.im) ? cx(0.0, im) : cx(0.0, -im);
    }
    if (z.re == 0.0) {
        const double x = sqrt(fabs(z.im) / 2.0);
        return sign_pos(z.im) ? cx(x, x) : cx(x, -x);
    }
    const double r = hypot(z.re, z.im), th = atan2(z.im, z.re);
    return from_polar(sqrt(r), th / 2.0);
}

PT_HD Cx ccbrt(Cx z) {
    if (z.im == 0.0) {
        if (sign_pos(z.re)) return cx(cbrt(z.re), z.im);
        const double re = cbrt(-z.re) / 2.0;
        const double im = sqrt(3.0) * re;
        return sign_pos(z.im) ? cx(re, im) : cx(re, -im);
    }
    if (z.re == 0.0) {
        const double im = cbrt(fabs(z.im)) / 2.0;
        const double re = sqrt(3.0) * im;
        return sign_pos(z.im) ? cx(re, im) : cx(re, -im);
    }
    const double r = hypot(z.re, z.im), th = atan2(z.im, z.re);
    return from_polar(cbrt(r), th / 3.0);
}

PT_HD bool approx_zero(double a) { return fabs(a - 0.0) < 1e-15; }  // approx_equal(a, 0.0)

// solve_quantic_equation (equation.rs:17-67), the four roots in its order.
PT_HD void solve_quartic(Cx a, Cx b, Cx c, Cx d, Cx e, Cx out[4]) {
    b = div(b, a);
    c = div(c, a);
    d = div(d, a);
    e = div(e, a);
    const Cx b2 = mul(b, b);
    const Cx alpha = sub(c, rmul(3.0 / 8.0, b2));
    const Cx beta = add(sub(divr(mul(b2, b), 8.0), divr(mul(b, c), 2.0)), d);
    const Cx gamma =
        add(sub(add(mul(rmul(-3.0 / 256.0, b2), b2), divr(mul(b2, c), 16.0)), divr(mul(b, d), 4.0)), e);
    const Cx alpha2 = mul(alpha, alpha);
    const Cx t = divr(neg(b), 4.0);
    if (approx_zero(beta.re) && approx_zero(beta.im)) {
        const Cx r = csqrt(sub(alpha2, rmul(4.0, gamma)));
        const Cx r1 = csqrt(divr(add(neg(alpha), r), 2.0));
        const Cx r2 = csqrt(divr(sub(neg(alpha), r), 2.0));
        out[0] = add(t, r1);
        out[1] = sub(t, r1);
        out[2] = add(t, r2);
        out[3] = sub(t, r2);
        return;
    }
    const Cx p = neg(add(divr(alpha2, 12.0), gamma));
    const Cx q = sub(add(divr(mul(neg(alpha2), alpha), 108.0), divr(mul(alpha, gamma), 3.0)), divr(mul(beta, beta), 8.0));
    const Cx r = add(divr(neg(q), 2.0), csqrt(add(divr(mul(q, q), 4.0), divr(mul(mul(p, p), p), 27.0))));
    const Cx u = ccbrt(r);
    Cx y = add(rmul(-5.0 / 6.0, alpha), u);
    if (approx_zero(u.re) && approx_zero(u.im)) y = sub(y, ccbrt(q));
    else y = sub(y, div(p, rmul(3.0, u)));
    const Cx w = csqrt(add(alpha, rmul(2.0, y)));
    const Cx s = add(rmul(3.0, alpha), rmul(2.0, y));
    const Cx bw = div(rmul(2.0, beta), w);
    const Cx r1 = csqrt(neg(add(s, bw)));
    const Cx r2 = csqrt(neg(sub(s, bw)));
    out[0] = add(t, divr(sub(w, r1), 2.0));
    out[1] = add(t, divr(add(w, r1), 2.0));
    out[2] = add(t, divr(sub(neg(w), r2), 2.0));
    out[3] = add(t, divr(add(neg(w), r2), 2.0));
}

// Torus::ray_intersect's distance (mod.rs:430-462) in object space: the
// smallest root whose imaginary part passes approx_equal(im, 0), then the
// range test.  R = radius, r = tube_radius.
PT_HD bool torus_t(double R, double r, double ox, double oy, double oz, double dx, double dy, double dz,
                   double min_t, double max_t, double *t_out) {
    const double t = 4.0 * R * R;
    const double g = t * (dx * dx + dy * dy);
    const double h = 2.0 * t * (ox * dx + oy * dy);
    const double i = t * (ox * ox + oy * oy);
    const double j = dx * dx + dy * dy + dz * dz;
    const double k = 2.0 * (ox * dx + oy * dy + oz * dz);
    const double l = ox * ox + oy * oy + oz * oz + R * R - r * r;
    const double a = j * j;
    const double b = 2.0 * j * k;
    const double c = 2.0 * j * l + k * k - g;
    const double d = 2.0 * k * l - h;
    const double e = l * l - i;
    Cx roots[4];
    solve_quartic(real(a), real(b), real(c), real(d), real(e), roots);
    double m = __builtin_inf();
    for (int q = 0; q < 4; q++)
        if (approx_zero(roots[q].im) && roots[q].re < m) m = roots[q].re;
    if (std::isinf(m) || m < min_t || m > max_t) return false;
    *t_out = m;
    return true;
}

}  // namespace torus
}  // namespace pt
