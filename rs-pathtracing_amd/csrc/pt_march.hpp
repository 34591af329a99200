// pt_march.hpp — exact, skipping RayMarchingShape march (host + device).
//
// The reference march (src/world/shapes/ray_marching.rs:20-74) walks
//   t += step; p += step*dir; next = f(p)
// thousands of times per ray (0.01 world units per step), stopping at the
// first sign change of f (then 3 refinement passes with step *= -0.01).  This
// file returns the SAME t, bit for bit, with far less work:
//
//  1. Closed-form accumulation.  Inside one binade [2^e, 2^(e+1)) every double
//     is an integer multiple of u = 2^(e-52), so fl(x + c) = x + R*u with
//     R = rint(c/u), as long as x + c stays in the binade and c/u is not a
//     round-half-even tie.  With X = x/u an exact int64, B repeated additions
//     are X + B*R: exact, O(1) (a round-half-even tie is exact too, from an
//     even X).  Blocks stop where any of px, py, pz, t would leave its binade;
//     a coordinate near 0 falls back to one literal step.
//  2. Sign proof.  Within such a block the step points are exactly
//     p_j = p_k + j*ch, so heart_f along them is an exact degree-6 polynomial
//     in j.  Its Taylor coefficients, with a rigorous bound on every rounding
//     error (coefficients and the reference's own evaluation) plus the 1e-15
//     approx_equal threshold, prove when none of the B steps can stop the
//     pass; the march then jumps to p_{k+B} and evaluates f there exactly.
// Everything else (range checks, pass structure, final t test) is the
// reference's.  Compiled with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#ifndef PT_HD
#define PT_HD __host__ __device__ __forceinline__
#endif

namespace pt {
namespace march {

// Heart::shape_func (ray_marching.rs:147-155)
PT_HD double heart_f(double px, double py, double pz) {
    double x2 = px * px;
    double y2 = py * py;
    double z2 = pz * pz;
    double z3 = z2 * pz;
    double a = x2 + (9.0 / 4.0) * y2 + z2 - 1.0;
    return a * a * a - x2 * z3 - (9.0 / 80.0) * y2 * z3;
}

// Heart::intersect_bound (:135-145) + solve_quadratic_equation (algebra/equation.rs:5-15)
PT_HD bool heart_bound(double ox, double oy, double oz, double dx, double dy, double dz, double *start,
                       double *end) {
    const double rx = 1.45, ry = 1.45 / 2.05, rz = 1.45;
    double oox = ox / rx, ooy = oy / ry, ooz = oz / rz;
    double ddx = dx / rx, ddy = dy / ry, ddz = dz / rz;
    double a = ddx * ddx + ddy * ddy + ddz * ddz;
    double hb = ddx * oox + ddy * ooy + ddz * ooz;
    double c = oox * oox + ooy * ooy + ooz * ooz - 1.0;
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

// ------------------------------------------------------- closed-form adds
struct Lin {
    int64_t X = 0, R = 0;  // value = X * 2^sh, step = R * 2^sh
    int sh = 0;            // e - 52
    bool frozen = false;   // c == 0: fl(x + 0) = x forever
};

constexpr int64_t BIG = (int64_t)1 << 40;
PT_HD int64_t imin(int64_t a, int64_t b) { return a < b ? a : b; }

// Largest B such that the first B additions fl(x_j + c), j = 0..B-1, are all
// x_j + R*u exactly; 0 if the closed form does not apply here.
PT_HD int64_t lin_init(double x, double c, Lin *L) {
    L->frozen = false;
    if (c == 0.0) {
        L->frozen = true;
        return BIG;
    }
    if (!(x != 0.0) || !(fabs(x) < 1e300) || !(fabs(c) < 1e300)) return 0;  // zero, inf, NaN
    int e = ilogb(x);
    if (e < -960) return 0;  // stay clear of subnormals
    double q = ldexp(c, 52 - e);  // c / u, exact (power-of-two scaling)
    if (!(fabs(q) < 4.0e15)) return 0;  // |c| >= 2^52 u: leaves the binade at once
    int64_t X = (int64_t)ldexp(x, 52 - e);
    double qf = floor(q);
    int64_t R;
    if (q - qf == 0.5) {
        // Round-half-even tie: x + c sits halfway between two grid points and
        // rounds to the even one.  From an even X the sum lands on an even X
        // again, advancing by the even one of {k, k+1} every step.
        if (X & 1) return 0;  // one literal step first makes X even
        int64_t k = (int64_t)qf;
        R = (k & 1) ? k + 1 : k;
    } else {
        R = (int64_t)rint(q);
    }
    int64_t C = (int64_t)ceil(fabs(q));
    const int64_t lo = ((int64_t)1 << 52) + C + 1, hi = ((int64_t)1 << 53) - C - 1;
    int64_t A = X >= 0 ? X : -X, Rs = X >= 0 ? R : -R;
    if (A < lo || A > hi) return 0;
    L->X = X;
    L->R = R;
    L->sh = e - 52;
    if (Rs == 0) return BIG;
    // room = floor(span / |Rs|) without a (software) int64 division: both are
    // integers < 2^53, exact in f64; the rounded quotient is off by at most one.
    int64_t span = Rs > 0 ? hi - A : A - lo, step = Rs > 0 ? Rs : -Rs;
    int64_t room = (int64_t)floor((double)span / (double)step);
    if (room * step > span) room--;
    else if ((room + 1) * step <= span) room++;
    return room + 1 < BIG ? room + 1 : BIG;
}

PT_HD double lin_at(const Lin &L, double x, int64_t j) {
    if (L.frozen) return x;
    return ldexp((double)(L.X + j * L.R), L.sh);
}

// x after n literal additions fl(x + c), exactly, across any number of binade
// edges: closed form inside each binade, literal adds in the thin zone at an
// edge (and near zero).  Each coordinate's sequence is independent of the
// others, so p, t can be advanced separately.
PT_HD double advance(double x, double c, int64_t n) {
    while (n > 0) {
        Lin L;
        int64_t room = lin_init(x, c, &L);
        if (room >= 2) {
            int64_t k = room < n ? room : n;
            x = lin_at(L, x, k);
            n -= k;
        } else {
            x = x + c;
            n--;
        }
    }
    return x;
}

// Largest b (<= cap) such that t_0 .. t_{b-1} of t_{j+1} = fl(t_j + s) all lie
// in [start, end] (the reference's check before each step), given t_0 does.
PT_HD int64_t steps_in_range(double t, double s, double start, double end, int64_t cap) {
    double lim = s > 0.0 ? end : start;
    double est = (lim - t) / s;  // >= 0
    int64_t k = est >= (double)cap ? cap : (int64_t)est;  // candidate last index
    auto inside = [&](int64_t j) {
        double tj = advance(t, s, j);
        return !(tj > end || tj < start);
    };
    while (k > 0 && !inside(k)) k--;
    while (k + 1 < cap && inside(k + 1)) k++;
    return k + 1;
}

// ------------------------------------------------ polynomial sign proof
// Inside a block every coordinate advances by an exact constant (R*u), so the
// step points are exactly p_j = p0 + j*ch (ch = per-step displacement, exact),
// and heart_f along them is the degree-6 polynomial g(j) = f(p0 + j*ch) of the
// exact arithmetic.  heart_poly computes its coefficients; the bound below
// proves that every f64 evaluation of heart_f at p_1..p_B keeps one sign and
// stays clear of the 1e-15 stop.
struct Poly {
    double g[7];                       // coefficients of g(j)
    double ax, ay, az, cx, cy, cz;     // |p0|, |ch| for the magnitude bound
};

PT_HD void heart_poly(double x, double y, double z, double cx, double cy, double cz, Poly *P) {
    double x2[3] = {x * x, 2.0 * x * cx, cx * cx};
    double y2[3] = {y * y, 2.0 * y * cy, cy * cy};
    double z2[3] = {z * z, 2.0 * z * cz, cz * cz};
    double z3[4] = {z2[0] * z, z2[0] * cz + z2[1] * z, z2[1] * cz + z2[2] * z, z2[2] * cz};
    double A[3] = {x2[0] + 2.25 * y2[0] + z2[0] - 1.0, x2[1] + 2.25 * y2[1] + z2[1], x2[2] + 2.25 * y2[2] + z2[2]};
    double A2[5] = {A[0] * A[0], 2.0 * A[0] * A[1], A[1] * A[1] + 2.0 * A[0] * A[2], 2.0 * A[1] * A[2], A[2] * A[2]};
    double A3[7];
    A3[0] = A2[0] * A[0];
    A3[1] = A2[0] * A[1] + A2[1] * A[0];
    A3[2] = A2[0] * A[2] + A2[1] * A[1] + A2[2] * A[0];
    A3[3] = A2[1] * A[2] + A2[2] * A[1] + A2[3] * A[0];
    A3[4] = A2[2] * A[2] + A2[3] * A[1] + A2[4] * A[0];
    A3[5] = A2[3] * A[2] + A2[4] * A[1];
    A3[6] = A2[4] * A[2];
    const double K = 9.0 / 80.0;  // the reference's constant, as rounded
    for (int k = 0; k < 7; k++) {
        double pk = 0.0, qk = 0.0;
        for (int i = 0; i < 3; i++) {
            int j = k - i;
            if (j >= 0 && j < 4) {
                pk += x2[i] * z3[j];
                qk += y2[i] * z3[j];
            }
        }
        P->g[k] = A3[k] - pk - K * qk;
    }
    P->ax = fabs(x);
    P->ay = fabs(y);
    P->az = fabs(z);
    P->cx = fabs(cx);
    P->cy = fabs(cy);
    P->cz = fabs(cz);
}

// True if sgn * (f64 heart_f at p_j) > 1e-15 for every j in [1, b] (so neither
// the approx_equal stop nor a sign change can fire inside the block).
//  * margin: 1e-15 + 256 eps M(b), where M(b) bounds the magnitudes of all
//    monomials over the block; it covers the coefficients' rounding, the
//    Horner evaluation below and the reference's own f64 evaluation of f.
//  * monotone form: if |g1| exceeds the derivative's other terms over [0, b]
//    (with the same kind of margin), g is monotone there and its extreme on
//    [1, b] is g(b) (decreasing) or at least g(0) (increasing);
//  * otherwise the absolute Taylor bound g0 - sum_k |g_k| b^k.
PT_HD double poly_mag(const Poly &P, double b) {
    double xm = P.ax + P.cx * b, ym = P.ay + P.cy * b, zm = P.az + P.cz * b;
    double x2 = xm * xm, y2 = ym * ym, z2 = zm * zm, z3 = z2 * zm;
    double am = x2 + 2.25 * y2 + z2 + 1.0;
    return am * am * am + x2 * z3 + 0.1125 * y2 * z3;
}

PT_HD bool poly_sign_definite(const Poly &P, double b, double sgn) {
    const double e256 = 2.8421709430404007e-14;  // 256 * 2^-53
    double mag = poly_mag(P, b);
    // The step points are p_j = p0 + j*c + delta_j with |delta_j,k| <= j*ulp_k/2
    // (each literal add rounds once): add max|grad f| . |delta| over the block.
    double xm = P.ax + P.cx * b, ym = P.ay + P.cy * b, zm = P.az + P.cz * b;
    double x2 = xm * xm, y2 = ym * ym, z2 = zm * zm, z3 = z2 * zm;
    double am = x2 + 2.25 * y2 + z2 + 1.0, am2 = am * am;
    double gx = 6.0 * xm * am2 + 2.0 * xm * z3;
    double gy = 13.5 * ym * am2 + 0.225 * ym * z3;
    double gz = 6.0 * zm * am2 + 3.0 * x2 * z2 + 0.3375 * y2 * z2;
    double drift = b * 2.3e-16 * (gx * xm + gy * ym + gz * zm);  // ulp(v)/2 <= 2^-53 |v| (2.3e-16 > 2^-52)
    double margin = 1e-15 + e256 * mag + drift;
    double g0 = sgn * P.g[0], g1 = sgn * P.g[1];
    if (g0 <= margin) return false;
    // derivative remainder sum_{k>=2} k |g_k| b^(k-1)
    double d1 = 0.0;
    for (int k = 6; k >= 2; k--) d1 = d1 * b + k * fabs(P.g[k]);
    d1 *= b;
    if (fabs(g1) - d1 > e256 * 6.0 * mag / b) {
        if (g1 > 0.0) return true;  // increasing away from zero: min is g(0+) > g0 > margin
        double gb = 0.0;            // decreasing: the minimum is g(b)
        for (int k = 6; k >= 0; k--) gb = gb * b + sgn * P.g[k];
        return gb > margin;
    }
    double d = 0.0;
    for (int k = 6; k >= 1; k--) d = (d + fabs(P.g[k])) * b;
    return g0 - d > margin;
}

// Predicted first crossing (in steps) from the quadratic part of sgn*g; the
// search starts there and the proof decides.
PT_HD double poly_root_guess(const Poly &P, double sgn, double cap) {
    double L = sgn * P.g[0], S = sgn * P.g[1], Q = sgn * P.g[2];
    if (L <= 0.0) return 1.0;
    if (Q == 0.0) return S < 0.0 ? fmin(cap, L / -S) : cap;
    double disc = S * S - 4.0 * Q * L;
    if (disc < 0.0) return cap;  // no real root of the quadratic
    double sq = sqrt(disc);
    double r1 = (-S - sq) / (2.0 * Q), r2 = (-S + sq) / (2.0 * Q);
    double lo = fmin(r1, r2), hi = fmax(r1, r2);
    double r = lo > 0.0 ? lo : (hi > 0.0 ? hi : cap);
    return fmin(cap, r);
}

// ------------------------------------------------------- the march
struct MarchStats {
    uint32_t steps, blocks, tries;
};

// Resumable form of RayMarchingShape::ray_intersect (ray_marching.rs:20-74) so
// a lane can march a few iterations per pass of the kernel's main loop while
// the other lanes of its wave keep tracing.
struct MarchState {
    double t, px, py, pz, r, s, start, end, dx, dy, dz;
    int pass, passes;
};
enum MarchStatus : int { M_RUNNING = 0, M_DONE = 1, M_MISS = 2 };

// Bound test and start of the march; false if the ray misses the bound.
PT_HD bool march_begin(double step0, int passes, double ox, double oy, double oz, double dx, double dy, double dz,
                       MarchState *m) {
    double start, end;
    if (!heart_bound(ox, oy, oz, dx, dy, dz, &start, &end)) return false;
    m->start = start;
    m->end = end;
    m->s = step0;
    m->t = start;
    m->px = ox + dx * start;
    m->py = oy + dy * start;
    m->pz = oz + dz * start;
    m->r = heart_f(m->px, m->py, m->pz);
    m->dx = dx;
    m->dy = dy;
    m->dz = dz;
    m->pass = 0;
    m->passes = passes;
    return true;
}

// One iteration of the march loop: a proven jump, or one literal step (after a
// failed proof).  M_DONE: the passes ended (the caller applies the final
// t-in-[min_t, max_t] test); M_MISS: t left [start, end].
template <bool STATS>
PT_HD int march_iter(MarchState &m, MarchStats *st) {
    if (m.pass >= m.passes) return M_DONE;
    if (m.t > m.end || m.t < m.start) return M_MISS;
    double s = m.s;
    double cx = m.dx * s, cy = m.dy * s, cz = m.dz * s;
    // ---- try to jump a block of b steps (exact advance + sign proof)
    if (m.r != 0.0) {
        int64_t bmax = steps_in_range(m.t, s, m.start, m.end, (int64_t)1 << 24);
        if (bmax >= 2) {
            Poly P;
            heart_poly(m.px, m.py, m.pz, cx, cy, cz, &P);
            if (STATS) st->tries++;
            // largest provable block: start at the predicted crossing, drop by
            // 4x until proven, then refine upward (gallop / bisect)
            double sgn = m.r > 0.0 ? 1.0 : -1.0;
            double guess = poly_root_guess(P, sgn, (double)bmax);
            int64_t good = 0, bad = bmax + 1;
            int64_t b = (int64_t)(guess * 0.999);
            b = b < 2 ? 2 : (b > bmax ? bmax : b);
            int evals = 0;
            while (b >= 2 && evals < 10) {
                evals++;
                if (poly_sign_definite(P, (double)b, sgn)) {
                    good = b;
                    break;
                }
                bad = b;
                b >>= 2;
            }
            while (good >= 2 && evals < 10 && bad - good > 1 + good / 16) {
                b = bad > bmax ? (2 * good > bmax ? bmax : 2 * good) : good + (bad - good) / 2;
                if (b <= good || b >= bad) break;
                evals++;
                if (poly_sign_definite(P, (double)b, sgn)) good = b;
                else bad = b;
            }
            if (good >= 2) {
                m.t = advance(m.t, s, good);
                m.px = advance(m.px, cx, good);
                m.py = advance(m.py, cy, good);
                m.pz = advance(m.pz, cz, good);
                m.r = heart_f(m.px, m.py, m.pz);
                if (STATS) st->blocks++;
                return M_RUNNING;
            }
        }
    }
    // ---- one literal step (ray_marching.rs:37-51)
    m.t += s;
    m.px += cx;
    m.py += cy;
    m.pz += cz;
    double next = heart_f(m.px, m.py, m.pz);
    if (STATS) st->steps++;
    if (fabs(next - 0.0) < 1e-15) {  // approx_equal(next, 0.0): break 'outer
        m.pass = m.passes;
        return M_DONE;
    }
    if ((m.r < 0.0 && next > 0.0) || (m.r > 0.0 && next < 0.0)) {
        m.s = s * -0.01;
        m.r = next;
        m.pass++;
        return m.pass >= m.passes ? M_DONE : M_RUNNING;
    }
    m.r = next;
    return M_RUNNING;
}

// RayMarchingShape::ray_intersect for the Heart in object space (o, d):
// returns true with *t_out on a hit in [min_t, max_t].
template <bool STATS>
PT_HD bool heart_march(double step0, int passes, double ox, double oy, double oz, double dx, double dy, double dz,
                       double min_t, double max_t, double *t_out, MarchStats *st) {
    MarchState m;
    if (!march_begin(step0, passes, ox, oy, oz, dx, dy, dz, &m)) return false;
    int status;
    while ((status = march_iter<STATS>(m, st)) == M_RUNNING) {
    }
    if (status == M_MISS) return false;
    if (m.t < min_t || m.t > max_t) return false;  // ray_marching.rs:55-57
    *t_out = m.t;
    return true;
}

}  // namespace march
}  // namespace pt
