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

// True if sgn * g(j) exceeds every rounding error and the 1e-15 stop for all
// j in [1, b]: sgn*g0 - sum_k |g_k| b^k > 1e-15 + 128 eps M(b), where M(b) bounds
// the magnitudes of all monomials over the block (it covers both the error of
// the coefficients above and that of the reference's own f64 evaluation).
PT_HD bool poly_sign_definite(const Poly &P, double b, double sgn) {
    double d = 0.0;
    for (int k = 6; k >= 1; k--) d = (d + fabs(P.g[k])) * b;
    double xm = P.ax + P.cx * b, ym = P.ay + P.cy * b, zm = P.az + P.cz * b;
    double x2 = xm * xm, y2 = ym * ym, z2 = zm * zm, z3 = z2 * zm;
    double am = x2 + 2.25 * y2 + z2 + 1.0;
    double m = am * am * am + x2 * z3 + 0.1125 * y2 * z3;
    return sgn * P.g[0] - d > 1e-15 + 1.4210854715202004e-14 * m;  // 128 * 2^-53
}

// ------------------------------------------------------- the march
struct MarchStats {
    uint32_t steps, blocks, tries;
};

// RayMarchingShape::ray_intersect for the Heart in object space (o, d):
// returns true with *t_out on a hit in [min_t, max_t].
template <bool STATS>
PT_HD bool heart_march(double step0, int passes, double ox, double oy, double oz, double dx, double dy, double dz,
                       double min_t, double max_t, double *t_out, MarchStats *st) {
    double start, end;
    if (!heart_bound(ox, oy, oz, dx, dy, dz, &start, &end)) return false;
    double s = step0;
    double t = start;
    double px = ox + dx * t, py = oy + dy * t, pz = oz + dz * t;
    double r = heart_f(px, py, pz);
    bool hit = false;
    for (int pass = 0; pass < passes && !hit; pass++) {
        double cx = dx * s, cy = dy * s, cz = dz * s;
        for (;;) {
            if (t > end || t < start) return false;
            // ---- try to jump a block of b steps (exact closed form + sign proof)
            if (r != 0.0) {
                Lin Lx, Ly, Lz, Lt;
                int64_t bmax = lin_init(px, cx, &Lx);
                if (bmax >= 2) bmax = imin(bmax, lin_init(py, cy, &Ly));
                if (bmax >= 2) bmax = imin(bmax, lin_init(pz, cz, &Lz));
                if (bmax >= 2) bmax = imin(bmax, lin_init(t, s, &Lt));
                bmax = imin(bmax, (int64_t)1 << 24);
                if (bmax >= 2) {
                    // exact per-step displacement of each coordinate
                    double hx = Lx.frozen ? 0.0 : ldexp((double)Lx.R, Lx.sh);
                    double hy = Ly.frozen ? 0.0 : ldexp((double)Ly.R, Ly.sh);
                    double hz = Lz.frozen ? 0.0 : ldexp((double)Lz.R, Lz.sh);
                    Poly P;
                    heart_poly(px, py, pz, hx, hy, hz, &P);
                    if (STATS) st->tries++;
                    // first guess from the linear term, then halve until proven
                    double sgn = r > 0.0 ? 1.0 : -1.0;
                    double lead = sgn * P.g[0], slope = fabs(P.g[1]);
                    int64_t b = bmax;
                    if (slope > 0.0 && lead > 0.0) {
                        double est = lead / slope;
                        if (est < (double)b) b = est < 2.0 ? 2 : (int64_t)est;
                    }
                    bool jumped = false;
                    while (b >= 2) {
                        double tl = lin_at(Lt, t, b - 1);  // t before the last step of the block
                        if (!(tl > end || tl < start) && poly_sign_definite(P, (double)b, sgn)) {
                            t = lin_at(Lt, t, b);
                            px = lin_at(Lx, px, b);
                            py = lin_at(Ly, py, b);
                            pz = lin_at(Lz, pz, b);
                            r = heart_f(px, py, pz);
                            if (STATS) st->blocks++;
                            jumped = true;
                            break;
                        }
                        b >>= 1;
                    }
                    if (jumped) continue;
                }
            }
            // ---- one literal step (ray_marching.rs:38-51)
            t += s;
            px += cx;
            py += cy;
            pz += cz;
            double next = heart_f(px, py, pz);
            if (STATS) st->steps++;
            if (fabs(next - 0.0) < 1e-15) {
                hit = true;
                break;
            }
            if ((r < 0.0 && next > 0.0) || (r > 0.0 && next < 0.0)) {
                s *= -0.01;
                r = next;
                break;
            }
            r = next;
        }
    }
    if (t < min_t || t > max_t) return false;
    *t_out = t;
    return true;
}

}  // namespace march
}  // namespace pt
