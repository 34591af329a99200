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
#include <cstring>

#include "pt_funcs.hpp"

#ifndef PT_HD
#define PT_HD __host__ __device__ __forceinline__
#endif

// Host-only profiling hooks (tools/march_prof.cpp); no-ops in the product.
#ifndef PT_MPROF
#define PT_MPROF(field) ((void)0)
#endif
#ifndef PT_MHOOK
#define PT_MHOOK(what) ((void)0)
#endif
#ifndef PT_MSEG
#define PT_MSEG(k) ((void)0)
#endif
#ifndef PT_MTRACE
#define PT_MTRACE(guess, B, good, bmax) ((void)0)
#endif
#ifndef PT_MREG  // device region timing (variant builds with PT_MARCH_REGIONS, pt_wave.hip)
#define PT_MREG(what) ((void)0)
#endif
#ifndef PT_MCAPTURE
#define PT_MCAPTURE(step0, passes, ox, oy, oz, dx, dy, dz) ((void)0)
#endif

namespace pt {
namespace march {

// Heart::shape_func and Heart::intersect_bound (ray_marching.rs:135-155), as
// FParams-free helpers (tests, tools); the march itself is generic.
PT_HD double heart_f(double px, double py, double pz) { return f_heart(px, py, pz); }
PT_HD bool heart_bound(double ox, double oy, double oz, double dx, double dy, double dz, double *start,
                       double *end) {
    FParams F{};
    F.func = F_HEART;
    return shape_bound(F, ox, oy, oz, dx, dy, dz, start, end);
}

// ------------------------------------------------------- closed-form adds
// All closed-form arithmetic is done in f64: grid integers (X, R, spans) stay
// below 2^53, so every product and sum below is exact, and the GPU never
// needs emulated int64 multiplies or divisions.
struct Lin {
    double X = 0.0, R = 0.0;  // value = X * u, step = R * u (X, R integers)
    double u = 0.0;           // grid of x's binade, 2^(e-52)
    bool frozen = false;      // c == 0: fl(x + 0) = x forever
};

constexpr int64_t BIG = (int64_t)1 << 40;
constexpr double BIGD = 1099511627776.0;  // 2^40
PT_HD int64_t imin(int64_t a, int64_t b) { return a < b ? a : b; }

// 1/x to a few ulp: the hardware reciprocal (v_rcp_f64 is only good to about
// 2^-23 relative) polished by two Newton steps; callers correct the floor of a
// quotient computed with it by exact integer tests.  (Explicit fma here is not
// a contraction of the reference's arithmetic: the result is only an estimate.)
PT_HD double approx_rcp(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(x);
    r = fma(r, fma(-x, r, 1.0), r);
    r = fma(r, fma(-x, r, 1.0), r);
    return r;
#else
    return 1.0 / x;
#endif
}

PT_HD uint64_t f64_to_bits(double x) {
    uint64_t u;
    memcpy(&u, &x, 8);
    return u;
}
PT_HD double bits_to_f64(uint64_t u) {
    double x;
    memcpy(&x, &u, 8);
    return x;
}

// floor(n / d) for integers 0 <= n, 1 <= d, n / d < 2^41, all exact in f64.
PT_HD double floor_div(double n, double d) {
    double k = floor(n * approx_rcp(d));
    // the estimate is within a fraction of 1 of n / d; two exact corrections
    if (k * d > n) k -= 1.0;
    if (k * d > n) k -= 1.0;
    if ((k + 1.0) * d <= n) k += 1.0;
    if ((k + 1.0) * d <= n) k += 1.0;
    return k;
}

// Largest B such that the first B additions fl(x_j + c), j = 0..B-1, are all
// x_j + R*u exactly; 0 if the closed form does not apply here.
PT_HD int64_t lin_init(double x, double c, Lin *L) {
    PT_MPROF(lin_init);
    L->frozen = false;
    if (c == 0.0) {
        L->frozen = true;
        return BIG;
    }
    if (!(x != 0.0) || !(fabs(x) < 1e300) || !(fabs(c) < 1e300)) return PT_MPROF(lin_fail_zero), 0;  // zero, inf, NaN
    const int e = ilogb(x);
    if (e < -960) return 0;  // stay clear of subnormals
    const double sc = ldexp(1.0, 52 - e);  // 1/u, a power of two: scaling by it is exact
    const double q = c * sc;               // c / u
    if (!(fabs(q) < 4.0e15)) return PT_MPROF(lin_fail_q), 0;  // |c| >= 2^52 u: leaves the binade at once
    const double X = x * sc;               // integer, 2^52 <= |X| < 2^53
    const double qf = floor(q);
    double R;
    if (q - qf == 0.5) {
        // Round-half-even tie: x + c sits halfway between two grid points and
        // rounds to the even one.  From an even X the sum lands on an even X
        // again, advancing by the even one of {k, k+1} every step.
        if (floor(X * 0.5) * 2.0 != X) return PT_MPROF(lin_fail_tie), 0;  // one literal step first makes X even
        R = floor(qf * 0.5) * 2.0 == qf ? qf : qf + 1.0;
    } else {
        R = rint(q);
    }
    // Only the binade edge the sequence moves toward matters: moving away from
    // zero (Rs > 0) every exact sum A + |q| must stay below 2^53, moving toward
    // it (Rs < 0) every A - |q| at or above 2^52 (then the sum rounds on grid u).
    const double C = ceil(fabs(q));
    const double lo = 4503599627370496.0 + C + 1.0, hi = 9007199254740992.0 - C - 1.0;
    const double A = fabs(X), Rs = X >= 0.0 ? R : -R;
    if (Rs > 0.0 ? A > hi : (Rs < 0.0 && A < lo)) return PT_MPROF(lin_fail_zone), 0;
    L->X = X;
    L->R = R;
    L->u = ldexp(1.0, e - 52);  // 1 / sc, exactly (a power of two; no division)
    if (Rs == 0.0) return BIG;
    const double span = Rs > 0.0 ? hi - A : A - lo, step = fabs(Rs);
    if (span >= BIGD * step) return BIG;
    return (int64_t)floor_div(span, step) + 1;
}

PT_HD double lin_at(const Lin &L, double x, int64_t j) {
    if (L.frozen) return x;
    return (L.X + (double)j * L.R) * L.u;
}

// lin_init as straight-line code for SIMT lanes: every quantity is computed,
// the cases are selects, and the room comes back as an exact f64 integer
// (0: the closed form does not apply here; BIGD: unbounded).  The same room and
// the same (X, R, u) wherever lin_init's room is >= 2, which is all its callers
// use.  floor(span / step) needs one correction each way: span / step < 2^41
// and the polished reciprocal is good to a few ulp, so the estimate is off by
// less than 1.  need: a room of at least `need` comes back as `need` without
// the division (the callers take min(room, need)).
PT_HD double lin_room(double x, double c, Lin *L, double need = BIGD) {
    PT_MPROF(lin_init);
    const double ax = fabs(x), ac = fabs(c);
    const bool ok0 = x != 0.0 && ax < 1e300 && ac < 1e300;  // zero, inf, NaN: no
#if defined(__HIP_DEVICE_COMPILE__)
    // v_frexp_exp: ilogb for finite nonzero x (0, inf, NaN give a value the ok
    // test below masks), without libm's special-case selects
    const int e = __builtin_amdgcn_frexp_exp(x) - 1;
#else
    const int e = ilogb(ok0 ? x : 1.0);
#endif
    // X = x / u, q = c / u: scaling by a power of two is exact (ldexp: no multiply)
    const double q = ldexp(c, 52 - e), X = ldexp(x, 52 - e), aq = fabs(q);
    // rint rounds half to even: on a tie it is the even one of floor(q) and
    // floor(q) + 1, the step a sum from an even X takes (q - R is exact)
    const double R = rint(q);
    const bool tie = fabs(q - R) == 0.5;  // round-half-even: only from an even X
    const bool xodd = (f64_to_bits(x) & 1u) != 0;  // X's parity is x's last mantissa bit (x normal)
    const double C = ceil(aq);
    const double lo = 4503599627370496.0 + C + 1.0, hi = 9007199254740992.0 - C - 1.0;
    const double A = fabs(X), Rs = X >= 0.0 ? R : -R;
    L->X = X;
    L->R = R;
    L->u = ldexp(1.0, e - 52);
    L->frozen = c == 0.0;
    // grid steps to the edge the sequence moves toward (negative: already past it)
    const double span = Rs > 0.0 ? hi - A : A - lo, step = fabs(Rs);
    const bool zone = Rs != 0.0 && span < 0.0;
    const bool ok = ok0 && e >= -960 && aq < 4.0e15 && !(tie && xodd) && !zone;
    double room;
    if (Rs == 0.0 || span >= BIGD * step) {
        room = BIGD;
    } else if ((need - 1.0) * step <= span) {
        // the caller's `need` steps fit (room = floor(span / step) + 1 >= need;
        // the product is exact below 2^53 and above span otherwise): no division
        room = need;
    } else {
        double k = floor(span * approx_rcp(step));
        k = k * step > span ? k - 1.0 : k;
        k = (k + 1.0) * step <= span ? k + 1.0 : k;
        room = k + 1.0;
    }
    if (c == 0.0) return BIGD;
    return ok ? room : 0.0;
}

// x after n literal additions fl(x + c), exactly, across any number of binade
// edges: closed form inside each binade, literal adds in the thin zone at an
// edge and within ADV_NZ |c| of zero (a coordinate crossing zero passes
// ~2 log2(|x| / |c|) binades; the ones near zero hold a few steps each, and a
// closed-form segment costs ~150 instructions against ~5 per literal add: C2
// one-stream march 183 -> 172 ms).  Each coordinate's sequence is independent of the
// others, so p, t can be advanced separately.
constexpr int ADV_NZB = 4;         // literal adds per trip in the near-zero zone
constexpr double ADV_NZ = 24.0;    // |x| below this many |c|: literal adds (the binades there hold a few steps each)
PT_HD double advance(double x, double c, double n) {
    PT_MHOOK(adv_begin);
    while (n > 0.0) {
        if (fabs(x) < ADV_NZ * fabs(c)) {
            // near zero every binade holds only a few steps: ADV_NZB
            // literal adds per trip instead of one closed-form segment per binade
#pragma unroll
            for (int j = 0; j < ADV_NZB; j++) {
                PT_MPROF(lit_adds);
                const bool go = n > 0.0;
                x = go ? x + c : x;
                n = go ? n - 1.0 : n;
            }
            continue;
        }
        PT_MPROF(advance_loops);
        Lin L;
        const double room = lin_room(x, c, &L, n);
        // the closed form to the end of the segment (or n), then the literal
        // add that leaves it; a literal add alone in an edge zone
        const double k = room >= 2.0 ? (room < n ? room : n) : 0.0;
        if (k > 0.0) x = L.frozen ? x : (L.X + k * L.R) * L.u;
        n -= k;
        if (n > 0.0 && k == (room >= 2.0 ? room : 0.0)) {
            x = x + c;
            n -= 1.0;
        }
    }
    PT_MHOOK(adv_end);
    return x;
}

// One segment of advance(): the closed form to the end of x's binade segment
// (and the literal add leaving it), or one literal add in an edge zone.
PT_HD void seg_step(double &x, double c, double &n) {
    if (fabs(x) < ADV_NZ * fabs(c)) {  // near zero: a literal add (see advance)
        x = x + c;
        n -= 1.0;
        return;
    }
    Lin L;
    const double room = lin_room(x, c, &L, n);
    const double k = room >= 2.0 ? (room < n ? room : n) : 0.0;
    if (k > 0.0) x = L.frozen ? x : (L.X + k * L.R) * L.u;
    n -= k;
    if (n > 0.0 && k == (room >= 2.0 ? room : 0.0)) {
        x = x + c;
        n -= 1.0;
    }
}

// A lower bound on steps_in_range, in closed form: every add rounds by at
// most delta = 2^-53 max(|start|, |end|) while t stays in range, so
// t_j <= t + j (s + delta) (s > 0; mirrored for s < 0) and all j with
// j <= (lim - t) / (|s| + delta) are in range; the quotient is shrunk by a
// relative 1e-12 and one step for its own rounding.  Blocks only need a
// lower bound: the last few steps before the range end are taken literally.
PT_HD double steps_in_range_lb(double t, double s, double start, double end, double cap) {
    const double dist = s > 0.0 ? end - t : t - start;
    const double delta = 1.1102230246251565e-16 * fmax(fabs(start), fabs(end));
    // the quotient through a polished reciprocal (a few ulp): far inside the 1e-12 shrink
    const double k = floor(dist * approx_rcp(fabs(s) + delta) * (1.0 - 1e-12)) - 1.0;
    const double b = !(k >= 0.0) ? 1.0 : (k + 1.0 >= cap ? cap : k + 1.0);
    return dist >= 0.0 ? b : 0.0;
}

// An upper bound on the index J of the first t_J outside [start, end] (the
// step at which the reference's range check ends the pass with a miss):
// t_j >= t + j (s - delta) (s > 0; mirrored for s < 0), so J <= floor(dist /
// (|s| - delta)) + 1; grown by a relative 1e-12 and two steps for rounding.
PT_HD double steps_exit_ub(double t, double s, double start, double end) {
    const double dist = s > 0.0 ? end - t : t - start;
    const double delta = 1.1102230246251565e-16 * fmax(fabs(start), fabs(end));
    const double as = fabs(s);
    const double k = ceil(dist * approx_rcp(as - delta) * (1.0 + 1e-12)) + 2.0;  // reciprocal: see above
    return !(dist >= 0.0) || !(as > 2.0 * delta) || !(k < BIGD) ? BIGD : k;
}

// Largest b (<= cap) such that t_0 .. t_{b-1} of t_{j+1} = fl(t_j + s) all lie
// in [start, end] (the reference's check before each step), given t_0 does.
// Closed form per binade segment of t: t_k = (X + kR) u stays in range while
// k <= D / |R|, D the grid distance to the limit.
PT_HD int64_t steps_in_range(double t, double s, double start, double end, int64_t cap) {
    int64_t j0 = 0;  // index of x = t_j0, in range
    double x = t;
    for (;;) {
        PT_MPROF(sir_inside);
        Lin L;
        const int64_t room = lin_init(x, s, &L);
        if (room >= 2 && !L.frozen) {
            const int64_t B = imin(room, cap - 1 - j0);  // points x_0 .. x_B of the segment
            const double sc = 1.0 / L.u;
            const double D = s > 0.0 ? floor(end * sc) - L.X : L.X - ceil(start * sc);
            const double aR = fabs(L.R);
            const int64_t k = D >= aR * (double)B ? B : (int64_t)floor_div(D, aR);
            if (k < B || j0 + B >= cap - 1) return j0 + k + 1;
            j0 += B;
            x = lin_at(L, x, B);
        } else {
            if (L.frozen) return cap;  // s == 0 never leaves
            const double y = x + s;
            if (y > end || y < start) return j0 + 1;
            x = y;
            if (++j0 >= cap - 1) return cap;
        }
    }
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

// The Heart's expansion, by coefficient (fewer live temporaries than the
// generic degree-tracked expansion; both are exact-arithmetic expansions of
// the same polynomial, with rounding inside the proof's margin).
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

// The expansion for any of the ray-marched functions (pt_funcs.hpp).
template <int FK>
PT_HD void func_poly(const FParams &F, double x, double y, double z, double cx, double cy, double cz, Poly *P) {
    if constexpr (FK == F_HEART) {
        heart_poly(x, y, z, cx, cy, cz, P);
        return;
    }
    shape_poly_k<FK>(F, x, y, z, cx, cy, cz, P->g);
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
PT_HD double heart_mag(const Poly &P, double b) {
    double xm = P.ax + P.cx * b, ym = P.ay + P.cy * b, zm = P.az + P.cz * b;
    double x2 = xm * xm, y2 = ym * ym, z2 = zm * zm, z3 = z2 * zm;
    double am = x2 + 2.25 * y2 + z2 + 1.0;
    return am * am * am + x2 * z3 + 0.1125 * y2 * z3;
}
PT_HD double heart_margin(const Poly &P, double b) {
    const double e256 = 2.8421709430404007e-14;  // 256 * 2^-53
    double mag = heart_mag(P, b);
    // The step points are p_j = p0 + j*c + delta_j with |delta_j,k| <= j*ulp_k/2
    // (each literal add rounds once): add max|grad f| . |delta| over the block.
    double xm = P.ax + P.cx * b, ym = P.ay + P.cy * b, zm = P.az + P.cz * b;
    double x2 = xm * xm, y2 = ym * ym, z2 = zm * zm, z3 = z2 * zm;
    double am = x2 + 2.25 * y2 + z2 + 1.0, am2 = am * am;
    double gx = 6.0 * xm * am2 + 2.0 * xm * z3;
    double gy = 13.5 * ym * am2 + 0.225 * ym * z3;
    double gz = 6.0 * zm * am2 + 3.0 * x2 * z2 + 0.3375 * y2 * z2;
    double drift = b * 2.3e-16 * (gx * xm + gy * ym + gz * zm);  // ulp(v)/2 <= 2^-53 |v| (2.3e-16 > 2^-52)
    return 1e-15 + e256 * mag + drift;
}

template <int FK>
PT_HD double poly_margin(const FParams &F, const Poly &P, double b) {
    if constexpr (FK == F_HEART) return heart_margin(P, b);
    const double e256 = 2.8421709430404007e-14;  // 256 * 2^-53
    const double xm = P.ax + P.cx * b, ym = P.ay + P.cy * b, zm = P.az + P.cz * b;
    // M(b) bounds every monomial of f over the block (|f| and its f64
    // evaluation error scale); G bounds |df/dx_k| there.  The step points are
    // p_j = p0 + j*c + delta_j with |delta_j,k| <= j*ulp_k/2 (each literal
    // add rounds once): add max|grad f| . |delta| over the block.
    const DM m = shape_mag_k<FK>(F, xm, ym, zm);
    const double drift = b * 2.3e-16 * (m.gx * xm + m.gy * ym + m.gz * zm);  // ulp(v)/2 <= 2^-53 |v|
    return 1e-15 + e256 * m.v + drift;
}

// Bernstein form of sgn*g on j in [0, b] (lambda = j / b): g >= min_i beta_i
// over the whole block (convex hull property), and min beta = g(b) exactly
// when the control polygon is monotone, so the test is tight for the usual
// monotone approach to the surface.  The betas' own rounding (weights <= 1,
// at most 7 terms) is far inside the 256 eps M(b) part of the margin.
template <int FK = F_ANY>
PT_HD bool poly_sign_definite(const FParams &F, const Poly &P, double b, double sgn) {
    const double margin = poly_margin<FK>(F, P, b);
    double a[7];
    double bk = 1.0;
#pragma unroll
    for (int k = 0; k < 7; k++) {
        a[k] = sgn * P.g[k] * bk;
        bk *= b;
    }
    if (a[0] <= margin) return false;
    const double b1 = a[0] + a[1] * (1.0 / 6.0);
    const double b2 = a[0] + a[1] * (1.0 / 3.0) + a[2] * (1.0 / 15.0);
    const double b3 = a[0] + a[1] * 0.5 + a[2] * 0.2 + a[3] * 0.05;
    const double b4 = a[0] + a[1] * (2.0 / 3.0) + a[2] * 0.4 + a[3] * 0.2 + a[4] * (1.0 / 15.0);
    const double b5 = a[0] + a[1] * (5.0 / 6.0) + a[2] * (2.0 / 3.0) + a[3] * 0.5 + a[4] * (1.0 / 3.0) + a[5] * (1.0 / 6.0);
    const double b6 = a[0] + a[1] + a[2] + a[3] + a[4] + a[5] + a[6];
    const double mn = fmin(fmin(fmin(b1, b2), fmin(b3, b4)), fmin(b5, b6));
    return mn > margin;
}

constexpr int FOLD_MAX = 3;     // literal steps an iteration may take when the predicted crossing is that close
// literal batches after failed proofs double per failure in a row (round 5; one step each: C2 1978 vs 2068)
constexpr int LIT_BATCH = 2;  // literal steps after a proof that proved no block
constexpr int LIT_DOUBLINGS = 5;
constexpr int MAX_LEVELS = 40;  // de Casteljau halvings per prefix search (capping them: more iterations, slower)
// Longest provable prefix of a block: the largest integer b <= B such that
// sgn * (f64 heart_f at p_j) > 1e-15 for every j in [1, b] (so neither the
// approx_equal stop nor a sign change can fire before step b).  One Bernstein
// form on [0, B], then de Casteljau halving toward the first region the hull
// cannot clear: each level either proves the left half (and moves right) or
// descends into it.  The margin is the one for the whole block (M and the
// drift only grow with b), and the halving's own rounding (<= 24 levels of
// exact-weight averages) stays far inside its 256 eps M part.
constexpr int EM_LEVELS = 40;  // halvings of a failed early-miss proof (capped at 8/10/12: slower, round 2 emab)
template <int FK>
PT_HD double poly_prefix(const FParams &F, const Poly &P, double Bd, double sgn, double target = 0.0,
                         int max_levels = MAX_LEVELS) {
    const double margin = poly_margin<FK>(F, P, Bd);
    double a[7];
    double bk = 1.0;
#pragma unroll
    for (int k = 0; k < 7; k++) {
        a[k] = sgn * P.g[k] * bk;
        bk *= Bd;
    }
    if (a[0] <= margin) return 0.0;
    double c[7];
    c[0] = a[0];
    c[1] = a[0] + a[1] * (1.0 / 6.0);
    c[2] = a[0] + a[1] * (1.0 / 3.0) + a[2] * (1.0 / 15.0);
    c[3] = a[0] + a[1] * 0.5 + a[2] * 0.2 + a[3] * 0.05;
    c[4] = a[0] + a[1] * (2.0 / 3.0) + a[2] * 0.4 + a[3] * 0.2 + a[4] * (1.0 / 15.0);
    c[5] = a[0] + a[1] * (5.0 / 6.0) + a[2] * (2.0 / 3.0) + a[3] * 0.5 + a[4] * (1.0 / 3.0) + a[5] * (1.0 / 6.0);
    c[6] = a[0] + a[1] + a[2] + a[3] + a[4] + a[5] + a[6];
    if (target >= 2.0 && target < Bd) {
        // One split at the step just before the predicted crossing: de
        // Casteljau at lambda >= target / B gives the control points of
        // [0, lambda B], a superset of the steps [1, target]; if they clear
        // the margin, target is the prefix and the halving search below is
        // not needed.  lambda is target / B rounded up (an exact fma test),
        // and the lerps' rounding (6 levels, weights in [0, 1]) stays inside
        // the margin's 256 eps M part like the halvings' do.
        const double td = target;
        double lam = td * approx_rcp(Bd);  // > 0: the next double up is one more in its bits
        if (fma(lam, Bd, -td) < 0.0) lam = bits_to_f64(f64_to_bits(lam) + 1);
        if (fma(lam, Bd, -td) < 0.0) lam = bits_to_f64(f64_to_bits(lam) + 1);
        if (fma(lam, Bd, -td) >= 0.0 && lam <= 1.0) {
            double w[7];
#pragma unroll
            for (int i = 0; i < 7; i++) w[i] = c[i];
            double mn = w[0];
#pragma unroll
            for (int r = 1; r < 7; r++) {
#pragma unroll
                for (int i = 0; i < 7 - r; i++) w[i] = w[i] + lam * (w[i + 1] - w[i]);
                mn = fmin(mn, w[0]);
            }
            if (mn > margin) return target;
        }
    }
    double lo = 0.0, len = 1.0, proven = 0.0;  // in units of B
    PT_MHOOK(lv_begin);
    PT_MREG(halve_begin);
    for (int level = 0; level < max_levels; level++) {
        PT_MPROF(evals);
        double mn = fmin(fmin(fmin(c[1], c[2]), fmin(c[3], c[4])), fmin(fmin(c[5], c[6]), c[0]));
        if (mn > margin) {
            proven = lo + len;
            break;
        }
        if (len * Bd < 1.0) break;  // resolution reached (one step): stop here
        // de Casteljau at 1/2 in place: level r overwrites c[0 .. 6-r], so
        // afterwards c[i] is the level-(6-i) point i = the right half's
        // control point i; the left half's are the levels' first points.
        double l[7];
        l[0] = c[0];
#pragma unroll
        for (int r = 1; r < 7; r++) {
#pragma unroll
            for (int i = 0; i < 7 - r; i++) c[i] = (c[i] + c[i + 1]) * 0.5;
            l[r] = c[0];
        }
        double mnl = fmin(fmin(fmin(l[1], l[2]), fmin(l[3], l[4])), fmin(fmin(l[5], l[6]), l[0]));
        len *= 0.5;
        if (mnl > margin) {
            proven = lo + len;
            lo += len;  // continue in the right half (c)
        } else {
            for (int i = 0; i < 7; i++) c[i] = l[i];
        }
    }
    PT_MREG(halve_end);
    PT_MHOOK(lv_end);
    const double b = floor(proven * Bd);
    return b < 0.0 ? 0.0 : b;
}

// Predicted first crossing (in steps) of sgn*g: the quadratic part's first
// positive root (Newton steps on the full polynomial measured worse: misses
// chase spurious roots of the degree-6 polynomial); the search starts just
// before it and the proof decides.
PT_HD double poly_eval(const Poly &P, double j, double *dg) {
    double g = P.g[6], d = 0.0;
#pragma unroll
    for (int k = 5; k >= 0; k--) {
        d = d * j + g;
        g = g * j + P.g[k];
    }
    *dg = d;
    return g;
}

// A heuristic only (it sizes the block; the proof decides what is skipped), so
// it divides through the hardware reciprocal.
PT_HD double poly_root_guess(const Poly &P, double sgn, double cap) {
    // straight-line: every case computed, then selected (the values are the
    // branchy form's wherever it used them)
    const double L = sgn * P.g[0], S = sgn * P.g[1], Q = sgn * P.g[2];
    const double disc = S * S - 4.0 * Q * L;
    const double sq = sqrt(fmax(disc, 0.0));
    const double i2q = approx_rcp(2.0 * Q);
    const double r1 = (-S - sq) * i2q, r2 = (-S + sq) * i2q;
    const double lo = fmin(r1, r2), hi = fmax(r1, r2);
    const double rq = disc < 0.0 ? cap : (lo > 0.0 ? lo : (hi > 0.0 ? hi : cap));  // (no real root: no crossing)
    const double rl = S < 0.0 ? L * approx_rcp(-S) : cap;
    double r = fmin(cap, Q == 0.0 ? rl : rq);
    return L <= 0.0 ? 1.0 : r;
}

// ------------------------------------------------------- the march
constexpr double MIN_GUESS = 2.0;     // a predicted crossing closer than this many steps: literal steps, no proof
constexpr int ADV_ROUNDS = 64;        // binade-segment rounds per march_advance call
constexpr double BLOCK_SCALE = 1.25;  // a block is sized BLOCK_SCALE * guess + BLOCK_PAD steps
constexpr double BLOCK_PAD = 4.0;
struct MarchStats {
    uint32_t steps, blocks, tries;
    uint32_t guard;  // marches dropped by the MARCH_GUARD (always counted, not only in STATS builds)
};

// Resumable form of RayMarchingShape::ray_intersect (ray_marching.rs:20-74) so
// a lane can march a few iterations per pass of the kernel's main loop while
// the other lanes of its wave keep tracing.
struct MarchState {
    FParams F;  // which implicit function, and its constants
    double t, px, py, pz, r, s, start, end, dx, dy, dz;
    double lim;  // a lower bound on the steps in range from the current point for this pass (-1: not known yet)
    int pass, passes;
    uint32_t iters;  // guard: a march that has not ended after MARCH_GUARD iterations is dropped
    int adv;         // 1 while a proven block's exact advance is still walking binade segments
    int lit;         // consecutive proof attempts of this pass that proved no block (each doubles the literal batch)
    double na[4];    // steps still to apply to t, px, py, pz during an advance
};
// M_GUARD: the march was dropped by MARCH_GUARD (callers take it as a miss
// and count it: pt_march_guard_drops).
enum MarchStatus : int { M_RUNNING = 0, M_DONE = 1, M_MISS = 2, M_GUARD = 3 };
constexpr uint32_t MARCH_GUARD = 1u << 24;

// Start of the march on a bound interval [start, end] already known
// (intersect_bound, ray_marching.rs:27-31), object-space ray (o, d).
template <int FK = F_ANY>
PT_HD void march_start(const FParams &F, double step0, int passes, double ox, double oy, double oz, double dx,
                       double dy, double dz, double start, double end, MarchState *m) {
    m->F = F;
    PT_MCAPTURE(step0, passes, ox, oy, oz, dx, dy, dz);
    m->start = start;
    m->end = end;
    m->s = step0;
    m->t = start;
    m->px = ox + dx * start;
    m->py = oy + dy * start;
    m->pz = oz + dz * start;
    m->r = shape_f_k<FK>(F, m->px, m->py, m->pz);
    m->dx = dx;
    m->dy = dy;
    m->dz = dz;
    m->pass = 0;
    m->passes = passes;
    m->lim = -1.0;
    m->iters = 0;
    m->adv = 0;
    m->lit = 0;
}

// Bound test and start of the march; false if the ray misses the bound.
template <int FK = F_ANY>
PT_HD bool march_begin(const FParams &F, double step0, int passes, double ox, double oy, double oz, double dx,
                       double dy, double dz, MarchState *m) {
    double start, end;
    if (!shape_bound_k<FK>(F, ox, oy, oz, dx, dy, dz, &start, &end)) return false;
    march_start<FK>(F, step0, passes, ox, oy, oz, dx, dy, dz, start, end, m);
    return true;
}

// One round of a proven block's exact advance: one binade segment for each
// of t, px, py, pz that still has steps to go; when all are done the block's
// end point is exact and f is evaluated there.
template <int FK = F_ANY, int ROUNDS = ADV_ROUNDS>
PT_HD void march_advance(MarchState &m, double cx, double cy, double cz) {
    PT_MHOOK(block_begin);
    for (int round = 0; round < ROUNDS; round++) {
        if (m.na[0] > 0.0) PT_MSEG(0), seg_step(m.t, m.s, m.na[0]);
        if (m.na[1] > 0.0) PT_MSEG(1), seg_step(m.px, cx, m.na[1]);
        if (m.na[2] > 0.0) PT_MSEG(2), seg_step(m.py, cy, m.na[2]);
        if (m.na[3] > 0.0) PT_MSEG(3), seg_step(m.pz, cz, m.na[3]);
        if (!(m.na[0] > 0.0 || m.na[1] > 0.0 || m.na[2] > 0.0 || m.na[3] > 0.0)) break;
    }
    if (m.na[0] > 0.0 || m.na[1] > 0.0 || m.na[2] > 0.0 || m.na[3] > 0.0) return;
    m.adv = 0;
    m.r = shape_f_k<FK>(m.F, m.px, m.py, m.pz);
}

// One iteration of the march loop: a proven jump, or one literal step (after a
// failed proof).  M_DONE: the passes ended (the caller applies the final
// t-in-[min_t, max_t] test); M_MISS: t left [start, end].
template <bool STATS, bool INLINE_ADV = true, int FK = F_ANY>
PT_HD int march_iter(MarchState &m, MarchStats *st) {
    PT_MPROF(iters);
    int nlit = 1;
    if (m.pass >= m.passes) return M_DONE;
    // Every iteration takes >= 1 reference step; a march still running after
    // 2^24 of them is one the reference itself would not finish (a step below
    // t's rounding, say: t + step == t forever).  Dropping it keeps every GPU
    // wave finite; the caller counts the drop (M_GUARD) and takes it as a miss.
    if (++m.iters > MARCH_GUARD) return M_GUARD;
    double s = m.s;
    double cx = m.dx * s, cy = m.dy * s, cz = m.dz * s;
    if (m.adv) {
        march_advance<FK>(m, cx, cy, cz);
        return M_RUNNING;
    }
    if (m.t > m.end || m.t < m.start) return M_MISS;
    // ---- try to jump a block of b steps (exact advance + sign proof)
    if (m.r != 0.0) {
        // the range limit moves with the sequence: computed once per pass
        if (m.lim < 0.0) m.lim = steps_in_range_lb(m.t, s, m.start, m.end, 16777216.0);
        const double bmax = m.lim;
        if (bmax >= 2.0) {
            Poly P;
            PT_MREG(poly_begin);
            // the polynomial along the steps, every coordinate with its drift term (proofs along the exact grid
            // steps of in-binade coordinates, without the drift, took fewer iterations but spilled the march
            // kernel: C2 2041 vs 2068, round 5, removed in round 6)
            func_poly<FK>(m.F, m.px, m.py, m.pz, cx, cy, cz, &P);
            if (STATS) st->tries++;
            // longest provable prefix of a block sized from the predicted
            // crossing (the margin scales with the block, so a block far
            // longer than the crossing distance would drown the near part)
            const double sgn = m.r > 0.0 ? 1.0 : -1.0;
            const double guess = poly_root_guess(P, sgn, bmax);
            PT_MREG(poly_end);
            if (guess < MIN_GUESS) {
                PT_MTRACE(guess, 0, 0, bmax);
                // the crossing is the next step or two: up to FOLD_MAX
                // literal steps in this iteration
                nlit = guess >= 1.0 ? FOLD_MAX : 1;
                goto literal;
            }
            // No crossing predicted before the range end: try to prove every
            // step up to (an upper bound on) the one that leaves the range;
            // then nothing can stop this pass first and the march misses.
            const double ub = guess >= bmax ? steps_exit_ub(m.t, s, m.start, m.end) : BIGD;
            const bool em = ub < BIGD;  // an early-miss proof
            double B = em ? ub : floor(guess * BLOCK_SCALE) + BLOCK_PAD;
            if (!em) B = B > bmax ? bmax : (B < 2.0 ? 2.0 : B);
            // the step just before the predicted crossing
            const double target = em ? 0.0 : ceil(guess) - 1.0;
            PT_MREG(prefix_begin);
            double good = poly_prefix<FK>(m.F, P, B, sgn, target, em ? EM_LEVELS : MAX_LEVELS);
            PT_MREG(prefix_end);
            PT_MTRACE(guess, B, good, bmax);
            if (em && good >= ub) return M_MISS;
            good = good > bmax ? bmax : good;
            // no block proven (good < 2): the crossing (or the range end) is inside the proof's margin, the band
            // where f64 rounding of f can decide either way, and only literal steps get through it.  Each failed
            // attempt in a row doubles the literal batch, so a march that grazes the surface over tens of steps
            // pays for a few proofs, not one per step (round 5: the longest captured job 63+ -> 22 iterations).
            // (Selects, not a branch: a branch here spilled an exec mask of the march kernel.)
            nlit = good >= 2.0 ? nlit : LIT_BATCH << (m.lit < LIT_DOUBLINGS ? m.lit : LIT_DOUBLINGS);
            m.lit = good >= 2.0 ? 0 : m.lit + 1;
            if (good >= 2.0) {
                // the block's exact advance runs one binade segment per
                // coordinate per iteration (march_advance), so a lane whose
                // coordinates cross many binades does not stall its wave
                m.na[0] = m.na[1] = m.na[2] = m.na[3] = good;
                m.lim -= good;
                m.adv = 1;
                if (STATS) st->blocks++;
                if (INLINE_ADV) {
                    // one loop per coordinate: a lane pays only for the binade
                    // segments each coordinate actually crosses
                    PT_MREG(adv_begin);
                    // every coordinate's first segment side by side (four
                    // independent chains), then the rest for those that cross
                    // binade edges
                    double n0 = good, n1 = good, n2 = good, n3 = good;
                    seg_step(m.t, s, n0);
                    seg_step(m.px, cx, n1);
                    seg_step(m.py, cy, n2);
                    seg_step(m.pz, cz, n3);
                    if (n0 > 0.0) m.t = advance(m.t, s, n0);
                    if (n1 > 0.0) m.px = advance(m.px, cx, n1);
                    if (n2 > 0.0) m.py = advance(m.py, cy, n2);
                    if (n3 > 0.0) m.pz = advance(m.pz, cz, n3);
                    m.na[0] = m.na[1] = m.na[2] = m.na[3] = 0.0;
                    m.adv = 0;
                    m.r = shape_f_k<FK>(m.F, m.px, m.py, m.pz);
                    PT_MREG(adv_end);
                    // a prefix that stopped short of B ends just before the
                    // crossing: take that literal step in this iteration
                    if (good < B && m.lim >= 1) {
                        // more than one when the predicted crossing is past the first
                        nlit = guess > good + 1.0 ? FOLD_MAX : 1;
                        goto literal;
                    }
                }
                return M_RUNNING;
            }
        }
    }
literal:
    // ---- literal steps (ray_marching.rs:37-51): nlit of them while no
    // crossing ends the pass; the range check before each step after the
    // first is covered by lim >= 1
    PT_MREG(lit_begin);
    for (;;) {
        if (m.lim > 0.0) m.lim -= 1.0;
        m.t += s;
        m.px += cx;
        m.py += cy;
        m.pz += cz;
        const double next = shape_f_k<FK>(m.F, m.px, m.py, m.pz);
        if (STATS) st->steps++;
        if (fabs(next - 0.0) < 1e-15) {  // approx_equal(next, 0.0): break 'outer
            m.pass = m.passes;
            return M_DONE;
        }
        if ((m.r < 0.0 && next > 0.0) || (m.r > 0.0 && next < 0.0)) {
            m.s = s * -0.01;
            m.r = next;
            m.lim = -1.0;
            m.lit = 0;
            m.pass++;
            return m.pass >= m.passes ? M_DONE : M_RUNNING;
        }
        m.r = next;
        if (--nlit <= 0 || m.lim < 1.0) return M_RUNNING;
    }
}

// The iteration the march loops use.  (Round 2 measured a variant with one
// shared advance region and at most K binade segments per coordinate per
// iteration, resumed in later iterations: slower for K = 2, 3, 4 and 64 —
// DESIGN.md §3.2 — so a proven block's advance completes in its iteration.)
template <bool STATS, bool INLINE_ADV = true, int FK = F_ANY>
PT_HD int march_step(MarchState &m, MarchStats *st) {
    return march_iter<STATS, INLINE_ADV, FK>(m, st);
}

// What the next march_iter call will do, for wave-level phase scheduling
// (wf_march): MP_CHEAP = a literal step or the end of the march, MP_ADV = an
// advance round of a proven block, MP_PROOF = build the polynomial and prove
// a block (which may still end in a literal step).  Computes the pass's range
// limit if it is not known yet, exactly as march_iter would.
enum MarchPhase : int { MP_CHEAP = 0, MP_ADV = 1, MP_PROOF = 2 };
PT_HD int march_phase(MarchState &m) {
    if (m.pass >= m.passes || m.iters + 1 > MARCH_GUARD) return MP_CHEAP;
    if (m.adv) return MP_ADV;
    if (m.t > m.end || m.t < m.start || m.r == 0.0) return MP_CHEAP;
    if (m.lim < 0.0) m.lim = steps_in_range_lb(m.t, m.s, m.start, m.end, 16777216.0);
    return m.lim >= 2.0 ? MP_PROOF : MP_CHEAP;
}

// RayMarchingShape::ray_intersect for the Heart in object space (o, d):
// returns true with *t_out on a hit in [min_t, max_t].
template <bool STATS, int FK = F_ANY>
PT_HD bool func_march(const FParams &F, double step0, int passes, double ox, double oy, double oz, double dx,
                      double dy, double dz, double min_t, double max_t, double *t_out, MarchStats *st) {
    MarchState m;
    if (!march_begin<FK>(F, step0, passes, ox, oy, oz, dx, dy, dz, &m)) return false;
    int status;
    while ((status = march_step<STATS, true, FK>(m, st)) == M_RUNNING) {
    }
    if (status == M_GUARD) st->guard++;
    if (status != M_DONE) return false;
    if (m.t < min_t || m.t > max_t) return false;  // ray_marching.rs:55-57
    *t_out = m.t;
    return true;
}

template <bool STATS>
PT_HD bool heart_march(double step0, int passes, double ox, double oy, double oz, double dx, double dy, double dz,
                       double min_t, double max_t, double *t_out, MarchStats *st) {
    FParams F{};
    F.func = F_HEART;
    return func_march<STATS, F_HEART>(F, step0, passes, ox, oy, oz, dx, dy, dz, min_t, max_t, t_out, st);
}

}  // namespace march
}  // namespace pt
