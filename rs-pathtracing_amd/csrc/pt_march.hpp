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
//     are X + B*R: exact, O(1).  Blocks stop where any of px, py, pz, t would
//     leave its binade; a tie or a coordinate near 0 falls back to one
//     literal step.
//  2. Sign proof.  Over the axis-aligned box spanned by p_k .. p_{k+B} (each
//     coordinate is monotone), interval arithmetic bounds heart_f; if the bound
//     keeps the sign of r with a margin covering f64 evaluation error plus the
//     1e-15 approx_equal threshold, none of the B steps can stop the pass, so
//     the march jumps to p_{k+B} and evaluates f there exactly.
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
    double qr = rint(q);
    if (fabs(q - qr) == 0.5) return 0;  // round-half-even tie: depends on x's last bit
    int64_t X = (int64_t)ldexp(x, 52 - e);
    int64_t R = (int64_t)qr;
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

// ------------------------------------------------------- interval bound
PT_HD void isq(double lo, double hi, double *a, double *b) {
    if (lo >= 0.0) {
        *a = lo * lo;
        *b = hi * hi;
    } else if (hi <= 0.0) {
        *a = hi * hi;
        *b = lo * lo;
    } else {
        *a = 0.0;
        *b = fmax(lo * lo, hi * hi);
    }
}
// [a] (a >= 0) times [b]
PT_HD void imulpos(double alo, double ahi, double blo, double bhi, double *lo, double *hi) {
    if (blo >= 0.0) {
        *lo = alo * blo;
        *hi = ahi * bhi;
    } else if (bhi <= 0.0) {
        *lo = ahi * blo;
        *hi = alo * bhi;
    } else {
        *lo = ahi * blo;
        *hi = ahi * bhi;
    }
}

// True if every f64 evaluation of heart_f at a point of the box has the sign
// of `sgn` and magnitude >= 1e-15 (so neither the approx_equal stop nor a
// sign change can fire).
PT_HD bool heart_sign_definite(double xlo, double xhi, double ylo, double yhi, double zlo, double zhi,
                               double sgn) {
    double x2l, x2h, y2l, y2h, z2l, z2h;
    isq(xlo, xhi, &x2l, &x2h);
    isq(ylo, yhi, &y2l, &y2h);
    isq(zlo, zhi, &z2l, &z2h);
    double z3l = zlo * zlo * zlo, z3h = zhi * zhi * zhi;
    double al = x2l + 2.25 * y2l + z2l - 1.0, ah = x2h + 2.25 * y2h + z2h - 1.0;
    double a3l = al * al * al, a3h = ah * ah * ah;
    double pl, ph, ql, qh;
    imulpos(x2l, x2h, z3l, z3h, &pl, &ph);
    imulpos(y2l, y2h, z3l, z3h, &ql, &qh);
    double fl = a3l - ph - 0.1125 * qh;
    double fh = a3h - pl - 0.1125 * ql;
    double aa = fmax(fabs(al), fabs(ah));
    double z3a = fmax(fabs(z3l), fabs(z3h));
    double s = aa * aa * aa + x2h * z3a + 0.1125 * y2h * z3a + 3.0 * aa * aa * (x2h + 2.25 * y2h + z2h + 1.0);
    double m = 1e-15 + 1e-14 * s;  // >= 90 ulp-factors of the evaluation error
    return sgn > 0.0 ? fl > m : fh < -m;
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
    int64_t btry = 64;
    bool hit = false;
    for (int pass = 0; pass < passes && !hit; pass++) {
        double cx = dx * s, cy = dy * s, cz = dz * s;
        for (;;) {
            if (t > end || t < start) return false;
            // ---- try to jump a block of B steps
            if (r != 0.0) {
                Lin Lx, Ly, Lz, Lt;
                int64_t bmax = lin_init(px, cx, &Lx);
                if (bmax >= 2) bmax = imin(bmax, lin_init(py, cy, &Ly));
                if (bmax >= 2) bmax = imin(bmax, lin_init(pz, cz, &Lz));
                if (bmax >= 2) bmax = imin(bmax, lin_init(t, s, &Lt));
                int64_t b = imin(bmax, btry);
                bool jumped = false;
                while (b >= 2) {
                    if (STATS) st->tries++;
                    double tl = lin_at(Lt, t, b - 1);  // t before the last step of the block
                    if (tl > end || tl < start) {
                        b >>= 1;
                        continue;
                    }
                    double qx = lin_at(Lx, px, b), qy = lin_at(Ly, py, b), qz = lin_at(Lz, pz, b);
                    if (heart_sign_definite(fmin(px, qx), fmax(px, qx), fmin(py, qy), fmax(py, qy), fmin(pz, qz),
                                            fmax(pz, qz), r)) {
                        t = lin_at(Lt, t, b);
                        px = qx;
                        py = qy;
                        pz = qz;
                        r = heart_f(px, py, pz);
                        if (STATS) st->blocks++;
                        jumped = true;
                        break;
                    }
                    b >>= 1;
                }
                if (jumped) {
                    btry = imin(b * 2, (int64_t)1 << 20);
                    continue;
                }
                btry = 4;
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
                btry = 8;
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
