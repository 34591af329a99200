// pt_device.hpp — device-side math of the sample path, CDNA4 (gfx950), f64.
//
// Every expression keeps the Rust reference's operation order and the file is
// compiled with -ffp-contract=off (rustc never forms an FMA), so each result is
// the IEEE double the reference computes: f64 division and sqrt lower to
// correctly rounded sequences on gfx950.  Citations are to the reference.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "pt_types.hpp"

namespace pt {
namespace dev {

struct V3 {
    double x, y, z;
};
__device__ __forceinline__ V3 v3(double x, double y, double z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }  // algebra/mod.rs:319-349
__device__ __forceinline__ V3 scale(V3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 divs(V3 a, double s) { return v3(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ V3 neg(V3 a) { return v3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ V3 normalize(V3 a) { return divs(a, sqrt(dot(a, a))); }  // :107-110
__device__ __forceinline__ bool approx_zero(double a) { return fabs(a - 0.0) < 1e-15; }  // :14-17

// --------------------------------------------------------------- RNG spec
// SplitMix64 stream keyed by (seed, pixel, sample) — the documented stand-in
// for rand::thread_rng; float conversions are rand 0.8's.
constexpr uint64_t GAMMA = 0x9E3779B97F4A7C15ull;
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t sample_key(uint64_t seed, uint64_t pixel, uint64_t sample) {
    uint64_t k = mix64(seed ^ 0x6A09E667F3BCC909ull);
    k = mix64(k + (pixel + 1) * GAMMA);
    return mix64(k + (sample + 1) * 0xD1B54A32D192ED03ull);
}
struct Rng {
    uint64_t s;
    __device__ __forceinline__ uint64_t next() {
        s += GAMMA;
        return mix64(s);
    }
    // Standard f64: (u >> 11) * 2^-53
    __device__ __forceinline__ double gen() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
    // UniformFloat::sample: ([1,2) from 52 bits) - 1, * scale + low
    __device__ __forceinline__ double uniform(double lo, double sc) {
        double v = __longlong_as_double((long long)((next() >> 12) | (1023ull << 52)));
        return (v - 1.0) * sc + lo;
    }
};

// ---------------------------------------------------------- transforms
// transform_point / transform_vector / transform_normal (algebra/transform.rs:394-425)
__device__ __forceinline__ V3 xf_point(const double *m, V3 p) {
    return v3(p.x * m[0] + p.y * m[1] + p.z * m[2] + m[3], p.x * m[4] + p.y * m[5] + p.z * m[6] + m[7],
              p.x * m[8] + p.y * m[9] + p.z * m[10] + m[11]);
}
__device__ __forceinline__ V3 xf_vector(const double *m, V3 v) {
    return v3(v.x * m[0] + v.y * m[1] + v.z * m[2], v.x * m[4] + v.y * m[5] + v.z * m[6],
              v.x * m[8] + v.y * m[9] + v.z * m[10]);
}
__device__ __forceinline__ V3 xf_normal(const double *m, V3 n) {
    return v3(n.x * m[0] + n.y * m[4] + n.z * m[8], n.x * m[1] + n.y * m[5] + n.z * m[9],
              n.x * m[2] + n.y * m[6] + n.z * m[10]);
}

// ------------------------------------------------------------ primitives
// Each returns true and sets *t on a hit in [min_t, max_t], object space.

// Sphere::ray_intersect (shapes/mod.rs:330-374)
__device__ __forceinline__ bool sphere_t(V3 o, V3 d, double min_t, double max_t, double *t) {
    double a = dot(d, d);
    double hb = dot(d, o);
    double c = dot(o, o) - 1.0;
    double disc = hb * hb - a * c;
    if (disc < 0.0) return false;
    double x;
    if (disc == 0.0) {
        x = -hb * a;  // reference quirk: no division, no range check
    } else {
        double sq = sqrt(disc);
        x = (-hb - sq) / a;
        if (x < min_t || x > max_t) {
            x = (-hb + sq) / a;
            if (x < min_t || x > max_t) return false;
        }
    }
    *t = x;
    return true;
}
// Rectangle::ray_intersect (shapes/mod.rs:181-204)
__device__ __forceinline__ bool rect_t(const double *p, V3 o, V3 d, double min_t, double max_t, double *t) {
    double tt = -o.z / d.z;
    if (tt < min_t || tt > max_t) return false;
    double px = o.x + d.x * tt, py = o.y + d.y * tt;
    if (px < p[0] || px > p[2] || py < p[1] || py > p[3]) return false;
    *t = tt;
    return true;
}
// Cube::ray_intersect (shapes/mod.rs:250-285), slab on [-1, 1]^3
__device__ __forceinline__ bool cube_t(V3 o, V3 d, double min_t, double max_t, double *t) {
    double lx = (-1.0 - o.x) / d.x, ly = (-1.0 - o.y) / d.y, lz = (-1.0 - o.z) / d.z;
    double ux = (1.0 - o.x) / d.x, uy = (1.0 - o.y) / d.y, uz = (1.0 - o.z) / d.z;
    double tmin = fmax(fmax(fmax(fmin(lx, ux), fmin(ly, uy)), fmin(lz, uz)), min_t);
    double tmax = fmin(fmin(fmin(fmax(lx, ux), fmax(ly, uy)), fmax(lz, uz)), max_t);
    if (tmin > tmax || tmin > max_t) return false;
    *t = tmin;
    return true;
}

// Heart (ray_marching.rs:121-188)
__device__ __forceinline__ double heart_f(double px, double py, double pz) {  // :147-155
    double x2 = px * px;
    double y2 = py * py;
    double z2 = pz * pz;
    double z3 = z2 * pz;
    double a = x2 + (9.0 / 4.0) * y2 + z2 - 1.0;
    return a * a * a - x2 * z3 - (9.0 / 80.0) * y2 * z3;
}
__device__ __forceinline__ V3 heart_gradient(V3 p) {  // :157-168 (27/40 kept as in the reference)
    double a = p.x * p.x + (9.0 / 4.0) * p.y * p.y + p.z * p.z - 1.0;
    a = 3.0 * a * a;
    double z2 = p.z * p.z;
    double z3 = z2 * p.z;
    return v3(2.0 * p.x * (a - z3), (9.0 / 2.0) * p.y * (a - 0.05 * z3),
              2.0 * p.z * (a - p.z * (1.5 * p.x * p.x + (27.0 / 40.0) * p.y * p.y)));
}
// Heart::intersect_bound (:135-145) + solve_quadratic_equation (algebra/equation.rs:5-15)
__device__ __forceinline__ bool heart_bound(V3 o, V3 d, double *start, double *end) {
    const double rx = 1.45, ry = 1.45 / 2.05, rz = 1.45;
    V3 oo = v3(o.x / rx, o.y / ry, o.z / rz), dd = v3(d.x / rx, d.y / ry, d.z / rz);
    double a = dot(dd, dd), hb = dot(dd, oo), c = dot(oo, oo) - 1.0;
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
// RayMarchingShape::ray_intersect (ray_marching.rs:20-74), exact fixed-step
// sign-change march with `depth` refinement passes (step *= -0.01).
__device__ __forceinline__ bool march_t(double step0, int passes, V3 o, V3 d, double min_t, double max_t,
                                        double *t_out) {
    double start, end;
    if (!heart_bound(o, d, &start, &end)) return false;
    double step = step0;
    double t = start;
    double px = o.x + d.x * t, py = o.y + d.y * t, pz = o.z + d.z * t;
    double r = heart_f(px, py, pz);
    for (int pass = 0; pass < passes; pass++) {
        double cx = d.x * step, cy = d.y * step, cz = d.z * step;
        bool hit = false;
        for (;;) {
            if (t > end || t < start) return false;
            t += step;
            px += cx;
            py += cy;
            pz += cz;
            double next = heart_f(px, py, pz);
            if (approx_zero(next)) {
                hit = true;
                break;
            }
            if ((r < 0.0 && next > 0.0) || (r > 0.0 && next < 0.0)) {
                step *= -0.01;
                r = next;
                break;
            }
            r = next;
        }
        if (hit) break;
    }
    if (t < min_t || t > max_t) return false;
    *t_out = t;
    return true;
}

// ------------------------------------------------------------ closest hit
struct Ray {
    V3 o, d;
};

__device__ __forceinline__ bool shape_test(const DShape &s, const Ray &r, double min_t, double max_t, double *t) {
    V3 o = xf_point(s.inv, r.o);  // inverse_transform_ray (transform.rs:32-37), no renormalisation
    V3 d = xf_vector(s.inv, r.d);
    switch (s.type) {
    case SPHERE: return sphere_t(o, d, min_t, max_t, t);
    case RECTANGLE: return rect_t(s.p, o, d, min_t, max_t, t);
    case CUBE: return cube_t(o, d, min_t, max_t, t);
    default: return march_t(s.p[0], s.depth, o, d, min_t, max_t, t);
    }
}

// Closest hit over the shape list: ShapeCollection semantics (shapes/mod.rs:587-596),
// max_t shrinks to each accepted distance, later shape wins an exact tie.
__device__ __forceinline__ int closest(const DShape *__restrict__ shapes, int n, const Ray &r, double min_t,
                                       double max_t, double *best_t) {
    double best = max_t;
    int who = -1;
    for (int i = 0; i < n; i++) {
        double t;
        if (shape_test(shapes[i], r, min_t, best, &t)) {
            best = t;
            who = i;
        }
    }
    *best_t = best;
    return who;
}

struct Hit {
    V3 p, n;
    bool front;
};
// ray_hit_transformed (shapes/mod.rs:112-124): world point = direct * p_obj,
// world normal = inverse^T * normalize(n_obj), then RayHit::set_normal (ray.rs:60-64).
__device__ __forceinline__ Hit finish(const DShape &s, const Ray &r, double t) {
    V3 o = xf_point(s.inv, r.o);
    V3 d = xf_vector(s.inv, r.d);
    V3 p = v3(o.x + d.x * t, o.y + d.y * t, o.z + d.z * t);
    V3 n;
    switch (s.type) {
    case SPHERE: n = s.inverse_normal ? neg(p) : p; break;  // :358-359
    case RECTANGLE: n = v3(0.0, 0.0, 1.0); break;         // :195
    case CUBE: {                                          // :270-281
        double ax = fabs(p.x), ay = fabs(p.y), az = fabs(p.z);
        double mc = fmax(fmax(ax, ay), az);
        if (mc == ax) n = v3(p.x, 0.0, 0.0);
        else if (mc == ay) n = v3(0.0, p.y, 0.0);
        else if (mc == az) n = v3(0.0, 0.0, p.z);
        else n = v3(__builtin_nan(""), __builtin_nan(""), __builtin_nan(""));
        break;
    }
    default: n = heart_gradient(p); break;  // ray_marching.rs:59-60
    }
    n = normalize(n);  // RayHit::new (ray.rs:32-52)
    V3 wn = xf_normal(s.inv, n);
    Hit h;
    h.front = dot(wn, r.d) < 0.0;
    h.n = normalize(h.front ? wn : neg(wn));
    h.p = xf_point(s.dir, p);
    return h;
}

// ------------------------------------------------------------ materials
// random_in_unit_sphere (algebra/mod.rs:77-84): rejection in [-1, 1]^3
__device__ __forceinline__ V3 random_in_unit_sphere(Rng &rng, double s11) {
    for (;;) {
        double x = rng.uniform(-1.0, s11);
        double y = rng.uniform(-1.0, s11);
        double z = rng.uniform(-1.0, s11);
        if (x * x + y * y + z * z <= 1.0) return v3(x, y, z);
    }
}
__device__ __forceinline__ V3 reflect(V3 d, V3 n) {  // algebra/mod.rs:122-125
    V3 b = scale(n, dot(d, n));
    return sub(d, scale(b, 2.0));
}
__device__ __forceinline__ V3 refract(V3 d, V3 n, double ratio) {  // :127-133
    double c = dot(neg(d), n);
    V3 perp = scale(add(d, scale(n, c)), ratio);
    double ps = -(sqrt(fabs(1.0 - dot(perp, perp))));
    return add(perp, scale(n, ps));
}
// Scene::background (src/world/mod.rs:199-202)
__device__ __forceinline__ V3 background(V3 d) {
    double t = 0.5 * (d.y + 1.0);
    double u = 1.0 * (1.0 - t);
    return v3(u + 0.5 * t, u + 0.7 * t, u + 1.0 * t);
}

// Attenuation stack: the reference multiplies attenuation ⊙ ray_color(child)
// on the way back up its recursion (renderer/mod.rs:29-33).  Only albedo
// attenuations are pushed (Dielectric's (1,1,1) is an exact identity), as
// 32-bit material ids in NW 64-bit words, unwound after the leaf radiance.
template <int NW>
struct IdStack {
    uint64_t w[NW];
    int n;
    __device__ __forceinline__ void clear() {
#pragma unroll
        for (int i = 0; i < NW; i++) w[i] = 0;
        n = 0;
    }
    __device__ __forceinline__ void push(uint32_t id) {
#pragma unroll
        for (int i = NW - 1; i > 0; i--) w[i] = (w[i] << 32) | (w[i - 1] >> 32);
        w[0] = (w[0] << 32) | id;
        n++;
    }
    __device__ __forceinline__ uint32_t pop() {
        uint32_t id = (uint32_t)w[0];
#pragma unroll
        for (int i = 0; i < NW - 1; i++) w[i] = (w[i] >> 32) | (w[i + 1] << 32);
        w[NW - 1] >>= 32;
        n--;
        return id;
    }
};

struct Scene {
    const DShape *__restrict__ shapes;
    const DMaterial *__restrict__ mats;
    int nshapes;
};

// ray_color (src/renderer/mod.rs:23-45), iterative with exact product order.
template <int NW>
__device__ __forceinline__ V3 ray_color(const Scene &sc, Ray ray, uint32_t depth, Rng &rng, double s11) {
    IdStack<NW> stk;
    stk.clear();
    V3 leaf;
    for (;;) {
        double t;
        int who = closest(sc.shapes, sc.nshapes, ray, T_MIN, __builtin_inf(), &t);
        if (who < 0) {
            leaf = background(ray.d);
            break;
        }
        if (depth == 0) {
            leaf = v3(0.0, 0.0, 0.0);
            break;
        }
        const DShape &s = sc.shapes[who];
        Hit h = finish(s, ray, t);
        const DMaterial &m = sc.mats[s.material];
        V3 dir;
        if (m.type == LAMBERTIAN) {  // material.rs:41-54
            V3 u = normalize(random_in_unit_sphere(rng, s11));
            dir = add(h.n, u);
            if (approx_zero(dir.x) && approx_zero(dir.y) && approx_zero(dir.z)) dir = h.n;
            stk.push((uint32_t)s.material);
        } else if (m.type == METAL) {  // :63-76
            V3 rf = reflect(ray.d, h.n);
            dir = m.fuzz == 0.0 ? rf : add(rf, scale(random_in_unit_sphere(rng, s11), m.fuzz));
            stk.push((uint32_t)s.material);
        } else if (m.type == DIELECTRIC) {  // :92-115
            double ratio = h.front ? 1.0 / m.ior : m.ior;
            double c = dot(neg(ray.d), h.n);
            double sn = sqrt(1.0 - c * c);
            bool refl = ratio * sn > 1.0;
            if (!refl) {
                double r0 = (1.0 - ratio) / (1.0 + ratio);
                r0 = r0 * r0;
                double x = 1.0 - c;
                double x5 = x * ((x * x) * (x * x));  // powi(5)
                refl = r0 + (1.0 - r0) * x5 > rng.gen();
            }
            dir = refl ? reflect(ray.d, h.n) : refract(ray.d, h.n, ratio);
        } else {  // DiffuseLight / EmptyMaterial: no scatter, emitted()
            leaf = m.type == DIFFUSE_LIGHT ? v3(m.emit[0], m.emit[1], m.emit[2]) : v3(0.0, 0.0, 0.0);
            break;
        }
        ray.o = h.p;
        ray.d = normalize(dir);  // Ray::new (ray.rs:12-17)
        depth--;
    }
    V3 c = leaf;
    while (stk.n > 0) {
        const DMaterial &m = sc.mats[stk.pop()];
        c = v3(m.albedo[0] * c.x, m.albedo[1] * c.y, m.albedo[2] * c.z);  // Vector3d::product
    }
    return c;
}

// Camera sample: MultisamplerRayCaster::next (ray_caster.rs:103-118), u then v.
__device__ __forceinline__ Ray camera_ray(const FrameParams &P, uint32_t x, uint32_t y, Rng &rng) {
    double u = rng.gen();
    double v = rng.gen();
    double sx = P.pixel_resolution * ((double)x + u);
    double sy = P.pixel_resolution * ((double)y + v);
    V3 d = v3((P.left_top[0] + P.right[0] * sx) - P.up[0] * sy, (P.left_top[1] + P.right[1] * sx) - P.up[1] * sy,
              (P.left_top[2] + P.right[2] * sx) - P.up[2] * sy);
    V3 pos = v3(P.pos[0], P.pos[1], P.pos[2]);
    Ray r;
    r.o = pos;
    r.d = normalize(sub(d, pos));
    return r;
}

// trace_pixel_samples (renderer/mod.rs:151-155): in-order sum, then / spp.
template <int NW>
__device__ __forceinline__ V3 trace_pixel(const Scene &sc, const FrameParams &P, uint32_t x, uint32_t y) {
    uint64_t pixel = (uint64_t)x + (uint64_t)y * P.width;
    V3 acc = v3(0.0, 0.0, 0.0);
    for (uint32_t s = 0; s < P.spp; s++) {
        Rng rng{sample_key(P.seed, pixel, s)};
        Ray r = camera_ray(P, x, y, rng);
        acc = add(acc, ray_color<NW>(sc, r, P.depth, rng, P.s11));
    }
    return divs(acc, (double)P.spp);
}

}  // namespace dev
}  // namespace pt
