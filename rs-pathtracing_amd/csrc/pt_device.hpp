// pt_device.hpp — the sample path for CDNA4 (gfx950), f64.
//
// Every expression keeps the Rust reference's operation order and the library
// is compiled with -ffp-contract=off (rustc never forms an FMA), so each value
// is the IEEE double the reference computes; f64 division and sqrt lower to
// correctly rounded sequences on gfx950.  Functions are __host__ __device__
// only so that a test-only host build (tests/native) can check the same code
// against the oracle on a CPU; the product runs them on the GPU only.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "pt_lprof.hpp"
#include "pt_march.hpp"
#include "pt_torus.hpp"
#include "pt_types.hpp"

namespace pt {
namespace dev {

// A stop_rendering in flight (pt_render_stop): the frame is being discarded.
// The flag is host-mapped memory, so a read crosses the host link (about a
// microsecond): one lane per launch reads it (stop_gate) or one per block
// (render_tiles), never one per wave of a hot kernel.
__device__ __forceinline__ bool stopped(const int *flag) {
    return flag && __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}

struct V3 {
    double x, y, z;
};
PT_HD V3 v3(double x, double y, double z) { return V3{x, y, z}; }
PT_HD V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
PT_HD V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
PT_HD double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }  // algebra/mod.rs:319-349
PT_HD V3 scale(V3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }
PT_HD V3 divs(V3 a, double s) { return v3(a.x / s, a.y / s, a.z / s); }
PT_HD V3 neg(V3 a) { return v3(-a.x, -a.y, -a.z); }
PT_HD V3 normalize(V3 a) { return divs(a, sqrt(dot(a, a))); }  // :107-110
PT_HD bool approx_zero(double a) { return fabs(a - 0.0) < 1e-15; }  // :14-17

// --------------------------------------------------------------- RNG spec
// SplitMix64 stream keyed by (seed, pixel, sample) — the documented stand-in
// for rand::thread_rng; float conversions are rand 0.8's.
constexpr uint64_t GAMMA = 0x9E3779B97F4A7C15ull;
PT_HD uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
PT_HD uint64_t sample_key(uint64_t seed, uint64_t pixel, uint64_t sample) {
    uint64_t k = mix64(seed ^ 0x6A09E667F3BCC909ull);
    k = mix64(k + (pixel + 1) * GAMMA);
    return mix64(k + (sample + 1) * 0xD1B54A32D192ED03ull);
}
PT_HD double bits_to_double(uint64_t b) {
    union {
        uint64_t u;
        double d;
    } x;
    x.u = b;
    return x.d;
}
struct Rng {
    uint64_t s;
    PT_HD uint64_t next() {
        s += GAMMA;
        return mix64(s);
    }
    // Standard f64: (u >> 11) * 2^-53
    PT_HD double gen() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
    // UniformFloat::sample: ([1,2) from 52 bits) - 1, * scale + low
    PT_HD double uniform(double lo, double sc) {
        double v = bits_to_double((next() >> 12) | (1023ull << 52));
        return (v - 1.0) * sc + lo;
    }
};

// ---------------------------------------------------------- transforms
// transform_point / transform_vector / transform_normal (algebra/transform.rs:394-425)
PT_HD V3 xf_point(const double *m, V3 p) {
    return v3(p.x * m[0] + p.y * m[1] + p.z * m[2] + m[3], p.x * m[4] + p.y * m[5] + p.z * m[6] + m[7],
              p.x * m[8] + p.y * m[9] + p.z * m[10] + m[11]);
}
PT_HD V3 xf_vector(const double *m, V3 v) {
    return v3(v.x * m[0] + v.y * m[1] + v.z * m[2], v.x * m[4] + v.y * m[5] + v.z * m[6],
              v.x * m[8] + v.y * m[9] + v.z * m[10]);
}
PT_HD V3 xf_normal(const double *m, V3 n) {
    return v3(n.x * m[0] + n.y * m[4] + n.z * m[8], n.x * m[1] + n.y * m[5] + n.z * m[9],
              n.x * m[2] + n.y * m[6] + n.z * m[10]);
}

// (Measured and removed in round 6: the rectangles' rejection of rays moving away from the plane before the
// division, C2 2061 -> 2034; the quantized walk loading node n + 1 with node n, C5 2112 -> 2035.)

// ------------------------------------------------------------ primitives
// Each returns true and sets *t on a hit in [min_t, max_t], object space.

// Sphere::ray_intersect (shapes/mod.rs:330-374)
PT_HD bool sphere_t(V3 o, V3 d, double min_t, double max_t, double *t) {
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
// A sphere whose inverse transform is diag(m0, m5, m10) plus a translation (m3, m7, m11) with every
// translation entry nonzero (DShape::axis; add_random_spheres' spheres): xf_point's
// ((o.x m0 + o.y m1) + o.z m2) + m3 adds two zero products (+-0) to o.x m0 and then the nonzero m3, so it is
// fl(o.x m0 + m3) bit for bit, and xf_vector's component is fl(d.x m0) when that product is a nonzero finite
// value (adding +-0 to it changes nothing).  `ray_ok` (axis_ray_ok) is false for a ray with an inf or NaN
// component (inf * 0 = NaN in the full form) or a direction component whose product could vanish: those
// rays take the full transform.
PT_HD bool axis_ray_ok(const V3 &o, const V3 &d) {
    const double sum = o.x + o.y + o.z + d.x + d.y + d.z;  // inf or NaN if any component is
    return sum - sum == 0.0 && fabs(d.x) > 1e-200 && fabs(d.y) > 1e-200 && fabs(d.z) > 1e-200;
}
PT_HD bool sphere_axis_t(const double *m, V3 ro, V3 rd, double min_t, double max_t, double *t) {
    const V3 o = v3(ro.x * m[0] + m[3], ro.y * m[5] + m[7], ro.z * m[10] + m[11]);
    const V3 d = v3(rd.x * m[0], rd.y * m[5], rd.z * m[10]);
    return sphere_t(o, d, min_t, max_t, t);
}
// Rectangle::ray_intersect (shapes/mod.rs:181-204)
PT_HD bool rect_t(const double *p, V3 o, V3 d, double min_t, double max_t, double *t) {
    double tt = -o.z / d.z;
    if (tt < min_t || tt > max_t) return false;
    double px = o.x + d.x * tt, py = o.y + d.y * tt;
    if (px < p[0] || px > p[2] || py < p[1] || py > p[3]) return false;
    *t = tt;
    return true;
}
// Cube::ray_intersect (shapes/mod.rs:250-285), slab on [-1, 1]^3
PT_HD bool cube_t(V3 o, V3 d, double min_t, double max_t, double *t) {
    double lx = (-1.0 - o.x) / d.x, ly = (-1.0 - o.y) / d.y, lz = (-1.0 - o.z) / d.z;
    double ux = (1.0 - o.x) / d.x, uy = (1.0 - o.y) / d.y, uz = (1.0 - o.z) / d.z;
    double tmin = fmax(fmax(fmax(fmin(lx, ux), fmin(ly, uy)), fmin(lz, uz)), min_t);
    double tmax = fmin(fmin(fmin(fmax(lx, ux), fmax(ly, uy)), fmax(lz, uz)), max_t);
    if (tmin > tmax || tmin > max_t) return false;
    *t = tmin;
    return true;
}

// Heart gradient (ray_marching.rs:157-168; the 27/40 coefficient kept as in the reference)
PT_HD V3 heart_gradient(V3 p) {
    double a = p.x * p.x + (9.0 / 4.0) * p.y * p.y + p.z * p.z - 1.0;
    a = 3.0 * a * a;
    double z2 = p.z * p.z;
    double z3 = z2 * p.z;
    return v3(2.0 * p.x * (a - z3), (9.0 / 2.0) * p.y * (a - 0.05 * z3),
              2.0 * p.z * (a - p.z * (1.5 * p.x * p.x + (27.0 / 40.0) * p.y * p.y)));
}

// The implicit function of a ray-marched shape.
PT_HD march::FParams shape_params(const DShape &S) {
    march::FParams F;
    F.func = S.func;
    F.pad = 0;
    F.k[0] = S.fk[0];
    F.k[1] = S.fk[1];
    F.k[2] = S.fk[2];
    F.k[3] = S.fk[3];
    F.radius = S.fradius;
    return F;
}

// ------------------------------------------------------------ closest hit
struct Ray {
    V3 o, d;
};

// Counts a march dropped by the march guard (pt_march_guard_drops).
PT_HD void note_guard(unsigned long long *guard) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (guard) atomicAdd(guard, 1ull);
#else
    if (guard) ++*guard;
#endif
}

// A stop-gated launch that found its frame stopped (pt_render_stop_stats): counters[1] counts them, counters[2]
// those that still had work to do (0 unless the stop gate failed to empty the queue).
PT_HD void note_stop(unsigned long long *counters, bool worked) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (!counters) return;
    atomicAdd(counters + 1, 1ull);
    if (worked) atomicAdd(counters + 2, 1ull);
#else
    (void)counters;
    (void)worked;
#endif
}

// MARCHED=false: the caller's lists hold no ray-marched shape (build_accel puts
// every one on the march list), so the march branch is not compiled in.
// EXT: the extended build (scenes with a Torus or non-solid textures) that
// also carries the Torus' quartic; other builds never see a Torus.
template <bool STATS, int FK = march::F_ANY, bool MARCHED = true, bool EXT = false>
PT_HD bool shape_test(const DShape &s, const Ray &r, double min_t, double max_t, double *t, Ctr *ct,
                      unsigned long long *guard = nullptr) {
    if (STATS) ct->c[s.type == TORUS ? C_TEST_TORUS : C_TEST_SPHERE + s.type]++;
    if (s.type == RECTANGLE) {
        // Rectangle: t needs only the object-space z row; x and y are
        // transformed only for a t in range.  Each component is the same
        // expression as in xf_point / xf_vector, so every value is unchanged.
        const double *m = s.inv;
        const double oz = r.o.x * m[8] + r.o.y * m[9] + r.o.z * m[10] + m[11];
        const double dz = r.d.x * m[8] + r.d.y * m[9] + r.d.z * m[10];
        const double tt = -oz / dz;
        if (tt < min_t || tt > max_t) return false;
        PT_LP(RECT_ROWS);
        const double ox = r.o.x * m[0] + r.o.y * m[1] + r.o.z * m[2] + m[3];
        const double oy = r.o.x * m[4] + r.o.y * m[5] + r.o.z * m[6] + m[7];
        const double dx = r.d.x * m[0] + r.d.y * m[1] + r.d.z * m[2];
        const double dy = r.d.x * m[4] + r.d.y * m[5] + r.d.z * m[6];
        const double px = ox + dx * tt, py = oy + dy * tt;
        if (px < s.p[0] || px > s.p[2] || py < s.p[1] || py > s.p[3]) return false;
        *t = tt;
        return true;
    }
    V3 o = xf_point(s.inv, r.o);  // inverse_transform_ray (transform.rs:32-37), no renormalisation
    V3 d = xf_vector(s.inv, r.d);
    switch (s.type) {
    case SPHERE: return sphere_t(o, d, min_t, max_t, t);
    case RECTANGLE: return rect_t(s.p, o, d, min_t, max_t, t);
    case CUBE: return cube_t(o, d, min_t, max_t, t);
    case TORUS:
        if (!EXT) return false;
        return torus::torus_t(s.p[0], s.p[1], o.x, o.y, o.z, d.x, d.y, d.z, min_t, max_t, t);
    default: {
        if (!MARCHED) return false;
        march::MarchStats ms{0, 0, 0, 0};
        bool h = march::func_march<STATS, FK>(shape_params(s), s.p[0], s.depth, o.x, o.y, o.z, d.x, d.y, d.z, min_t, max_t,
                                          t, &ms);
        if (ms.guard) note_guard(guard);
        if (STATS) {
            ct->c[C_MARCH_STEPS] += ms.steps;
            ct->c[C_MARCH_BLOCKS] += ms.blocks;
            ct->c[C_MARCH_TRIES] += ms.tries;
            ct->c[C_MARCH_GUARD] += ms.guard;
        }
        return h;
    }
    }
}

// Read of scene data at a wave-uniform address: through the constant address
// space, so the compiler may use scalar loads (the scene is read-only while
// kernels run; __restrict__ on struct members does not tell it so).
template <class T>
PT_HD T uniform_load(const T *p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return *(const __attribute__((address_space(4))) T *)p;
#else
    return *p;
#endif
}

// A shape at a wave-uniform address, all fields but `dir` loaded one by one
// (an aggregate copy is folded back to the global pointer); the unused ones
// are dropped by the compiler.
// A wave-uniform shape index from the scene's lists, kept in a scalar
// register: the compiler's uniformity analysis loses it inside loops with
// lane-dependent exits, and then loads the shape with per-lane vector loads
// (C2 bounce +30 % when that happened to the march pre-check's Heart).
PT_HD int uniform_index(int i) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_readfirstlane(i);
#else
    return i;
#endif
}

PT_HD DShape uniform_shape(const DShape *p) {
    DShape s;
#pragma unroll
    for (int k = 0; k < 12; k++) s.inv[k] = uniform_load(&p->inv[k]);
#pragma unroll
    for (int k = 0; k < 4; k++) s.p[k] = uniform_load(&p->p[k]);
    s.type = uniform_load(&p->type);
    s.material = uniform_load(&p->material);
    s.depth = uniform_load(&p->depth);
    s.func = uniform_load(&p->func);
#pragma unroll
    for (int k = 0; k < 4; k++) s.fk[k] = uniform_load(&p->fk[k]);
    s.fradius = uniform_load(&p->fradius);
    return s;
}

PT_HD DBox uniform_box(const DBox *p) {
    DBox b;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        b.lo[k] = uniform_load(&p->lo[k]);
        b.hi[k] = uniform_load(&p->hi[k]);
    }
    return b;
}

// Multi-rank tile deal (world > 1): rank r owns logical tiles k = r + i*world;
// logical tile k sits at column (k % tiles_x + row) % tiles_x of its row, so a
// rank's columns shift by one per row (a diagonal deal) instead of repeating
// in every row when tiles_x is a multiple of world.  world == 1: identity.
PT_HD uint32_t tile_position(uint32_t k, uint32_t tiles_x, uint32_t world) {
    if (world <= 1) return k;
    const uint32_t ty = k / tiles_x;
    return ty * tiles_x + (k % tiles_x + ty) % tiles_x;
}
PT_HD uint32_t tile_logical(uint32_t p, uint32_t tiles_x, uint32_t world) {
    if (world <= 1) return p;
    const uint32_t ty = p / tiles_x;
    return ty * tiles_x + (p % tiles_x + tiles_x - ty % tiles_x) % tiles_x;
}

struct Scene {
    const DShape *__restrict__ shapes;
    const DMaterial *__restrict__ mats;
    const DNodeC *__restrict__ nodes;  // compact form (pt_types.hpp)
    const DQGrid *__restrict__ qnodes;  // quantized form after its grid (large trees; else null)
    const int32_t *__restrict__ leaf;
    const int32_t *__restrict__ lin;
    const int32_t *__restrict__ march;
    const DBox *__restrict__ boxes;
    const DTexture *__restrict__ tex;  // non-solid texture trees (null when the scene has none)
    const DPerlin *__restrict__ perlin;
    const DImage *__restrict__ images;
    const uint8_t *__restrict__ pixels;
    int nnodes, nlin, nmarch, diag;  // diag bit 0: skip marched shapes (timing ablation only)
    int nmats;
    int ext;  // the scene needs the extended (EXT) builds: non-solid textures or a Torus
    float bvh_bound;  // >= |every BVH node plane| (the f32 slab's error bound)
    // marches dropped by the march guard (pt_march.hpp MARCH_GUARD), counted
    // on the device (pt_march_guard_drops); null: not counted
    unsigned long long *guard;
};


// Padded-box slab test against [min_t, max_t] (conservative: boxes are padded
// far beyond the rounding of this test).
PT_HD bool slab(const double *lo, const double *hi, const Ray &r, V3 inv, double min_t, double max_t) {
    double tx1 = (lo[0] - r.o.x) * inv.x, tx2 = (hi[0] - r.o.x) * inv.x;
    double ty1 = (lo[1] - r.o.y) * inv.y, ty2 = (hi[1] - r.o.y) * inv.y;
    double tz1 = (lo[2] - r.o.z) * inv.z, tz2 = (hi[2] - r.o.z) * inv.z;
    double tn = fmax(fmax(fmin(tx1, tx2), fmin(ty1, ty2)), fmax(fmin(tz1, tz2), min_t));
    double tf = fmin(fmin(fmax(tx1, tx2), fmax(ty1, ty2)), fmin(fmax(tz1, tz2), max_t));
    return tn <= tf;
}

// Closest hit with the linear scan's result (ShapeCollection, shapes/mod.rs:587-596):
// a candidate replaces the best one if it is nearer, or equally near and later
// in the shape list — the linear scan's "later shape wins a tie" rule, which
// makes the visiting order (uniform list, BVH, marched shapes last) irrelevant.
// This part covers the uniform list and the BVH; marched shapes follow.
// any: only whether the ray hits something matters (its hit will be shaded
// at depth 0, where ray_color returns black for every hit, mod.rs:25-27):
// the wave leaves the uniform list once each of its lanes has a hit, and a
// lane with a hit skips the BVH.
PT_HD bool wave_all(bool p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __all(p);
#else
    return p;
#endif
}
// A leaf record's sphere with a diagonal inverse transform (DLeafRec::axis): sphere_axis_t on the record's six
// entries, the same operations on the same values.
PT_HD bool sphere_axis_rec(const double *m, V3 ro, V3 rd, double min_t, double max_t, double *t) {
    const V3 o = v3(ro.x * m[0] + m[3], ro.y * m[1] + m[4], ro.z * m[2] + m[5]);
    const V3 d = v3(rd.x * m[0], rd.y * m[1], rd.z * m[2]);
    return sphere_t(o, d, min_t, max_t, t);
}

// One leaf of the BVH (a shape id, or `count` ids from leaf[first]) against (best, who), with the tie rule.
template <bool STATS>
PT_HD void bvh_leaf_test(const Scene &sc, const Ray &r, bool axis_ok, int first, int count, bool direct,
                         double min_t, double &best, int &who, Ctr *ct) {
    for (int k = 0; k < count; k++) {
        int i = direct ? first : sc.leaf[first + k];
        PT_LP(BVH_LEAF);
        double t;
        const DShape &S = sc.shapes[i];
        bool h;
        if (axis_ok && S.axis) {
            if (STATS) ct->c[C_TEST_SPHERE]++;
            h = sphere_axis_t(S.inv, r.o, r.d, min_t, best, &t);
        } else {
            h = shape_test<STATS, march::F_ANY, false>(S, r, min_t, best, &t, ct);
        }
        if (h && (t < best || i > who)) {
            best = t;
            who = i;
        }
    }
}

// QN (with FMA_SLAB; sc.qnodes set): the BVH walk reads the quantized nodes (DNodeQ), 16 bytes
// instead of 32: t = fma(q, gs / d, (g0 - o) / d -/+ e') per plane, the same culling with the grid folded into
// the per-ray offsets and a wider margin (below).
// PART: bit 0 the uniform list, bit 1 the BVH.
template <bool STATS = false, bool EXT = false, bool FMA_SLAB = false, bool QN = false, int PART = 3>
PT_HD void closest_nomarch(const Scene &sc, const Ray &r, V3 inv, double min_t, double *best_t, int *who_out,
                           Ctr *ct = nullptr, bool any = false) {
    double best = *best_t;
    int who = *who_out;
    // wave-uniform list (few JSON shapes): scalar loads of each shape
    for (int k = 0; k < ((PART & 1) ? sc.nlin : 0); k++) {
        if (any && wave_all(who >= 0)) break;
        const int i = uniform_index(uniform_load(&sc.lin[k]));
        const DShape s = uniform_shape(&sc.shapes[i]);
        PT_LP(ULIST_SHAPE);
        if (s.type == CUBE || s.type == SPHERE) {
            // the padded world box first (12 FLOP with the caller's 1/d):
            // a miss there is a miss of the exact test, which costs a full
            // inverse transform and, for a cube, six divisions
            if (STATS) ct->c[C_NODE_SLABS]++;
            const DBox b = uniform_box(&sc.boxes[i]);
            if (!slab(b.lo, b.hi, r, inv, min_t, best)) continue;
            PT_LP(UBOX_PASS);
        }
        double t;
        if (shape_test<STATS, march::F_ANY, false, EXT>(s, r, min_t, best, &t, ct) && (t < best || i > who)) {
            best = t;
            who = i;
        }
    }
    // threaded BVH over the remaining non-marched shapes, in the layout of the
    // ray's direction octant (near child first, pt_accel.hpp).  The octant is
    // the direction's sign bits (a -0 component has 1/d = -inf: its near plane
    // is the box's hi), and the layout stores each box as its near and far
    // planes for that octant, so a node's entry and exit are max(near t's,
    // min_t) and min(far t's, best): 6 min/max instead of 12 (C5 +2.2 %).  The
    // t's round as the symmetric slab's do; a NaN t (1/d infinite and b = o)
    // drops out of fmax/fmin and leaves that axis open (conservative).
    // FMA_SLAB (the wavefront builds for scenes with a large BVH, C5): t =
    // fma(b, 1/d, -o/d), 6 FMAs instead of 6 subtractions and 6 multiplies
    // (C5 +1.7 %); its rounding moves a plane by ~2^-53 (|b| + |o|) as the
    // subtraction's does, far inside the boxes' padding, and an infinite 1/d
    // gives NaN t's (an open axis, conservative).  Not in the other builds:
    // its three live -o/d values cost the C2 bounce kernel 9 % through
    // register allocation (profiles/r3/ab_round3_experiments.txt r3y).
    const int oct = (__builtin_signbit(r.d.x) ? 1 : 0) | (__builtin_signbit(r.d.y) ? 2 : 0) |
                    (__builtin_signbit(r.d.z) ? 4 : 0);
    const DNodeC *nodes = sc.nodes + (size_t)oct * (size_t)sc.nnodes;
    // (FMA_SLAB) -o/d can overflow while 1/d is finite (|d| below ~|o| / 1.8e308): the axis's plane t's would be
    // +-inf and cull the node that holds the hit, so such an axis is left open for this ray (a NaN -o/d makes
    // every t of the axis NaN, which drops out of fmax/fmin): conservative, like an infinite 1/d
    auto open_inf = [](double m) { return __builtin_isinf(m) ? __builtin_nan("") : m; };
    const double mx = FMA_SLAB ? open_inf(-(r.o.x * inv.x)) : 0.0, my = FMA_SLAB ? open_inf(-(r.o.y * inv.y)) : 0.0,
                 mz = FMA_SLAB ? open_inf(-(r.o.z * inv.z)) : 0.0;
    auto tx = [&](float b) { return FMA_SLAB ? __builtin_fma((double)b, inv.x, mx) : ((double)b - r.o.x) * inv.x; };
    auto ty = [&](float b) { return FMA_SLAB ? __builtin_fma((double)b, inv.y, my) : ((double)b - r.o.y) * inv.y; };
    auto tz = [&](float b) { return FMA_SLAB ? __builtin_fma((double)b, inv.z, mz) : ((double)b - r.o.z) * inv.z; };
    // Axis-aligned sphere leaves (DShape::axis) take sphere_axis_t in the large-tree (FMA_SLAB) builds only (C5
    // +3.2 %; in the C2 bounce build the extra path costs 9 % through register allocation: round-4 A/B r4g)
    const bool axis_ok = FMA_SLAB && axis_ray_ok(r.o, r.d);
    // SLAB32 (the FMA_SLAB builds; C5 +1.3 %, r4f): the planes' t in f32, t = fma(b, 1/d, lo) for near planes and
    // fma(b, 1/d, hi) for far ones, lo / hi = fl32(-o/d -/+ e), the widening e = 2^-21 (B + |o|) |1/d| (B >= every
    // plane's |b|) folded into the offset in f64: against the real t = (b - o) / d, the f32 1/d and lo / hi
    // (each one f32 rounding of the f64 value: 2^-24 relative) and the fma's rounding add up to less than
    // 2^-23 ((|b| + |o|) |1/d| + e), so the widened interval contains the real one and the cull stays
    // conservative (1e-30 more covers an f32 flush of tiny values).  The six FMAs run as three packed ones over
    // the node's register pairs (nr0, nr1), (nr2, fr0), (fr1, fr2) (C5 +0.9 %, r4h).  An axis whose
    // 1/d or -o/d does not fit an f32 is left open (NaN t's drop out of fmax/fmin), and so is one whose |1/d| is
    // below 1e-30, where an f32 flush of b * 1/d could exceed the widening; min_t is rounded down and best up.
    // The hits are decided by the exact f64 leaf tests as in every walk.
    constexpr bool S32 = FMA_SLAB;
    constexpr bool Q = S32 && QN;
    auto axis32 = [&](double o, double iv, float *i32, float *lo32, float *hi32) {
        const double m = -(o * iv);
        const bool fits = fabs(iv) < 1e30 && fabs(iv) > 1e-30 && fabs(m) < 1e30;
        const double e = (0x1p-21 * (1.0 + 0x1p-20)) * ((double)sc.bvh_bound + fabs(o)) * fabs(iv) + 1e-30;
        *i32 = (float)iv;
        *lo32 = fits ? (float)(m - e) : __builtin_nanf("");
        *hi32 = fits ? (float)(m + e) : __builtin_nanf("");
    };
    // QN: plane b = g0 + q gs (exact), so t = (b - o) / d = q (gs / d) + (g0 / d - o / d).  With i32 = fl32(1/d),
    // si = gs * i32 (exact: gs is a power of two; |si| > 1e-30 is required, so no f32 flush), gl = fl32(g0 * i32
    // + (m -/+ e')) and the fma's one rounding, the computed t is off the widened real t by at most
    // 2^-24 (3B + 2|o|) |1/d| + 2^-23 e' (B >= |b|, |g0|: DQGrid::bound), far inside e' = 2^-19 (B + |o|) |1/d|:
    // the culling stays conservative.  An axis whose values do not fit f32 is left open (NaN t's), as above.
    auto axisq = [&](int k, double o, double iv, float *si, float *gln, float *glf) {
        const double m = -(o * iv);
        const float i32 = (float)iv;
        const double s64 = (double)i32 * sc.qnodes->gs[k];
        const double e = 0x1p-19 * ((double)sc.qnodes->bound + fabs(o)) * fabs(iv) + 1e-30;
        const double g = sc.qnodes->g0[k] * (double)i32;
        const bool fits = fabs(iv) < 1e30 && fabs(iv) > 1e-30 && fabs(m) < 1e30 && fabs(s64) > 1e-30 &&
                          fabs(s64) < 1e30 && fabs(g) < 1e30;
        *si = (float)s64;
        *gln = fits ? (float)(g + (m - e)) : __builtin_nanf("");
        *glf = fits ? (float)(g + (m + e)) : __builtin_nanf("");
    };
    float ix = 0.f, iy = 0.f, iz = 0.f, lox = 0.f, loy = 0.f, loz = 0.f, hix = 0.f, hiy = 0.f, hiz = 0.f;
    if (Q) {
        axisq(0, r.o.x, inv.x, &ix, &lox, &hix);
        axisq(1, r.o.y, inv.y, &iy, &loy, &hiy);
        axisq(2, r.o.z, inv.z, &iz, &loz, &hiz);
    } else if (S32) {
        axis32(r.o.x, inv.x, &ix, &lox, &hix);
        axis32(r.o.y, inv.y, &iy, &loy, &hiy);
        axis32(r.o.z, inv.z, &iz, &loz, &hiz);
    }
    typedef float f2v __attribute__((ext_vector_type(2)));
    const f2v pa_i = {ix, iy}, pa_m = {lox, loy}, pb_i = {iz, ix}, pb_m = {loz, hix}, pc_i = {iy, iz},
              pc_m = {hiy, hiz};
    const float mt32 = S32 ? (float)(min_t - fabs(min_t) * 0x1p-20) : 0.f;
    float best32 = S32 ? (float)(best + fabs(best) * 0x1p-20) : 0.f;
    // The large-tree builds start inside the root: its box holds the whole tree, and nearly every ray of such a
    // scene starts in it (a field of shapes the paths bounce within), so its test is spent work (C5 node tests per
    // sample 120.6 -> 117.9, +0.9 %, r4p); a ray that misses it tests the root's children instead, and the
    // culling stays exact either way.  Small trees keep the test: most of cornell's rays miss its BVH's root
    // (node tests per sample 15.4 -> 20.6 without it).
    int n = any && who >= 0 ? sc.nnodes : (FMA_SLAB && sc.nnodes > 1 ? 1 : 0);
    if (!(PART & 2)) n = sc.nnodes;
    if (Q) {  // the quantized layouts
        const DNodeQ *qn = (const DNodeQ *)(sc.qnodes + 1) + (size_t)oct * (size_t)sc.nnodes;
        while (n < sc.nnodes) {
            const uint4 raw = *(const uint4 *)(qn + n);
            PT_LP(BVH_NODE);
            if (STATS) ct->c[C_NODE_SLABS]++;
            const f2v a = __builtin_elementwise_fma((f2v){(float)(raw.x & 0xffffu), (float)(raw.x >> 16)}, pa_i, pa_m);
            const f2v b = __builtin_elementwise_fma((f2v){(float)(raw.y & 0xffffu), (float)(raw.y >> 16)}, pb_i, pb_m);
            const f2v c = __builtin_elementwise_fma((f2v){(float)(raw.z & 0xffffu), (float)(raw.z >> 16)}, pc_i, pc_m);
            const bool enter = fmaxf(fmaxf(a.x, a.y), fmaxf(b.x, mt32)) <= fminf(fminf(b.y, c.x), fminf(c.y, best32));
            const uint32_t link = raw.w;
            if (enter) {
                PT_LP(BVH_ENTER);
                if (link >> 31) {  // a leaf
                    const int first = (int)(link & 0xffffffu), count = (int)(link >> 24 & 0x3fu);
                    if ((link >> 30) & 1u) {  // a one-shape leaf's 64-byte record
                        const DLeafRec &L = ((const DLeafRec *)((const char *)sc.qnodes + qleaf_offset(sc.nnodes)))[first];
                        const int i = L.shape;
                        double t;
                        bool h;
                        if (axis_ok && L.axis) {
                            if (STATS) ct->c[C_TEST_SPHERE]++;
                            h = sphere_axis_rec(L.m, r.o, r.d, min_t, best, &t);
                        } else {
                            h = shape_test<STATS, march::F_ANY, false>(sc.shapes[i], r, min_t, best, &t, ct);
                        }
                        if (h && (t < best || i > who)) {
                            best = t;
                            who = i;
                        }
                    } else {
                        bvh_leaf_test<STATS>(sc, r, axis_ok, first, count, (link >> 30) & 1u, min_t, best, who, ct);
                    }
                    best32 = (float)(best + fabs(best) * 0x1p-20);
                }
                n++;
            } else {
                n = (link >> 31) ? n + 1 : (int)link;  // a leaf's skip is the next node
            }
        }
    }
    while (!Q && n < sc.nnodes) {
        const DNodeC nd = nodes[n];
        PT_LP(BVH_NODE);
        if (STATS) ct->c[C_NODE_SLABS]++;
        bool enter;
        if (S32) {
            const f2v a = __builtin_elementwise_fma((f2v){nd.nr[0], nd.nr[1]}, pa_i, pa_m);
            const f2v b = __builtin_elementwise_fma((f2v){nd.nr[2], nd.fr[0]}, pb_i, pb_m);
            const f2v c = __builtin_elementwise_fma((f2v){nd.fr[1], nd.fr[2]}, pc_i, pc_m);
            enter = fmaxf(fmaxf(a.x, a.y), fmaxf(b.x, mt32)) <= fminf(fminf(b.y, c.x), fminf(c.y, best32));
        } else {
            const double tn = fmax(fmax(tx(nd.nr[0]), ty(nd.nr[1])), fmax(tz(nd.nr[2]), min_t));
            const double tf = fmin(fmin(tx(nd.fr[0]), ty(nd.fr[1])), fmin(tz(nd.fr[2]), best));
            enter = tn <= tf;
        }
        if (enter) {
            PT_LP(BVH_ENTER);
            const int first = (int)(nd.first_count & 0xffffffu), count = (int)(nd.first_count >> 24 & 0x7fu);
            const bool direct = nd.first_count >> 31;  // one-shape leaf: `first` is the shape id
            bvh_leaf_test<STATS>(sc, r, axis_ok, first, count, direct, min_t, best, who, ct);
            if (S32) best32 = (float)(best + fabs(best) * 0x1p-20);
            n++;
        } else {
            n = nd.skip;
        }
    }
    *best_t = best;
    *who_out = who;
}

template <bool STATS = false, bool EXT = false>
PT_HD int closest(const Scene &sc, const Ray &r, double min_t, double max_t, double *best_t, Ctr *ct = nullptr) {
    double best = max_t;
    int who = -1;
    V3 inv = v3(1.0 / r.d.x, 1.0 / r.d.y, 1.0 / r.d.z);
    closest_nomarch<STATS, EXT>(sc, r, inv, min_t, &best, &who, ct);
    // ray-marched shapes last, only if their padded box is entered before `best`
    for (int k = 0; k < ((sc.diag & 1) ? 0 : sc.nmarch); k++) {
        int i = sc.march[k];
        const DBox &b = sc.boxes[i];
        if (STATS) ct->c[C_MARCH_SLABS]++;
        if (!slab(b.lo, b.hi, r, inv, min_t, best)) continue;
        double t;
        if (shape_test<STATS>(sc.shapes[i], r, min_t, best, &t, ct, sc.guard) && (t < best || i > who)) {
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
template <int FK = march::F_ANY>
PT_HD Hit finish(const DShape &s, const Ray &r, double t) {
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
    case TORUS:  // mod.rs:465: p - normalize((p.x, p.y, 0)) * radius
        n = sub(p, scale(normalize(v3(p.x, p.y, 0.0)), s.p[0]));
        break;
    default: {  // ray_marching.rs:59-60: the function's gradient at p
        double g[3];
        march::shape_gradient_k<FK>(shape_params(s), p.x, p.y, p.z, g);
        n = v3(g[0], g[1], g[2]);
        break;
    }
    }
    n = normalize(n);  // RayHit::new (ray.rs:32-52)
    V3 wn = xf_normal(s.inv, n);
    Hit h;
    h.front = dot(wn, r.d) < 0.0;
    h.n = normalize(h.front ? wn : neg(wn));
    h.p = xf_point(s.dir, p);
    return h;
}

// (u, v) of a hit as each ray_intersect computes them from the object-space
// point (only textures read them): Sphere shapes/mod.rs:361-373, Rectangle
// :189-190, Cube :263-282, ray-marched shapes ray_marching.rs:60 (Heart, Sine,
// Star :170, :239, :302 give (0, 0); DupinCyclide, HuntsSurface, Cushion
// :371, :436, :506 give (p.x, p.y)).
PT_HD void hit_uv(const DShape &s, const Ray &r, double t, double *u, double *v) {
    V3 o = xf_point(s.inv, r.o);
    V3 d = xf_vector(s.inv, r.d);
    V3 p = v3(o.x + d.x * t, o.y + d.y * t, o.z + d.z * t);
    const double PI = 3.141592653589793;
    switch (s.type) {
    case SPHERE: {
        const double theta = acos(-p.y);
        const double phi = atan2(-p.z, p.x) + PI;
        *u = phi / (2.0 * PI);
        *v = theta / PI;
        return;
    }
    case RECTANGLE:
        *u = (p.x - s.p[0]) / (s.p[2] - s.p[0]);
        *v = (p.y - s.p[1]) / (s.p[3] - s.p[1]);
        return;
    case CUBE: {
        double ax = fabs(p.x), ay = fabs(p.y), az = fabs(p.z);
        double mc = fmax(fmax(ax, ay), az);
        if (mc == ax) *u = p.y, *v = p.z;
        else if (mc == ay) *u = p.x, *v = p.z;
        else if (mc == az) *u = p.x, *v = p.y;
        else *u = *v = __builtin_nan("");
        return;
    }
    case TORUS: {  // mod.rs:466-467
        const double theta = asin(p.z / s.p[1]);
        const double phi = acos(p.z / (s.p[0] + s.p[1] * cos(theta))) + PI;
        *u = phi / (2.0 * PI);
        *v = theta / PI;
        return;
    }
    default:
        if (s.func == march::F_DUPIN || s.func == march::F_HUNTS || s.func == march::F_CUSHION) *u = p.x, *v = p.y;
        else *u = *v = 0.0;
        return;
    }
}

// Rust `f64 as i32` / `as u32`: saturating, NaN -> 0.
PT_HD int32_t sat_i32(double x) {
    if (!(x == x)) return 0;
    if (x >= 2147483647.0) return 2147483647;
    if (x <= -2147483648.0) return -2147483647 - 1;
    return (int32_t)x;
}
PT_HD uint32_t sat_u32(double x) {
    if (!(x > 0.0)) return 0u;
    if (x >= 4294967295.0) return 4294967295u;
    return (uint32_t)x;
}

// Perlin::noise (src/algebra/noise.rs:44-74): the 8 corners in
// multi_cartesian_product order (last index fastest), summed in order.
PT_HD double perlin_noise(const DPerlin &P, V3 p) {
    const double fx = floor(p.x), fy = floor(p.y), fz = floor(p.z);
    const uint32_t x = (uint32_t)sat_i32(fx), y = (uint32_t)sat_i32(fy), z = (uint32_t)sat_i32(fz);
    const double u = p.x - fx, v = p.y - fy, w = p.z - fz;
    const double u2 = u * u * (3.0 - 2.0 * u);
    const double v2 = v * v * (3.0 - 2.0 * v);
    const double w2 = w * w * (3.0 - 2.0 * w);
    double acc = 0.0;
    for (int c = 0; c < 8; c++) {
        const int d0 = c >> 2, d1 = (c >> 1) & 1, d2 = c & 1;
        const int32_t k = P.perm[0][(x + (uint32_t)d0) & 255u] ^ P.perm[1][(y + (uint32_t)d1) & 255u] ^
                          P.perm[2][(z + (uint32_t)d2) & 255u];
        const double fi = (double)d0, fj = (double)d1, fk = (double)d2;
        const double dot = P.ranvec[k][0] * (u - fi) + P.ranvec[k][1] * (v - fj) + P.ranvec[k][2] * (w - fk);
        acc = acc + (fi * u2 + (double)(1 - d0) * (1.0 - u2)) * (fj * v2 + (double)(1 - d1) * (1.0 - v2)) *
                        (fk * w2 + (double)(1 - d2) * (1.0 - w2)) * dot;
    }
    return acc;
}
// Perlin::turb (:76-88) as the reference runs it: every octave samples the
// unscaled p (its temp_p is never read), weights 1, 1/2, ..., 1/64.
PT_HD double perlin_turb(const DPerlin &P, V3 p) {
    const double n = perlin_noise(P, p);
    double acc = 0.0, weight = 1.0;
    for (int i = 0; i < 7; i++) {
        acc = acc + weight * n;
        weight *= 0.5;
    }
    return fabs(acc);
}

// Texture::value (src/world/texture.rs) down the tree from `node`.
PT_HD V3 tex_value(const Scene &sc, int node, double u, double v, V3 p) {
    const double PI = 3.141592653589793;
    for (int guard = 0; guard < 64; guard++) {
        const DTexture &t = sc.tex[node];
        switch (t.type) {
        case TEX_SOLID: return v3(t.c[0], t.c[1], t.c[2]);
        case TEX_CHECKER: {  // :40-51
            const double sines = sin(t.c[0] * p.x) * sin(t.c[1] * p.y) * sin(t.c[2] * p.z);
            node = sines < 0.0 ? t.odd : t.even;
            break;
        }
        case TEX_UVCHECKER: {  // :76-87
            const double sines = sin(v * t.c[0] * PI) * sin(u * t.c[1] * PI);
            node = sines < 0.0 ? t.odd : t.even;
            break;
        }
        case TEX_NOISE: {  // :60-66
            const double s = 0.5 * (1.0 + sin(t.c[0] * p.z + 10.0 * perlin_turb(sc.perlin[t.aux], p)));
            return v3(1.0 * s, 1.0 * s, 1.0 * s);
        }
        default: {  // TEX_IMAGE :96-116 (get_pixel panics at u = 1 or v = 0; clamped here)
            const DImage im = sc.images[t.aux];
            const double uc = u < 0.0 ? 0.0 : (u > 1.0 ? 1.0 : u);
            const double vc = 1.0 - (v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v));
            uint32_t x = sat_u32(uc * (double)im.width), y = sat_u32(vc * (double)im.height);
            x = x < im.width ? x : im.width - 1;
            y = y < im.height ? y : im.height - 1;
            const uint8_t *px = sc.pixels + im.offset + ((size_t)y * im.width + x) * 4;
            const double cs = 1.0 / 255.0;
            return v3((double)px[0] * cs, (double)px[1] * cs, (double)px[2] * cs);
        }
        }
    }
    return v3(__builtin_nan(""), __builtin_nan(""), __builtin_nan(""));
}

// Diagnostic phase timing (TIMING build only): wave-level s_memtime deltas.
struct PhaseTimes {
    uint64_t trace, march, select, shade, passes, march_passes, finish, scatter, restart;
};
#if defined(__HIP_DEVICE_COMPILE__)
#define PT_STAMP() __builtin_amdgcn_s_memtime()
#else
#define PT_STAMP() 0ull
#endif

// ------------------------------------------------------------ materials
// random_in_unit_sphere (algebra/mod.rs:77-84): rejection in [-1, 1]^3
template <bool STATS = false>
PT_HD V3 random_in_unit_sphere(Rng &rng, double s11, Ctr *ct = nullptr) {
    for (;;) {
        PT_LP(REJECT_TRY);
        if (STATS) ct->c[C_REJECT_TRIES]++;
        double x = rng.uniform(-1.0, s11);
        double y = rng.uniform(-1.0, s11);
        double z = rng.uniform(-1.0, s11);
        if (x * x + y * y + z * z <= 1.0) return v3(x, y, z);
    }
}
PT_HD V3 reflect(V3 d, V3 n) {  // algebra/mod.rs:122-125
    V3 b = scale(n, dot(d, n));
    return sub(d, scale(b, 2.0));
}
PT_HD V3 refract(V3 d, V3 n, double ratio) {  // :127-133
    double c = dot(neg(d), n);
    V3 perp = scale(add(d, scale(n, c)), ratio);
    double ps = -(sqrt(fabs(1.0 - dot(perp, perp))));
    return add(perp, scale(n, ps));
}
// Scene::background (src/world/mod.rs:199-202)
PT_HD V3 background(V3 d) {
    double t = 0.5 * (d.y + 1.0);
    double u = 1.0 * (1.0 - t);
    return v3(u + 0.5 * t, u + 0.7 * t, u + 1.0 * t);
}

// Attenuation stack: the reference multiplies attenuation ⊙ ray_color(child)
// on the way back up its recursion (renderer/mod.rs:29-33).  Only albedo
// attenuations are pushed (Dielectric's (1,1,1) is an exact identity), as
// 32-bit material ids in NW 64-bit words, unwound after the leaf radiance.
// A textured albedo depends on the hit: its value is stored at the entry's
// level in memory (vb[(level * 3 + c) * vs]) and the entry is VAL_BIT.
constexpr uint32_t VAL_BIT = 0x80000000u;
template <int NW>
struct IdStack {
    uint64_t w[NW];
    int n;
    double *vb = nullptr;  // textured attenuation values (scenes with textures only)
    size_t vs = 0;
    PT_HD void push_val(V3 a) {
        vb[(size_t)(n * 3 + 0) * vs] = a.x;
        vb[(size_t)(n * 3 + 1) * vs] = a.y;
        vb[(size_t)(n * 3 + 2) * vs] = a.z;
        push(VAL_BIT);
    }
    PT_HD V3 val(int level) const {
        return v3(vb[(size_t)(level * 3 + 0) * vs], vb[(size_t)(level * 3 + 1) * vs], vb[(size_t)(level * 3 + 2) * vs]);
    }
    PT_HD void clear() {
#pragma unroll
        for (int i = 0; i < NW; i++) w[i] = 0;
        n = 0;
    }
    PT_HD void push(uint32_t id) {
#pragma unroll
        for (int i = NW - 1; i > 0; i--) w[i] = (w[i] << 32) | (w[i - 1] >> 32);
        w[0] = (w[0] << 32) | id;
        n++;
    }
    PT_HD uint32_t pop() {
        uint32_t id = (uint32_t)w[0];
#pragma unroll
        for (int i = 0; i < NW - 1; i++) w[i] = (w[i] >> 32) | (w[i + 1] << 32);
        w[NW - 1] >>= 32;
        n--;
        return id;
    }
};

// One bounce of ray_color (src/renderer/mod.rs:23-45).  Returns true when the
// path ends, with the leaf radiance in *leaf; otherwise advances ray/depth.
// Everything in a bounce after the closest hit (who, t) is known.
// Stack: any type with push(id), pop() and a count n (IdStack in registers,
// or the wavefront engine's per-slot id array in HBM).
// EXT: the build for scenes with non-solid textures or a Torus (textured albedos are
// evaluated at the hit and pushed by value; textured lights emit their value).
template <bool STATS = false, int FK = march::F_ANY, bool EXT = false, class Stack>
PT_HD bool shade(const Scene &sc, int who, double t, Ray &ray, uint32_t &depth, Stack &stk, Rng &rng,
                 double s11, V3 *leaf, Ctr *ct = nullptr, uint64_t *tfin = nullptr) {
    if (who < 0) {
        *leaf = background(ray.d);
        return true;
    }
    if (depth == 0) {
        *leaf = v3(0.0, 0.0, 0.0);
        return true;
    }
    const DShape &s = sc.shapes[who];
    if (STATS) ct->c[C_HITS]++;
    PT_LP(SHADE_HIT);
    Hit h = finish<FK>(s, ray, t);
    const DMaterial &m = sc.mats[s.material];
    if (tfin) *tfin = PT_STAMP();
    // the texture value at this hit (RayHit u, v and world point)
    auto textured = [&]() {
        double u, v;
        hit_uv(s, ray, t, &u, &v);
        return tex_value(sc, m.tex, u, v, h.p);
    };
    V3 dir;
    if (m.type == LAMBERTIAN) {  // material.rs:41-54
        PT_LP(LAMBERT);
        if (STATS) ct->c[C_LAMBERT]++;
        V3 u = normalize(random_in_unit_sphere<STATS>(rng, s11, ct));
        dir = add(h.n, u);
        if (approx_zero(dir.x) && approx_zero(dir.y) && approx_zero(dir.z)) dir = h.n;
        if (EXT && m.tex >= 0) stk.push_val(textured());
        else stk.push((uint32_t)s.material);
    } else if (m.type == METAL) {  // :63-76
        PT_LP(METAL);
        if (STATS) ct->c[C_METAL]++;
        V3 rf = reflect(ray.d, h.n);
        dir = m.fuzz == 0.0 ? rf : add(rf, scale(random_in_unit_sphere<STATS>(rng, s11, ct), m.fuzz));
        if (EXT && m.tex >= 0) stk.push_val(textured());
        else stk.push((uint32_t)s.material);
    } else if (m.type == DIELECTRIC) {  // :92-115
        PT_LP(DIELECTRIC);
        if (STATS) ct->c[C_DIELECTRIC]++;
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
        PT_LP(EMIT);
        if (EXT && m.type == DIFFUSE_LIGHT && m.tex >= 0) *leaf = textured();
        else *leaf = m.type == DIFFUSE_LIGHT ? v3(m.emit[0], m.emit[1], m.emit[2]) : v3(0.0, 0.0, 0.0);
        return true;
    }
    ray.o = h.p;
    ray.d = normalize(dir);  // Ray::new (ray.rs:12-17)
    depth--;
    return false;
}

template <int NW, bool STATS = false, bool EXT = false>
PT_HD bool bounce(const Scene &sc, Ray &ray, uint32_t &depth, IdStack<NW> &stk, Rng &rng, double s11, V3 *leaf,
                  Ctr *ct = nullptr) {
    double t;
    if (STATS) ct->c[C_BOUNCES]++;
    int who = closest<STATS, EXT>(sc, ray, T_MIN, __builtin_inf(), &t, ct);
    return shade<STATS, march::F_ANY, EXT>(sc, who, t, ray, depth, stk, rng, s11, leaf, ct);
}

template <bool STATS = false, bool EXT = false, class Stack>
PT_HD V3 unwind(const Scene &sc, Stack &stk, V3 c, Ctr *ct = nullptr) {
    while (stk.n > 0) {
        if (STATS) ct->c[C_UNWIND]++;
        const uint32_t id = stk.pop();
        if (EXT && (id & VAL_BIT)) {
            const V3 a = stk.val(stk.n);
            c = v3(a.x * c.x, a.y * c.y, a.z * c.z);
        } else {
            const DMaterial &m = sc.mats[id];
            c = v3(m.albedo[0] * c.x, m.albedo[1] * c.y, m.albedo[2] * c.z);  // Vector3d::product
        }
    }
    return c;
}

// ray_color (src/renderer/mod.rs:23-45), iterative with the recursion's product order.
// vb, vs: the textured-attenuation area of this lane (EXT builds).
template <int NW, bool EXT = false>
PT_HD V3 ray_color(const Scene &sc, Ray ray, uint32_t depth, Rng &rng, double s11, double *vb = nullptr,
                   size_t vs = 0) {
    IdStack<NW> stk;
    stk.clear();
    stk.vb = vb;
    stk.vs = vs;
    V3 leaf;
    while (!bounce<NW, false, EXT>(sc, ray, depth, stk, rng, s11, &leaf)) {
    }
    return unwind<false, EXT>(sc, stk, leaf);
}

// Camera sample: MultisamplerRayCaster::next (ray_caster.rs:103-118), u then v.
PT_HD Ray camera_ray(const FrameParams &P, uint32_t x, uint32_t y, Rng &rng) {
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
//
// Each lane runs its pixel's samples as a small state machine, one pass of the
// loop at a time:  TRACE (uniform list + BVH) -> SELECT (next marched shape
// whose box is entered before the best hit; start its march) -> MARCH (a few
// march iterations per pass) -> SHADE (hit point, scatter or leaf radiance;
// next bounce or next sample).  A lane that is marching the Heart no longer
// holds its whole wave: the other lanes keep tracing their own paths in the
// same passes.  The per-lane sequence of operations, and so every value, is
// the reference's.
constexpr int MARCH_ITERS = 2;  // march iterations per pass of the loop

enum Phase : int { PH_TRACE = 0, PH_SELECT = 1, PH_MARCH = 2, PH_SHADE = 3 };


template <int NW, bool STATS = false, bool TIMING = false, int FK = march::F_ANY, bool EXT = false>
PT_HD V3 trace_pixel(const Scene &sc, const FrameParams &P, uint32_t x, uint32_t y, Ctr *ct = nullptr,
                     PhaseTimes *pt = nullptr, double *vb = nullptr, size_t vs = 0) {
    uint64_t pixel = (uint64_t)x + (uint64_t)y * P.width;
    V3 acc = v3(0.0, 0.0, 0.0);
    uint32_t s = 0;
    Rng rng{sample_key(P.seed, pixel, 0)};
    Ray ray = camera_ray(P, x, y, rng);
    uint32_t depth = P.depth;
    IdStack<NW> stk;
    stk.clear();
    stk.vb = vb;
    stk.vs = vs;
    const int nmarch = (sc.diag & 1) ? 0 : sc.nmarch;
    int phase = PH_TRACE, who = -1, km = 0, mshape = -1;
    double best = 0.0;
    V3 inv = v3(0.0, 0.0, 0.0);
    march::MarchState ms;
    march::MarchStats mst{0, 0, 0, 0};
    uint64_t ts = 0;
    for (;;) {
        if (TIMING) {
            ts = PT_STAMP();
            pt->passes++;
        }
        if (phase == PH_TRACE) {
            if (STATS) ct->c[C_BOUNCES]++;
            inv = v3(1.0 / ray.d.x, 1.0 / ray.d.y, 1.0 / ray.d.z);
            best = __builtin_inf();
            who = -1;
            closest_nomarch<STATS, EXT>(sc, ray, inv, T_MIN, &best, &who, ct);
            km = 0;
            phase = PH_SELECT;
        }
        if (TIMING) {
            uint64_t n = PT_STAMP();
            pt->trace += n - ts;
            ts = n;
        }
        if (phase == PH_MARCH) {
            if (TIMING) pt->march_passes++;
            for (int it = 0; it < MARCH_ITERS; it++) {
                int st = march::march_step<STATS, true, FK>(ms, &mst);
                if (st != march::M_RUNNING) {
                    if (st == march::M_GUARD) {
                        note_guard(sc.guard);
                        if (STATS) ct->c[C_MARCH_GUARD]++;
                    }
                    // final test of ray_marching.rs:55-57 against [T_MIN, best], then the tie rule
                    if (st == march::M_DONE && !(ms.t < T_MIN || ms.t > best) && (ms.t < best || mshape > who)) {
                        best = ms.t;
                        who = mshape;
                    }
                    phase = PH_SELECT;
                    break;
                }
            }
        }
        if (TIMING) {
            uint64_t n = PT_STAMP();
            pt->march += n - ts;
            ts = n;
        }
        if (phase == PH_SELECT) {
            phase = PH_SHADE;
            while (km < nmarch) {
                int i = sc.march[km++];
                const DBox &b = sc.boxes[i];
                if (STATS) ct->c[C_MARCH_SLABS]++;
                if (!slab(b.lo, b.hi, ray, inv, T_MIN, best)) continue;
                const DShape &S = sc.shapes[i];
                if (STATS) ct->c[C_TEST_MARCH]++;
                V3 o = xf_point(S.inv, ray.o), d = xf_vector(S.inv, ray.d);
                if (march::march_begin<FK>(shape_params(S), S.p[0], S.depth, o.x, o.y, o.z, d.x, d.y, d.z, &ms)) {
                    mshape = i;
                    phase = PH_MARCH;
                    break;
                }
            }
        }
        if (TIMING) {
            uint64_t n = PT_STAMP();
            pt->select += n - ts;
            ts = n;
        }
        if (phase == PH_SHADE) {
            V3 leaf;
            uint64_t tf = 0;
            const bool ended = shade<STATS, FK, EXT>(sc, who, best, ray, depth, stk, rng, P.s11, &leaf, ct,
                                                     TIMING ? &tf : nullptr);
            if (TIMING) {
                uint64_t n = PT_STAMP();
                if (tf) {
                    pt->finish += tf - ts;
                    pt->scatter += n - tf;
                }
                ts = n;
            }
            if (ended) {
                acc = add(acc, unwind<STATS, EXT>(sc, stk, leaf, ct));
                if (STATS) ct->c[C_SAMPLES]++;
                if (++s == P.spp) break;
                rng.s = sample_key(P.seed, pixel, s);
                ray = camera_ray(P, x, y, rng);
                depth = P.depth;
            }
            phase = PH_TRACE;
        }
        if (TIMING) pt->restart += PT_STAMP() - ts;
    }
    if (TIMING) pt->restart += PT_STAMP() - ts;
    if (STATS) {
        ct->c[C_MARCH_STEPS] += mst.steps;
        ct->c[C_MARCH_BLOCKS] += mst.blocks;
        ct->c[C_MARCH_TRIES] += mst.tries;
    }
    return divs(acc, (double)P.spp);
}

}  // namespace dev
}  // namespace pt
