/*
 * pt_oracle.c — CPU restatement of the rs-pathtracing sample path.
 *
 * TEST INFRASTRUCTURE ONLY (see pt_oracle.h).  Compiled with
 * -O2 -ffp-contract=off -fno-fast-math so that every f64 operation is a
 * single IEEE operation in source order, as in the Rust reference (rustc
 * never contracts a*b+c).  Expressions are written with the Rust evaluation
 * order spelled out; each function cites the reference file:line it follows.
 */
#include "pt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

/* ======================================================================= */
/* Vector3d (src/algebra/mod.rs)                                           */
/* ======================================================================= */
typedef struct {
    double x, y, z;
} v3;

static inline v3 V(double x, double y, double z) {
    v3 r = {x, y, z};
    return r;
}
static inline v3 vload(const double *p) { return V(p[0], p[1], p[2]); }
static inline void vstore(double *p, v3 a) {
    p[0] = a.x;
    p[1] = a.y;
    p[2] = a.z;
}
/* Add / Sub: mod.rs:223-318 */
static inline v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
/* Mul<Vector3d> for Vector3d is the dot product: mod.rs:319-349 */
static inline double vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
/* Mul<f64> for Vector3d / Mul<Vector3d> for f64: mod.rs:351-397 (rhs.x * s) */
static inline v3 vscale(v3 a, double s) { return V(a.x * s, a.y * s, a.z * s); }
/* Div<f64>: mod.rs:399-421 */
static inline v3 vdivs(v3 a, double s) { return V(a.x / s, a.y / s, a.z / s); }
static inline v3 vneg(v3 a) { return V(-a.x, -a.y, -a.z); }
/* product / divide: mod.rs:135-150 */
static inline v3 vprod(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vdivv(v3 a, v3 b) { return V(a.x / b.x, a.y / b.y, a.z / b.z); }
/* cross: mod.rs:99-105 */
static inline v3 vcross(v3 a, v3 b) {
    return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* length / normalize: mod.rs:107-120 */
static inline double vlen(v3 a) { return sqrt(vdot(a, a)); }
static inline v3 vnorm(v3 a) { return vdivs(a, vlen(a)); }
/* f64::min / f64::max ignore a NaN operand, as C fmin/fmax do: mod.rs:168-198 */
static inline v3 vmin(v3 a, v3 b) { return V(fmin(a.x, b.x), fmin(a.y, b.y), fmin(a.z, b.z)); }
static inline v3 vmax(v3 a, v3 b) { return V(fmax(a.x, b.x), fmax(a.y, b.y), fmax(a.z, b.z)); }
static inline double vmaxc(v3 a) { return fmax(fmax(a.x, a.y), a.z); }
static inline double vminc(v3 a) { return fmin(fmin(a.x, a.y), a.z); }
/* approx_equal: mod.rs:14-17 */
static inline int approx_equal(double a, double b) { return fabs(a - b) < 1e-15; }
/* is_zero: mod.rs:156-158 */
static inline int vis_zero(v3 a) {
    return approx_equal(a.x, 0.0) && approx_equal(a.y, 0.0) && approx_equal(a.z, 0.0);
}
/* reflect: mod.rs:122-125 — b = (self·n) * n ; self - 2.0 * b */
static inline v3 vreflect(v3 d, v3 n) {
    v3 b = vscale(n, vdot(d, n));
    return vsub(d, vscale(b, 2.0));
}
/* refract: mod.rs:127-133 */
static inline v3 vrefract(v3 d, v3 n, double ratio) {
    double cos_theta = vdot(vneg(d), n);
    v3 perp = vscale(vadd(d, vscale(n, cos_theta)), ratio);
    double par_s = -(sqrt(fabs(1.0 - vdot(perp, perp))));
    v3 par = vscale(n, par_s);
    return vadd(perp, par);
}

/* ======================================================================= */
/* Transform (src/algebra/transform.rs)                                    */
/* ======================================================================= */
typedef struct {
    double m[4][4];
} mat4;

/* Mul<Transform> for Transform: transform.rs:553-570 */
static mat4 mmul(const mat4 *a, const mat4 *b) {
    mat4 r;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            r.m[i][j] = a->m[i][0] * b->m[0][j] + a->m[i][1] * b->m[1][j] + a->m[i][2] * b->m[2][j] +
                        a->m[i][3] * b->m[3][j];
    return r;
}
static mat4 mident(void) {
    mat4 r;
    memset(&r, 0, sizeof r);
    r.m[0][0] = r.m[1][1] = r.m[2][2] = r.m[3][3] = 1.0;
    return r;
}
/* f64::to_radians: self * (PI / 180.0) */
double or_to_radians(double deg) { return deg * (M_PI / 180.0); }
/* translate / scale: transform.rs:316-332 */
static mat4 mtranslate(v3 v) {
    mat4 r = mident();
    r.m[0][3] = v.x;
    r.m[1][3] = v.y;
    r.m[2][3] = v.z;
    return r;
}
static mat4 mscale(v3 v) {
    mat4 r = mident();
    r.m[0][0] = v.x;
    r.m[1][1] = v.y;
    r.m[2][2] = v.z;
    return r;
}
/* rotate_roll / pitch / yaw: transform.rs:364-392 */
static mat4 mroll(double deg) {
    double r = or_to_radians(deg);
    mat4 m = mident();
    m.m[1][1] = cos(r);
    m.m[1][2] = -sin(r);
    m.m[2][1] = sin(r);
    m.m[2][2] = cos(r);
    return m;
}
static mat4 mpitch(double deg) {
    double r = or_to_radians(deg);
    mat4 m = mident();
    m.m[0][0] = cos(r);
    m.m[0][2] = sin(r);
    m.m[2][0] = -sin(r);
    m.m[2][2] = cos(r);
    return m;
}
static mat4 myaw(double deg) {
    double r = or_to_radians(deg);
    mat4 m = mident();
    m.m[0][0] = cos(r);
    m.m[0][1] = -sin(r);
    m.m[1][0] = sin(r);
    m.m[1][1] = cos(r);
    return m;
}
/* rotate: transform.rs:334-358 = roll(x) * pitch(y) * yaw(z) (left to right) */
static mat4 mrotate(v3 v) {
    mat4 a = mroll(v.x), b = mpitch(v.y), c = myaw(v.z);
    mat4 ab = mmul(&a, &b);
    return mmul(&ab, &c);
}
/* rotate_inverse: transform.rs:360-362 = yaw(z) * pitch(y) * roll(x) */
static mat4 mrotate_inverse(v3 v) {
    mat4 a = myaw(v.z), b = mpitch(v.y), c = mroll(v.x);
    mat4 ab = mmul(&a, &b);
    return mmul(&ab, &c);
}
/* InversableTransform::new: transform.rs:16-23 */
static void transform_new(v3 t, v3 r, v3 s, mat4 *direct, mat4 *inverse) {
    mat4 T = mtranslate(t), R = mrotate(r), S = mscale(s);
    mat4 TR = mmul(&T, &R);
    *direct = mmul(&TR, &S);
    mat4 Si = mscale(V(1.0 / s.x, 1.0 / s.y, 1.0 / s.z));
    mat4 Ri = mrotate_inverse(V(-r.x, -r.y, -r.z));
    mat4 Ti = mtranslate(V(-t.x, -t.y, -t.z));
    mat4 SR = mmul(&Si, &Ri);
    *inverse = mmul(&SR, &Ti);
}
/* transform_point / vector / normal: transform.rs:394-425 */
static inline v3 mpoint(const mat4 *M, v3 p) {
    const double(*m)[4] = M->m;
    return V(p.x * m[0][0] + p.y * m[0][1] + p.z * m[0][2] + m[0][3],
             p.x * m[1][0] + p.y * m[1][1] + p.z * m[1][2] + m[1][3],
             p.x * m[2][0] + p.y * m[2][1] + p.z * m[2][2] + m[2][3]);
}
static inline v3 mvector(const mat4 *M, v3 v) {
    const double(*m)[4] = M->m;
    return V(v.x * m[0][0] + v.y * m[0][1] + v.z * m[0][2], v.x * m[1][0] + v.y * m[1][1] + v.z * m[1][2],
             v.x * m[2][0] + v.y * m[2][1] + v.z * m[2][2]);
}
static inline v3 mnormal(const mat4 *M, v3 n) {
    const double(*m)[4] = M->m;
    return V(n.x * m[0][0] + n.y * m[1][0] + n.z * m[2][0], n.x * m[0][1] + n.y * m[1][1] + n.z * m[2][1],
             n.x * m[0][2] + n.y * m[1][2] + n.z * m[2][2]);
}

void or_transform_new(const double t[3], const double r[3], const double s[3], double direct[16],
                      double inverse[16]) {
    mat4 d, i;
    transform_new(vload(t), vload(r), vload(s), &d, &i);
    memcpy(direct, d.m, sizeof d.m);
    memcpy(inverse, i.m, sizeof i.m);
}
void or_rotate(const double r[3], double out[16]) {
    mat4 m = mrotate(vload(r));
    memcpy(out, m.m, sizeof m.m);
}
void or_mat_mul(const double a[16], const double b[16], double out[16]) {
    mat4 A, B;
    memcpy(A.m, a, sizeof A.m);
    memcpy(B.m, b, sizeof B.m);
    mat4 C = mmul(&A, &B);
    memcpy(out, C.m, sizeof C.m);
}
/* AABB::transform: src/world/shapes/mod.rs:93-108 (8 corners, i/j/k order) */
void or_aabb_transform(const double mn[3], const double mx[3], const double m[16], double out_mn[3],
                       double out_mx[3]) {
    mat4 M;
    memcpy(M.m, m, sizeof M.m);
    v3 b[2] = {vload(mn), vload(mx)};
    v3 lo = V(INFINITY, INFINITY, INFINITY), hi = V(-INFINITY, -INFINITY, -INFINITY);
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++)
            for (int k = 0; k < 2; k++) {
                v3 p = mpoint(&M, V(b[i].x, b[j].y, b[k].z));
                lo = vmin(lo, p);
                hi = vmax(hi, p);
            }
    vstore(out_mn, lo);
    vstore(out_mx, hi);
}

/* ======================================================================= */
/* RNG.  rand 0.8 (Cargo.toml:19) draws from thread_rng (unseedable); the  */
/* oracle keeps rand's f64 conversions and replaces the u64 source by a    */
/* counter-keyed SplitMix64 stream (the spec the HIP kernel implements).   */
/* ======================================================================= */
#define GAMMA 0x9E3779B97F4A7C15ull

uint64_t or_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
uint64_t or_sample_key(uint64_t seed, uint64_t pixel, uint64_t sample) {
    uint64_t k = or_mix64(seed ^ 0x6A09E667F3BCC909ull);
    k = or_mix64(k + (pixel + 1) * GAMMA);
    k = or_mix64(k + (sample + 1) * 0xD1B54A32D192ED03ull);
    return k;
}
uint64_t or_rng_next(uint64_t *state) {
    *state += GAMMA;
    return or_mix64(*state);
}
/* Standard f64: (u64 >> 11) * 2^-53 (rand 0.8 distributions/float.rs) */
double or_gen_f64(uint64_t *state) {
    return (1.0 / 9007199254740992.0) * (double)(or_rng_next(state) >> 11);
}
/* UniformFloat::new_inclusive (rand 0.8 distributions/uniform.rs) */
double or_uniform_incl_scale(double lo, double hi) {
    const double max_rand = 1.0 - 2.220446049250313e-16; /* (u64::MAX>>12) in [1,2) minus 1 */
    double scale = (hi - lo) / max_rand;
    while (scale * max_rand + lo > hi) {
        uint64_t b;
        memcpy(&b, &scale, 8);
        b -= 1;
        memcpy(&scale, &b, 8);
    }
    return scale;
}
/* UniformFloat::sample: value1_2 from 52 bits, minus 1, * scale + low */
static inline double uniform_sample(uint64_t *state, double lo, double scale) {
    uint64_t bits = (or_rng_next(state) >> 12) | (1023ull << 52);
    double v12;
    memcpy(&v12, &bits, 8);
    double v01 = v12 - 1.0;
    return v01 * scale + lo;
}
double or_gen_range_incl(uint64_t *state, double lo, double hi) {
    return uniform_sample(state, lo, or_uniform_incl_scale(lo, hi));
}

/* ======================================================================= */
/* Scene                                                                   */
/* ======================================================================= */
typedef struct {
    int type, material, inverse_normal, depth, func;
    mat4 direct, inverse;
    double x0, y0, x1, y1, step;
    double fa, fb, fc, fd, fr;
    double radius, tube_radius;
} shape_t;

typedef struct {
    int type;
    int tex; /* -1: SolidColor (albedo / emit) */
    v3 albedo;
    double fuzz, ior;
    v3 emit;
} mat_t;

typedef struct { /* Perlin (src/algebra/noise.rs:6-16) */
    int perm_x[256], perm_y[256], perm_z[256];
    v3 ranvec[256];
} perlin_t;

typedef struct {
    uint32_t w, h;
    uint8_t *rgba;
} image_t;

typedef struct {
    v3 mn, mx;   /* AABB (src/world/shapes/mod.rs:17-21) */
    int left;    /* node index, or -(shape+1) for a leaf shape */
    int right;   /* node index, -(shape+1), or INT32_MIN for None */
} bvh_node;

struct or_scene {
    shape_t *shapes;
    int nshapes, cap;
    mat_t *mats;
    int nmats, mcap;
    bvh_node *nodes;
    int nnodes, root;
    int use_bvh;
    or_texture_in *tex;
    int ntex;
    perlin_t *perlin; /* per texture node (NoiseTexture nodes only) */
    image_t *images;
    int nimages;
};

static int push_mat(or_scene *s, mat_t m) {
    if (s->nmats == s->mcap) {
        s->mcap = s->mcap ? 2 * s->mcap : 16;
        s->mats = realloc(s->mats, sizeof(mat_t) * s->mcap);
    }
    s->mats[s->nmats] = m;
    return s->nmats++;
}
static void push_shape(or_scene *s, shape_t sh) {
    if (s->nshapes == s->cap) {
        s->cap = s->cap ? 2 * s->cap : 16;
        s->shapes = realloc(s->shapes, sizeof(shape_t) * s->cap);
    }
    s->shapes[s->nshapes++] = sh;
}

static double gen_f64_scene(uint64_t *st) { return or_gen_f64(st); }

/* add_random_spheres: src/world/json_models.rs:50-133 */
static void add_random_spheres(or_scene *s, uint64_t seed) {
    uint64_t st = seed;
    double s01 = or_uniform_incl_scale(0.0, 1.0);
    for (int a = -11; a < 11; a++) {
        for (int b = -11; b < 11; b++) {
            double cx = (double)a + 0.9 * gen_f64_scene(&st);
            double cz = (double)b + 0.9 * gen_f64_scene(&st);
            v3 center = V(cx, 0.2, cz);
            double rad = 0.2;
            if (vlen(vsub(center, V(4.0, 0.2, 0.0))) > 0.9) {
                double choice = gen_f64_scene(&st);
                mat_t m;
                memset(&m, 0, sizeof m);
                m.tex = -1;
                if (choice < 0.8) {
                    double rx = uniform_sample(&st, 0.0, s01);
                    double ry = uniform_sample(&st, 0.0, s01);
                    double rz = uniform_sample(&st, 0.0, s01);
                    m.type = OR_LAMBERTIAN;
                    m.albedo = vprod(V(rx, ry, rz), V(rx, ry, rz));
                } else if (choice < 0.95) {
                    double rx = uniform_sample(&st, 0.0, s01);
                    double ry = uniform_sample(&st, 0.0, s01);
                    double rz = uniform_sample(&st, 0.0, s01);
                    m.type = OR_METAL;
                    m.albedo = V(0.5 * (1.0 - rx), 0.5 * (1.0 - ry), 0.5 * (1.0 - rz));
                    m.fuzz = 0.5 * gen_f64_scene(&st);
                } else {
                    m.type = OR_DIELECTRIC;
                    m.ior = 1.5;
                }
                shape_t sh;
                memset(&sh, 0, sizeof sh);
                sh.type = OR_SPHERE;
                sh.material = push_mat(s, m);
                transform_new(center, V(0.0, 0.0, 0.0), V(rad, rad, rad), &sh.direct, &sh.inverse);
                push_shape(s, sh);
            }
        }
    }
}

or_scene *or_scene_new(const or_shape_in *shapes, int n, const or_material_in *mats, int nm,
                       int random_spheres, uint64_t scene_seed) {
    or_scene *s = calloc(1, sizeof *s);
    for (int i = 0; i < nm; i++) {
        mat_t m;
        m.type = mats[i].type;
        m.tex = mats[i].tex;
        m.albedo = vload(mats[i].albedo);
        m.fuzz = mats[i].fuzz;
        m.ior = mats[i].ior;
        m.emit = vload(mats[i].emit);
        push_mat(s, m);
    }
    for (int i = 0; i < n; i++) {
        shape_t sh;
        memset(&sh, 0, sizeof sh);
        sh.type = shapes[i].type;
        sh.material = shapes[i].material;
        sh.inverse_normal = shapes[i].inverse_normal;
        sh.depth = shapes[i].depth;
        sh.func = shapes[i].func;
        sh.x0 = shapes[i].x0;
        sh.y0 = shapes[i].y0;
        sh.x1 = shapes[i].x1;
        sh.y1 = shapes[i].y1;
        sh.step = shapes[i].step;
        sh.fa = shapes[i].fa;
        sh.fb = shapes[i].fb;
        sh.fc = shapes[i].fc;
        sh.fd = shapes[i].fd;
        sh.fr = shapes[i].fr;
        sh.radius = shapes[i].radius;
        sh.tube_radius = shapes[i].tube_radius;
        transform_new(vload(shapes[i].translate), vload(shapes[i].rotate), vload(shapes[i].scale),
                      &sh.direct, &sh.inverse);
        push_shape(s, sh);
    }
    if (random_spheres) add_random_spheres(s, scene_seed);
    return s;
}
void or_scene_free(or_scene *s) {
    if (!s) return;
    for (int i = 0; i < s->nimages; i++) free(s->images[i].rgba);
    free(s->images);
    free(s->tex);
    free(s->perlin);
    free(s->nodes);
    free(s->shapes);
    free(s->mats);
    free(s);
}
int or_scene_num_shapes(const or_scene *s) { return s->nshapes; }
int or_scene_num_materials(const or_scene *s) { return s->nmats; }
void or_scene_get_shape(const or_scene *s, int i, or_shape_out *o) {
    const shape_t *sh = &s->shapes[i];
    memset(o, 0, sizeof *o);
    o->type = sh->type;
    o->material = sh->material;
    o->inverse_normal = sh->inverse_normal;
    o->depth = sh->depth;
    o->func = sh->func;
    memcpy(o->direct, sh->direct.m, sizeof o->direct);
    memcpy(o->inverse, sh->inverse.m, sizeof o->inverse);
    o->x0 = sh->x0;
    o->y0 = sh->y0;
    o->x1 = sh->x1;
    o->y1 = sh->y1;
    o->step = sh->step;
    o->fa = sh->fa;
    o->fb = sh->fb;
    o->fc = sh->fc;
    o->fd = sh->fd;
    o->fr = sh->fr;
    o->radius = sh->radius;
    o->tube_radius = sh->tube_radius;
}
void or_scene_get_material(const or_scene *s, int i, or_material_in *o) {
    const mat_t *m = &s->mats[i];
    memset(o, 0, sizeof *o);
    o->type = m->type;
    o->tex = m->tex;
    vstore(o->albedo, m->albedo);
    o->fuzz = m->fuzz;
    o->ior = m->ior;
    vstore(o->emit, m->emit);
}

/* ======================================================================= */
/* Camera (src/camera/mod.rs:48-88) and MultisamplerRayCaster             */
/* (src/camera/ray_caster.rs:30-118)                                       */
/* ======================================================================= */
void or_camera_new(const double pos[3], const double dir[3], const double up[3], double focal_length,
                   double fov_radians, or_camera *out) {
    v3 d = vload(dir);
    v3 right = vnorm(vcross(d, vload(up)));
    vstore(out->position, vload(pos));
    vstore(out->direction, vnorm(d));
    vstore(out->up, vnorm(vcross(right, d)));
    vstore(out->right, right);
    out->fov = fov_radians;
    out->focal_length = focal_length;
}
void or_caster_new(const or_camera *c, uint32_t width, uint32_t height, or_caster *k) {
    v3 center = vadd(vload(c->position), vscale(vload(c->direction), c->focal_length));
    double aspect = (double)width / (double)height;
    double vw = tan(c->fov / 2.0) * c->focal_length * 2.0;
    double vh = vw / aspect;
    v3 lt = vadd(vsub(center, vscale(vload(c->right), vw / 2.0)), vscale(vload(c->up), vh / 2.0));
    vstore(k->left_top, lt);
    vstore(k->position, vload(c->position));
    vstore(k->right, vload(c->right));
    vstore(k->up, vload(c->up));
    k->pixel_resolution = vw / (double)width;
    k->width = width;
    k->height = height;
}
/* get_ray: ray_caster.rs:77-81 / next: :110-113 */
void or_caster_ray(const or_caster *k, double x, double y, double origin[3], double dir[3]) {
    v3 d = vsub(vadd(vload(k->left_top), vscale(vload(k->right), k->pixel_resolution * x)),
                vscale(vload(k->up), k->pixel_resolution * y));
    vstore(origin, vload(k->position));
    vstore(dir, vnorm(vsub(d, vload(k->position)))); /* Ray::new normalises: ray.rs:12-17 */
}

/* ======================================================================= */
/* Shapes — object-space intersections return the distance t (the object  */
/* ray direction is NOT renormalised: transform.rs:32-37, so object t is   */
/* the world distance).                                                    */
/* ======================================================================= */

/* Sphere::ray_intersect: src/world/shapes/mod.rs:330-374 */
static int sphere_t(v3 o, v3 d, double min_t, double max_t, double *out) {
    double a = vdot(d, d);
    double half_b = vdot(d, o);
    double c = vdot(o, o) - 1.0;
    double disc = half_b * half_b - a * c;
    double x;
    if (disc < 0.0) return 0;
    if (disc == 0.0) {
        x = -half_b * a; /* reference quirk: no division, no range check */
    } else {
        x = (-half_b - sqrt(disc)) / a;
        if (x < min_t || x > max_t) {
            x = (-half_b + sqrt(disc)) / a;
            if (x < min_t || x > max_t) return 0;
        }
    }
    *out = x;
    return 1;
}
/* Rectangle::ray_intersect: src/world/shapes/mod.rs:181-204 */
static int rect_t(const shape_t *s, v3 o, v3 d, double min_t, double max_t, double *out) {
    double t = -o.z / d.z;
    if (t < min_t || t > max_t) return 0;
    v3 p = vadd(o, vscale(d, t));
    if (p.x < s->x0 || p.x > s->x1 || p.y < s->y0 || p.y > s->y1) return 0;
    *out = t;
    return 1;
}
/* Cube::ray_intersect: src/world/shapes/mod.rs:250-285 */
static int cube_t(v3 o, v3 d, double min_t, double max_t, double *out) {
    v3 tl = vdivv(vsub(V(-1.0, -1.0, -1.0), o), d);
    v3 tu = vdivv(vsub(V(1.0, 1.0, 1.0), o), d);
    v3 tmins = vmin(tl, tu), tmaxs = vmax(tl, tu);
    double tbmin = fmax(vmaxc(tmins), min_t);
    double tbmax = fmin(vminc(tmaxs), max_t);
    if (tbmin > tbmax || tbmin > max_t) return 0;
    *out = tbmin;
    return 1;
}

/* Heart (src/world/shapes/ray_marching.rs:121-188) */
static const double HEART_R = 1.45;
static inline double heart_f(v3 p) { /* shape_func :147-155 */
    double x2 = p.x * p.x;
    double y2 = p.y * p.y;
    double z2 = p.z * p.z;
    double z3 = z2 * p.z;
    double a = x2 + (9.0 / 4.0) * y2 + z2 - 1.0;
    return a * a * a - x2 * z3 - (9.0 / 80.0) * y2 * z3;
}
static inline v3 heart_gradient(v3 p) { /* gradient :157-168 (27/40 coefficient kept) */
    double a = p.x * p.x + (9.0 / 4.0) * p.y * p.y + p.z * p.z - 1.0;
    a = 3.0 * a * a;
    double z2 = p.z * p.z;
    double z3 = z2 * p.z;
    return V(2.0 * p.x * (a - z3), (9.0 / 2.0) * p.y * (a - 0.05 * z3),
             2.0 * p.z * (a - p.z * (1.5 * p.x * p.x + (27.0 / 40.0) * p.y * p.y)));
}
/* solve_quadratic_equation: src/algebra/equation.rs:5-15 */
static int solve_quadratic(double a, double half_b, double c, double *x1, double *x2) {
    double d = half_b * half_b - a * c;
    double ds = sqrt(d);
    if (d < 0.0) return 0;
    if (d == 0.0) {
        *x1 = -half_b;
        *x2 = -half_b;
    } else {
        *x1 = (-half_b - ds) / a;
        *x2 = (-half_b + ds) / a;
    }
    return 1;
}
/* Heart::intersect_bound :135-145 */
static int heart_bound(v3 o, v3 d, double *start, double *end) {
    v3 R = V(HEART_R, HEART_R / 2.05, HEART_R);
    v3 oo = vdivv(o, R), dd = vdivv(d, R);
    double x1, x2;
    if (!solve_quadratic(vdot(dd, dd), vdot(dd, oo), vdot(oo, oo) - 1.0, &x1, &x2)) return 0;
    if (x1 < 0.0 && x2 < 0.0) return 0;
    *start = fmax(x1, 0.0);
    *end = fmax(x2, 0.0);
    return 1;
}
/* Sine::shape_func ray_marching.rs:202-210 */
static double sine_f(const shape_t *s, v3 p) {
    return s->fa * s->fa * (p.x - p.y - p.z) * (p.x + p.y - p.z) * (p.x - p.y + p.z) * (p.x + p.y + p.z) +
           4.0 * p.x * p.x * p.y * p.y * p.z * p.z;
}
/* Sine::gradient :227-238 */
static v3 sine_gradient(const shape_t *s, v3 p) {
    double x2 = p.x * p.x, y2 = p.y * p.y, z2 = p.z * p.z;
    double a2 = s->fa * s->fa;
    return V(4.0 * p.x * (a2 * (x2 - y2 - z2) + 2.0 * y2 * z2),
             8.0 * x2 * p.y * z2 - 4.0 * a2 * p.y * (x2 - y2 + z2),
             8.0 * x2 * y2 * p.z - 4.0 * a2 * p.z * (x2 + y2 - z2));
}
/* Star::shape_func :258-264, gradient :279-289 */
static double star_f(const shape_t *s, v3 p) {
    double x2 = p.x * p.x, y2 = p.y * p.y, z2 = p.z * p.z;
    double c = x2 + y2 + z2 - 1.0;
    return s->fa * (x2 * y2 + x2 * z2 + y2 * z2) + (c * c * c);
}
static v3 star_gradient(const shape_t *s, v3 p) {
    double x2 = p.x * p.x, y2 = p.y * p.y, z2 = p.z * p.z;
    double c = x2 + y2 + z2 - 1.0;
    return V(2.0 * s->fa * p.x * (y2 + z2) + 6.0 * p.x * c * c, 2.0 * s->fa * p.y * (x2 + z2) + 6.0 * p.y * c * c,
             2.0 * s->fa * p.z * (x2 + y2) + 6.0 * p.z * c * c);
}
/* DupinCyclide::shape_func :339-344, gradient :359-367 */
static double dupin_f(const shape_t *s, v3 p) {
    double b2 = s->fb * s->fb;
    double e = p.x * p.x + p.y * p.y + p.z * p.z + b2 - s->fd * s->fd;
    double f = s->fa * p.x - s->fc * s->fd;
    return e * e - 4.0 * (f * f + b2 * p.y * p.y);
}
static v3 dupin_gradient(const shape_t *s, v3 p) {
    double b2 = s->fb * s->fb;
    double e = 4.0 * (p.x * p.x + p.y * p.y + p.z * p.z + b2 - s->fd * s->fd);
    return V(e * p.x - 8.0 * s->fa * (s->fa * p.x - s->fc * s->fd), e * p.y - 8.0 * b2 * p.y, e * p.z);
}
/* HuntsSurface::shape_func :399-406, gradient :421-433 */
static double hunts_f(v3 p) {
    double x2 = p.x * p.x, y2 = p.y * p.y, z2 = p.z * p.z;
    double a = x2 + y2 + z2 - 13.0;
    double b = 3.0 * x2 + y2 - 4.0 * z2 - 12.0;
    return 4.0 * a * a * a + 27.0 * b * b;
}
static v3 hunts_gradient(v3 p) {
    double x2 = p.x * p.x, y2 = p.y * p.y, z2 = p.z * p.z;
    double a = x2 + y2 + z2 - 13.0;
    double b = 3.0 * x2 + y2 - 4.0 * (z2 + 3.0);
    return V(24.0 * p.x * a * a + 324.0 * p.x * b, 12.0 * p.y * (2.0 * a * a + 9.0 * b),
             24.0 * p.z * (a * a - 18.0 * b));
}
/* Cushion::shape_func :456-472, gradient :487-496 */
static double cushion_f(v3 p) {
    double x2 = p.x * p.x, y2 = p.y * p.y, z2 = p.z * p.z;
    double a = x2 - p.z;
    return z2 * x2 - z2 * z2 - 2.0 * p.z * x2 + 2.0 * p.z * z2 + x2 - z2 - a * a - y2 * y2 - 2.0 * x2 * y2 - y2 * z2 +
           2.0 * y2 * p.z + y2;
}
static v3 cushion_gradient(v3 p) {
    double x2 = p.x * p.x, y2 = p.y * p.y, z2 = p.z * p.z;
    return V(2.0 * p.x * (-2.0 * x2 - 2.0 * y2 + z2 + 1.0),
             -2.0 * p.y * (2.0 * x2 + 2.0 * y2 + z2 - 2.0 * p.z - 1.0),
             2.0 * p.z * (x2 - 2.0 * z2 + 3.0 * p.z - 2.0) - 2.0 * p.y * (p.z - 1.0));
}
/* ShapeFunction::shape_func dispatch */
static double func_f(const shape_t *s, v3 p) {
    switch (s->func) {
    case OR_FUNC_SINE: return sine_f(s, p);
    case OR_FUNC_STAR: return star_f(s, p);
    case OR_FUNC_DUPIN: return dupin_f(s, p);
    case OR_FUNC_HUNTS: return hunts_f(p);
    case OR_FUNC_CUSHION: return cushion_f(p);
    default: return heart_f(p);
    }
}
static v3 func_gradient(const shape_t *s, v3 p) {
    switch (s->func) {
    case OR_FUNC_SINE: return sine_gradient(s, p);
    case OR_FUNC_STAR: return star_gradient(s, p);
    case OR_FUNC_DUPIN: return dupin_gradient(s, p);
    case OR_FUNC_HUNTS: return hunts_gradient(p);
    case OR_FUNC_CUSHION: return cushion_gradient(p);
    default: return heart_gradient(p);
    }
}
/* intersect_bound of the non-Heart functions (e.g. Sine :212-225): the
 * sphere_radius ball */
static int sphere_bound(double radius, v3 o, v3 d, double *start, double *end) {
    double x1, x2;
    if (!solve_quadratic(vdot(d, d), vdot(d, o), vdot(o, o) - radius * radius, &x1, &x2)) return 0;
    if (x1 < 0.0 && x2 < 0.0) return 0;
    *start = fmax(x1, 0.0);
    *end = fmax(x2, 0.0);
    return 1;
}

/* RayMarchingShape::ray_intersect: ray_marching.rs:20-74 */
static int march_t(const shape_t *s, v3 o, v3 d, double min_t, double max_t, double *out, or_stats *st) {
    double start, end;
    if (st) st->march_bounds++;
    if (s->func == OR_FUNC_HEART ? !heart_bound(o, d, &start, &end) : !sphere_bound(s->fr, o, d, &start, &end))
        return 0;
    double step = s->step;
    double t = start;
    v3 p = vadd(o, vscale(d, t));
    double r = func_f(s, p);
    for (int pass = 0; pass < s->depth; pass++) {
        for (;;) {
            if (t > end || t < start) return 0;
            t += step;
            p = vadd(p, vscale(d, step));
            double next = func_f(s, p);
            if (st) st->march_steps++;
            if (approx_equal(next, 0.0)) goto done;
            if ((r < 0.0 && next > 0.0) || (r > 0.0 && next < 0.0)) {
                step *= -0.01;
                r = next;
                break;
            }
            r = next;
        }
    }
done:
    if (t < min_t || t > max_t) return 0;
    *out = t;
    return 1;
}

/* ---- Torus ------------------------------------------------------------- */
/* num::Complex<f64> (num 0.4, unpinned release) as num-complex publishes it:
 * Mul / Div by the textbook formulas (Div via norm_sqr), real operands
 * componentwise, sqrt / cbrt special-cased on the axes (sign of a zero
 * imaginary part picks the root), else from_polar(hypot, atan2). */
typedef struct {
    double re, im;
} cplx;
static cplx C2(double re, double im) { cplx z = {re, im}; return z; }
static cplx c_add(cplx a, cplx b) { return C2(a.re + b.re, a.im + b.im); }
static cplx c_sub(cplx a, cplx b) { return C2(a.re - b.re, a.im - b.im); }
static cplx c_neg(cplx a) { return C2(-a.re, -a.im); }
static cplx c_mul(cplx a, cplx b) { return C2(a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re); }
static cplx c_div(cplx a, cplx b) {
    double n = b.re * b.re + b.im * b.im;
    return C2((a.re * b.re + a.im * b.im) / n, (a.im * b.re - a.re * b.im) / n);
}
static cplx c_scale(double k, cplx a) { return C2(k * a.re, k * a.im); }  /* f64 * Complex */
static cplx c_divr(cplx a, double k) { return C2(a.re / k, a.im / k); }   /* Complex / f64 */
static int sign_positive(double x) { return !signbit(x); }
static cplx c_polar(double r, double th) { return C2(r * cos(th), r * sin(th)); }
static cplx c_sqrt(cplx z) {
    if (z.im == 0.0) {
        if (sign_positive(z.re)) return C2(sqrt(z.re), z.im);
        double im = sqrt(-z.re);
        return sign_positive(z.im) ? C2(0.0, im) : C2(0.0, -im);
    }
    if (z.re == 0.0) {
        double x = sqrt(fabs(z.im) / 2.0);
        return sign_positive(z.im) ? C2(x, x) : C2(x, -x);
    }
    return c_polar(sqrt(hypot(z.re, z.im)), atan2(z.im, z.re) / 2.0);
}
static cplx c_cbrt(cplx z) {
    if (z.im == 0.0) {
        if (sign_positive(z.re)) return C2(cbrt(z.re), z.im);
        double re = cbrt(-z.re) / 2.0, im = sqrt(3.0) * re;
        return sign_positive(z.im) ? C2(re, im) : C2(re, -im);
    }
    if (z.re == 0.0) {
        double im = cbrt(fabs(z.im)) / 2.0, re = sqrt(3.0) * im;
        return sign_positive(z.im) ? C2(re, im) : C2(re, -im);
    }
    return c_polar(cbrt(hypot(z.re, z.im)), atan2(z.im, z.re) / 3.0);
}
/* solve_quantic_equation: equation.rs:17-67 */
static void quartic(cplx a, cplx b, cplx c, cplx d, cplx e, cplx out[4]) {
    b = c_div(b, a);
    c = c_div(c, a);
    d = c_div(d, a);
    e = c_div(e, a);
    cplx b2 = c_mul(b, b);
    cplx alpha = c_sub(c, c_scale(3.0 / 8.0, b2));
    cplx beta = c_add(c_sub(c_divr(c_mul(b2, b), 8.0), c_divr(c_mul(b, c), 2.0)), d);
    cplx gamma = c_add(c_sub(c_add(c_mul(c_scale(-3.0 / 256.0, b2), b2), c_divr(c_mul(b2, c), 16.0)),
                             c_divr(c_mul(b, d), 4.0)), e);
    cplx alpha2 = c_mul(alpha, alpha);
    cplx t = c_divr(c_neg(b), 4.0);
    if (approx_equal(beta.re, 0.0) && approx_equal(beta.im, 0.0)) {
        cplx r = c_sqrt(c_sub(alpha2, c_scale(4.0, gamma)));
        cplx r1 = c_sqrt(c_divr(c_add(c_neg(alpha), r), 2.0));
        cplx r2 = c_sqrt(c_divr(c_sub(c_neg(alpha), r), 2.0));
        out[0] = c_add(t, r1);
        out[1] = c_sub(t, r1);
        out[2] = c_add(t, r2);
        out[3] = c_sub(t, r2);
        return;
    }
    cplx p = c_neg(c_add(c_divr(alpha2, 12.0), gamma));
    cplx q = c_sub(c_add(c_divr(c_mul(c_neg(alpha2), alpha), 108.0), c_divr(c_mul(alpha, gamma), 3.0)),
                   c_divr(c_mul(beta, beta), 8.0));
    cplx r = c_add(c_divr(c_neg(q), 2.0), c_sqrt(c_add(c_divr(c_mul(q, q), 4.0), c_divr(c_mul(c_mul(p, p), p), 27.0))));
    cplx u = c_cbrt(r);
    cplx y = c_add(c_scale(-5.0 / 6.0, alpha), u);
    if (approx_equal(u.re, 0.0) && approx_equal(u.im, 0.0)) y = c_sub(y, c_cbrt(q));
    else y = c_sub(y, c_div(p, c_scale(3.0, u)));
    cplx w = c_sqrt(c_add(alpha, c_scale(2.0, y)));
    cplx r1 = c_sqrt(c_neg(c_add(c_add(c_scale(3.0, alpha), c_scale(2.0, y)), c_div(c_scale(2.0, beta), w))));
    cplx r2 = c_sqrt(c_neg(c_sub(c_add(c_scale(3.0, alpha), c_scale(2.0, y)), c_div(c_scale(2.0, beta), w))));
    out[0] = c_add(t, c_divr(c_sub(w, r1), 2.0));
    out[1] = c_add(t, c_divr(c_add(w, r1), 2.0));
    out[2] = c_add(t, c_divr(c_sub(c_neg(w), r2), 2.0));
    out[3] = c_add(t, c_divr(c_add(c_neg(w), r2), 2.0));
}
void or_solve_quartic(double a, double b, double c, double d, double e, double re[4], double im[4]) {
    cplx out[4];
    quartic(C2(a, 0.0), C2(b, 0.0), C2(c, 0.0), C2(d, 0.0), C2(e, 0.0), out);
    for (int i = 0; i < 4; i++) {
        re[i] = out[i].re;
        im[i] = out[i].im;
    }
}
/* Torus::ray_intersect distance: mod.rs:430-462 */
static int torus_t(const shape_t *s, v3 o, v3 d, double min_t, double max_t, double *out) {
    double R = s->radius, r = s->tube_radius;
    double t = 4.0 * R * R;
    double g = t * (d.x * d.x + d.y * d.y);
    double h = 2.0 * t * (o.x * d.x + o.y * d.y);
    double i = t * (o.x * o.x + o.y * o.y);
    double j = vdot(d, d);
    double k = 2.0 * vdot(o, d);
    double l = vdot(o, o) + R * R - r * r;
    cplx roots[4];
    quartic(C2(j * j, 0.0), C2(2.0 * j * k, 0.0), C2(2.0 * j * l + k * k - g, 0.0), C2(2.0 * k * l - h, 0.0),
            C2(l * l - i, 0.0), roots);
    double m = INFINITY;
    for (int q = 0; q < 4; q++)
        if (approx_equal(roots[q].im, 0.0) && roots[q].re < m) m = roots[q].re;
    if (isinf(m) || m < min_t || m > max_t) return 0;
    *out = m;
    return 1;
}

/* Object-space test dispatch. */
static int shape_t_obj(const shape_t *s, v3 o, v3 d, double min_t, double max_t, double *t, or_stats *st) {
    if (st && s->type >= 0 && s->type < 4) st->shape_tests[s->type]++; /* (Torus tests are not counted) */
    switch (s->type) {
    case OR_SPHERE: return sphere_t(o, d, min_t, max_t, t);
    case OR_RECT: return rect_t(s, o, d, min_t, max_t, t);
    case OR_CUBE: return cube_t(o, d, min_t, max_t, t);
    case OR_MARCH: return march_t(s, o, d, min_t, max_t, t, st);
    case OR_TORUS: return torus_t(s, o, d, min_t, max_t, t);
    }
    return 0;
}

/* Object-space point + (unnormalised) normal of an accepted hit at t, as
 * each ray_intersect builds its RayHit. */
static v3 shape_obj_normal(const shape_t *s, v3 o, v3 d, double t, v3 *p_out) {
    switch (s->type) {
    case OR_SPHERE: { /* mod.rs:358-359 */
        v3 p = vadd(o, vscale(d, t));
        *p_out = p;
        return s->inverse_normal ? vneg(p) : p;
    }
    case OR_RECT: { /* mod.rs:186,195 */
        *p_out = vadd(o, vscale(d, t));
        return V(0.0, 0.0, 1.0);
    }
    case OR_CUBE: { /* mod.rs:263-282 */
        v3 p = vadd(o, vscale(d, t));
        *p_out = p;
        v3 pa = V(fabs(p.x), fabs(p.y), fabs(p.z));
        double mc = vmaxc(pa);
        if (mc == pa.x) return V(p.x, 0.0, 0.0);
        if (mc == pa.y) return V(0.0, p.y, 0.0);
        if (mc == pa.z) return V(0.0, 0.0, p.z);
        return V(NAN, NAN, NAN); /* reference panics here (NaN point) */
    }
    case OR_MARCH: { /* ray_marching.rs:59-60 */
        v3 p = vadd(o, vscale(d, t));
        *p_out = p;
        return func_gradient(s, p);
    }
    case OR_TORUS: { /* mod.rs:464-465: p - normalize((p.x, p.y, 0)) * radius */
        v3 p = vadd(o, vscale(d, t));
        *p_out = p;
        return vsub(p, vscale(vnorm(V(p.x, p.y, 0.0)), s->radius));
    }
    }
    *p_out = V(NAN, NAN, NAN);
    return V(NAN, NAN, NAN);
}

/* RayHit u, v from the object-space point, as each ray_intersect builds it:
 * Sphere mod.rs:361-373 (theta = acos(-p.y), phi = atan2(-p.z, p.x) + PI),
 * Rectangle :189-190, Cube :267-281 (by the face of the largest |p| component),
 * ray-marched ShapeFunction::uv (Heart :170, Sine :239, Star :302 -> (0, 0);
 * DupinCyclide :371, HuntsSurface :436, Cushion :506 -> (p.x, p.y)). */
static void shape_uv(const shape_t *s, v3 p, double *u, double *v) {
    switch (s->type) {
    case OR_SPHERE: {
        double theta = acos(-p.y);
        double phi = atan2(-p.z, p.x) + M_PI;
        *u = phi / (2.0 * M_PI);
        *v = theta / M_PI;
        return;
    }
    case OR_RECT:
        *u = (p.x - s->x0) / (s->x1 - s->x0);
        *v = (p.y - s->y0) / (s->y1 - s->y0);
        return;
    case OR_CUBE: {
        v3 pa = V(fabs(p.x), fabs(p.y), fabs(p.z));
        double mc = vmaxc(pa);
        if (mc == pa.x) { *u = p.y; *v = p.z; }
        else if (mc == pa.y) { *u = p.x; *v = p.z; }
        else if (mc == pa.z) { *u = p.x; *v = p.y; }
        else { *u = NAN; *v = NAN; }
        return;
    }
    case OR_TORUS: { /* mod.rs:466-467 */
        double theta = asin(p.z / s->tube_radius);
        double phi = acos(p.z / (s->radius + s->tube_radius * cos(theta))) + M_PI;
        *u = phi / (2.0 * M_PI);
        *v = theta / M_PI;
        return;
    }
    default:
        if (s->func == OR_FUNC_DUPIN || s->func == OR_FUNC_HUNTS || s->func == OR_FUNC_CUSHION) {
            *u = p.x;
            *v = p.y;
        } else {
            *u = 0.0;
            *v = 0.0;
        }
    }
}

/* Shape::ray_hit_transformed: src/world/shapes/mod.rs:112-124, with
 * RayHit::new (ray.rs:32-52, normal normalised) and set_normal (ray.rs:60-64). */
static void finish_hit(const shape_t *s, int idx, v3 wo, v3 wd, double t, or_hit *h) {
    v3 o = mpoint(&s->inverse, wo);
    v3 d = mvector(&s->inverse, wd);
    v3 p_obj;
    v3 n_obj = vnorm(shape_obj_normal(s, o, d, t, &p_obj));
    v3 n = mnormal(&s->inverse, n_obj);
    int front = vdot(n, wd) < 0.0;
    v3 nn = vnorm(front ? n : vneg(n));
    v3 p = mpoint(&s->direct, p_obj);
    shape_uv(s, p_obj, &h->u, &h->v);
    h->t = t;
    vstore(h->point, p);
    vstore(h->normal, nn);
    h->front_face = front;
    h->shape = idx;
    h->material = s->material;
}

int or_shape_hit(const or_scene *sc, int i, const double o[3], const double d[3], double min_t,
                 double max_t, or_hit *out) {
    const shape_t *s = &sc->shapes[i];
    v3 wo = vload(o), wd = vload(d);
    double t;
    if (!shape_t_obj(s, mpoint(&s->inverse, wo), mvector(&s->inverse, wd), min_t, max_t, &t, NULL)) return 0;
    finish_hit(s, i, wo, wd, t, out);
    return 1;
}

/* ---- BvhNode (src/world/shapes/mod.rs:620-729) -------------------------- */
/* get_bounding_box of each leaf kind: Rectangle :214-220, Cube :295-301,
 * Sphere :384-398, RayMarchingShape ray_marching.rs:84-91 (+ Heart::get_bounds :174-187). */
static void shape_bbox(const shape_t *s, v3 *mn, v3 *mx) {
    double lo[3], hi[3], m[16];
    memcpy(m, s->direct.m, sizeof m);
    switch (s->type) {
    case OR_RECT: lo[0] = s->x0; lo[1] = s->y0; lo[2] = -0.0001; hi[0] = s->x1; hi[1] = s->y1; hi[2] = 0.0001; break;
    case OR_MARCH:
        if (s->func == OR_FUNC_HEART) {
            lo[0] = -HEART_R; lo[1] = -(HEART_R / 2.05); lo[2] = -HEART_R;
            hi[0] = HEART_R; hi[1] = HEART_R / 2.05; hi[2] = HEART_R;
        } else { /* the other functions' get_bounds: the sphere_radius cube (e.g. Sine :244-256) */
            lo[0] = lo[1] = lo[2] = -s->fr;
            hi[0] = hi[1] = hi[2] = s->fr;
        }
        break;
    case OR_TORUS: { /* mod.rs:478-485 */
        double a = s->radius + s->tube_radius;
        lo[0] = -a; lo[1] = -a; lo[2] = -s->tube_radius;
        hi[0] = a; hi[1] = a; hi[2] = s->tube_radius;
        break;
    }
    default: lo[0] = lo[1] = lo[2] = -1.0; hi[0] = hi[1] = hi[2] = 1.0; break;
    }
    double omn[3], omx[3];
    or_aabb_transform(lo, hi, m, omn, omx);
    *mn = vload(omn);
    *mx = vload(omx);
}
/* AABB::ray_hit: mod.rs:68-79 */
static inline int aabb_hit(v3 mn, v3 mx, v3 o, v3 d, double min_t, double max_t) {
    v3 tl = vdivv(vsub(mn, o), d), tu = vdivv(vsub(mx, o), d);
    double tbmin = fmax(vmaxc(vmin(tl, tu)), min_t);
    double tbmax = fmin(vminc(vmax(tl, tu)), max_t);
    return tbmin <= tbmax;
}
typedef struct {
    int idx;
    double key;
} sort_item;
static int cmp_items(const void *a, const void *b) {
    const sort_item *x = a, *y = b;
    if (x->key < y->key) return -1;
    if (x->key > y->key) return 1;
    return x->idx - y->idx;
}
static int bvh_push(or_scene *s, bvh_node n) {
    s->nodes[s->nnodes] = n;
    return s->nnodes++;
}
static void bbox_of(const or_scene *s, int ref, v3 *mn, v3 *mx) {
    if (ref < 0) shape_bbox(&s->shapes[-ref - 1], mn, mx);
    else {
        *mn = s->nodes[ref].mn;
        *mx = s->nodes[ref].mx;
    }
}
/* BvhNode::new: random axis in {x, y} (gen_range(0..2)), sort by bbox.min
 * along it, split at n/2; n == 1 -> leaf, n == 2 -> two leaves. */
static int bvh_build(or_scene *s, int *idx, int n, uint64_t *rng) {
    int axis = (int)(or_rng_next(rng) >> 63);
    sort_item *it = malloc(sizeof(sort_item) * n);
    for (int i = 0; i < n; i++) {
        v3 mn, mx;
        shape_bbox(&s->shapes[idx[i]], &mn, &mx);
        it[i].idx = idx[i];
        it[i].key = axis == 0 ? mn.x : mn.y;
    }
    qsort(it, n, sizeof *it, cmp_items);
    for (int i = 0; i < n; i++) idx[i] = it[i].idx;
    free(it);
    bvh_node node;
    if (n == 1) {
        node.left = -(idx[0] + 1);
        node.right = INT32_MIN;
    } else if (n == 2) {
        node.left = -(idx[0] + 1);
        node.right = -(idx[1] + 1);
    } else {
        node.left = bvh_build(s, idx, n / 2, rng);
        node.right = bvh_build(s, idx + n / 2, n - n / 2, rng);
    }
    v3 lmn, lmx;
    bbox_of(s, node.left, &lmn, &lmx);
    if (node.right != INT32_MIN) {
        v3 rmn, rmx;
        bbox_of(s, node.right, &rmn, &rmx);
        node.mn = vmin(lmn, rmn); /* AABB::max: mod.rs:81-86 */
        node.mx = vmax(lmx, rmx);
    } else {
        node.mn = lmn;
        node.mx = lmx;
    }
    return bvh_push(s, node);
}
void or_scene_use_bvh(or_scene *s, int enable, uint64_t seed) {
    free(s->nodes);
    s->nodes = NULL;
    s->nnodes = 0;
    s->use_bvh = 0;
    if (!enable || s->nshapes == 0) return; /* reference: n == 0 panics */
    s->nodes = malloc(sizeof(bvh_node) * 2 * s->nshapes);
    int *idx = malloc(sizeof(int) * s->nshapes);
    for (int i = 0; i < s->nshapes; i++) idx[i] = i;
    uint64_t rng = seed;
    s->root = bvh_build(s, idx, s->nshapes, &rng);
    free(idx);
    s->use_bvh = 1;
}
static int leaf_test(const or_scene *sc, int shape, v3 wo, v3 wd, double min_t, double max_t,
                     double *t, or_stats *st) {
    const shape_t *s = &sc->shapes[shape];
    return shape_t_obj(s, mpoint(&s->inverse, wo), mvector(&s->inverse, wd), min_t, max_t, t, st);
}
static int ref_hit(const or_scene *sc, int ref, v3 wo, v3 wd, double min_t, double max_t, double *t,
                   int *who, or_stats *st);
/* BvhNode::ray_hit :628-634 then ray_intersect :636-651 */
static int node_hit(const or_scene *sc, int ni, v3 wo, v3 wd, double min_t, double max_t, double *t,
                    int *who, or_stats *st) {
    const bvh_node *n = &sc->nodes[ni];
    if (!aabb_hit(n->mn, n->mx, wo, wd, min_t, max_t)) return 0;
    double lt;
    int lw;
    int lh = ref_hit(sc, n->left, wo, wd, min_t, max_t, &lt, &lw, st);
    if (n->right == INT32_MIN) {
        if (lh) { *t = lt; *who = lw; }
        return lh;
    }
    double rt;
    int rw;
    if (lh) {
        if (ref_hit(sc, n->right, wo, wd, min_t, lt, &rt, &rw, st)) { *t = rt; *who = rw; }
        else { *t = lt; *who = lw; }
        return 1;
    }
    if (ref_hit(sc, n->right, wo, wd, min_t, max_t, &rt, &rw, st)) { *t = rt; *who = rw; return 1; }
    return 0;
}
static int ref_hit(const or_scene *sc, int ref, v3 wo, v3 wd, double min_t, double max_t, double *t,
                   int *who, or_stats *st) {
    if (ref < 0) { /* leaf: Shape::ray_hit :126-137 (no AABB pre-test) */
        *who = -ref - 1;
        return leaf_test(sc, *who, wo, wd, min_t, max_t, t, st);
    }
    return node_hit(sc, ref, wo, wd, min_t, max_t, t, who, st);
}

/* Closest hit over the shape list.  Semantics of ShapeCollection
 * (src/world/shapes/mod.rs:573-597): each shape is tested with
 * max_t = the best distance so far, and a later shape wins an exact tie
 * (a hit is rejected only if t > max_t).  The reference's BvhNode
 * (mod.rs:620-729) returns the same hit up to exact-t ties. */
int or_closest_hit(const or_scene *sc, const double o[3], const double d[3], double min_t,
                   double max_t, or_hit *out, or_stats *st) {
    v3 wo = vload(o), wd = vload(d);
    double best = max_t;
    int besti = -1;
    if (st) st->bounces++;
    if (sc->use_bvh) {
        if (!node_hit(sc, sc->root, wo, wd, min_t, max_t, &best, &besti, st)) return 0;
        finish_hit(&sc->shapes[besti], besti, wo, wd, best, out);
        return 1;
    }
    for (int i = 0; i < sc->nshapes; i++) {
        const shape_t *s = &sc->shapes[i];
        double t;
        if (shape_t_obj(s, mpoint(&s->inverse, wo), mvector(&s->inverse, wd), min_t, best, &t, st)) {
            best = t;
            besti = i;
        }
    }
    if (besti < 0) return 0;
    finish_hit(&sc->shapes[besti], besti, wo, wd, best, out);
    return 1;
}

/* ======================================================================= */
/* Textures (src/world/texture.rs) and Perlin noise (src/algebra/noise.rs)  */
/* ======================================================================= */
/* Rng::gen::<u32> on the stream: the high half of the next output (RNG spec). */
static uint32_t rng_u32(uint64_t *st) { return (uint32_t)(or_rng_next(st) >> 32); }
/* gen_range(0..n) for u32 = UniformInt::sample_single_inclusive(0, n - 1)
 * (rand 0.8.5 distributions/uniform.rs): zone = (n << lz(n)) - 1, accept the
 * high word of v * n when the low word <= zone. */
static uint32_t rng_below(uint64_t *st, uint32_t n) {
    uint32_t zone = (n << __builtin_clz(n)) - 1u;
    for (;;) {
        uint64_t m = (uint64_t)rng_u32(st) * (uint64_t)n;
        if ((uint32_t)m <= zone) return (uint32_t)(m >> 32);
    }
}
/* SliceRandom::shuffle (rand 0.8 seq/mod.rs): i from len-1 down to 1, swap i with gen_index(i + 1). */
static void shuffle256(int *a, uint64_t *st) {
    for (int i = 0; i < 256; i++) a[i] = i;
    for (uint32_t i = 255; i >= 1; i--) {
        uint32_t j = rng_below(st, i + 1);
        int t = a[i];
        a[i] = a[j];
        a[j] = t;
    }
}
/* Perlin::new (noise.rs:23-42) on the k-th NoiseTexture's stream. */
static void perlin_new(uint64_t seed, uint32_t k, perlin_t *P) {
    uint64_t st = or_mix64(seed ^ 0x50455246494E4F49ull) + (uint64_t)(k + 1) * 0xD1B54A32D192ED03ull;
    shuffle256(P->perm_x, &st);
    shuffle256(P->perm_y, &st);
    shuffle256(P->perm_z, &st);
    for (int i = 0; i < 256; i++) (void)or_gen_f64(&st); /* ranfloat: drawn, never read */
    double s11 = or_uniform_incl_scale(-1.0, 1.0);
    for (int i = 0; i < 256; i++) { /* Vector3d::random(-1, 1): x, y, z draws (algebra/mod.rs:59-66) */
        double x = uniform_sample(&st, -1.0, s11);
        double y = uniform_sample(&st, -1.0, s11);
        double z = uniform_sample(&st, -1.0, s11);
        P->ranvec[i] = V(x, y, z);
    }
}
/* `f64 as i32`: saturating, NaN -> 0 */
static int32_t as_i32(double x) {
    if (isnan(x)) return 0;
    if (x >= 2147483647.0) return INT32_MAX;
    if (x <= -2147483648.0) return INT32_MIN;
    return (int32_t)x;
}
static uint32_t as_u32(double x) {
    if (isnan(x) || x <= 0.0) return 0;
    if (x >= 4294967295.0) return UINT32_MAX;
    return (uint32_t)x;
}
/* Perlin::noise (noise.rs:44-74): cartesian = (0..3).map(|_| 0..2).multi_cartesian_product()
 * (last coordinate fastest); (d + x) & 255 with wrapping i32 add; terms summed in order. */
static double perlin_noise(const perlin_t *P, v3 p) {
    int32_t x = as_i32(floor(p.x)), y = as_i32(floor(p.y)), z = as_i32(floor(p.z));
    double u = p.x - floor(p.x), v = p.y - floor(p.y), w = p.z - floor(p.z);
    double u2 = u * u * (3.0 - 2.0 * u);
    double v2 = v * v * (3.0 - 2.0 * v);
    double w2 = w * w * (3.0 - 2.0 * w);
    double sum = 0.0;
    for (int a = 0; a < 2; a++)
        for (int b = 0; b < 2; b++)
            for (int c = 0; c < 2; c++) {
                int ix = (int)(((uint32_t)a + (uint32_t)x) & 255u);
                int iy = (int)(((uint32_t)b + (uint32_t)y) & 255u);
                int iz = (int)(((uint32_t)c + (uint32_t)z) & 255u);
                v3 g = P->ranvec[P->perm_x[ix] ^ P->perm_y[iy] ^ P->perm_z[iz]];
                double fi = (double)a, fj = (double)b, fk = (double)c;
                double term = (fi * u2 + (double)(1 - a) * (1.0 - u2)) * (fj * v2 + (double)(1 - b) * (1.0 - v2)) *
                              (fk * w2 + (double)(1 - c) * (1.0 - w2)) * vdot(g, V(u - fi, v - fj, w - fk));
                sum = sum + term;
            }
    return sum;
}
/* Perlin::turb (noise.rs:76-88): the scan multiplies weight into noise(p) of
 * the ORIGINAL p every octave (temp_p is updated but never read). */
static double perlin_turb(const perlin_t *P, v3 p, int depth) {
    double weight = 1.0, sum = 0.0;
    for (int i = 0; i < depth; i++) {
        double ret = weight * perlin_noise(P, p);
        weight *= 0.5;
        sum = sum + ret;
    }
    return fabs(sum);
}
void or_perlin_tables(uint64_t seed, uint32_t k, int32_t perm[768], double ranvec[768]) {
    perlin_t P;
    perlin_new(seed, k, &P);
    for (int i = 0; i < 256; i++) {
        perm[i] = P.perm_x[i];
        perm[256 + i] = P.perm_y[i];
        perm[512 + i] = P.perm_z[i];
        vstore(ranvec + 3 * i, P.ranvec[i]);
    }
}
double or_perlin_turb(uint64_t seed, uint32_t k, const double p[3]) {
    perlin_t P;
    perlin_new(seed, k, &P);
    return perlin_turb(&P, vload(p), 7);
}
static v3 texture_value(const or_scene *sc, int node, double u, double v, v3 p) {
    const or_texture_in *t = &sc->tex[node];
    switch (t->type) {
    case OR_TEX_SOLID: return vload(t->c); /* :15-20 */
    case OR_TEX_CHECKER: { /* :40-51 */
        double sines = sin(t->c[0] * p.x) * sin(t->c[1] * p.y) * sin(t->c[2] * p.z);
        return texture_value(sc, sines < 0.0 ? t->odd : t->even, u, v, p);
    }
    case OR_TEX_UVCHECKER: { /* :76-87 */
        double sines = sin(v * t->c[0] * M_PI) * sin(u * t->c[1] * M_PI);
        return texture_value(sc, sines < 0.0 ? t->odd : t->even, u, v, p);
    }
    case OR_TEX_NOISE: { /* :60-66 */
        double a = 0.5 * (1.0 + sin(t->c[0] * p.z + 10.0 * perlin_turb(&sc->perlin[node], p, 7)));
        return V(1.0 * a, 1.0 * a, 1.0 * a);
    }
    case OR_TEX_IMAGE: { /* :96-116; get_pixel would panic at x == width / y == height: clamped */
        const image_t *im = &sc->images[t->aux];
        double uc = u < 0.0 ? 0.0 : (u > 1.0 ? 1.0 : u);
        double vc = 1.0 - (v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v));
        uint32_t x = as_u32(uc * (double)im->w), y = as_u32(vc * (double)im->h);
        if (x >= im->w) x = im->w - 1;
        if (y >= im->h) y = im->h - 1;
        const uint8_t *q = im->rgba + ((size_t)y * im->w + x) * 4;
        double cs = 1.0 / 255.0;
        return V((double)q[0] * cs, (double)q[1] * cs, (double)q[2] * cs);
    }
    }
    return V(NAN, NAN, NAN);
}
void or_scene_set_textures(or_scene *s, const or_texture_in *tex, int ntex, uint64_t seed) {
    free(s->tex);
    free(s->perlin);
    s->tex = malloc(sizeof(or_texture_in) * (ntex > 0 ? ntex : 1));
    s->perlin = calloc(ntex > 0 ? ntex : 1, sizeof(perlin_t));
    s->ntex = ntex;
    uint32_t k = 0;
    for (int i = 0; i < ntex; i++) {
        s->tex[i] = tex[i];
        if (tex[i].type == OR_TEX_NOISE) perlin_new(seed, k++, &s->perlin[i]);
    }
}
int or_scene_add_image(or_scene *s, uint32_t width, uint32_t height, const uint8_t *rgba) {
    s->images = realloc(s->images, sizeof(image_t) * (s->nimages + 1));
    image_t *im = &s->images[s->nimages];
    im->w = width;
    im->h = height;
    im->rgba = malloc((size_t)width * height * 4);
    memcpy(im->rgba, rgba, (size_t)width * height * 4);
    return s->nimages++;
}
void or_texture_value(const or_scene *s, int tex, double u, double v, const double p[3], double out[3]) {
    vstore(out, texture_value(s, tex, u, v, vload(p)));
}

/* ======================================================================= */
/* Materials (src/world/material.rs)                                       */
/* ======================================================================= */
static v3 random_in_unit_sphere(uint64_t *rng, double s11, or_stats *st) { /* algebra/mod.rs:77-84 */
    for (;;) {
        double x = uniform_sample(rng, -1.0, s11);
        double y = uniform_sample(rng, -1.0, s11);
        double z = uniform_sample(rng, -1.0, s11);
        if (st) st->rejection_tries++;
        v3 v = V(x, y, z);
        if (vdot(v, v) <= 1.0) return v;
    }
}
/* returns 1 if scattered (ray + attenuation), 0 if absorbed */
static int scatter(const or_scene *sc, const mat_t *m, v3 rd, const or_hit *h, uint64_t *rng, double s11, v3 *no,
                   v3 *nd, v3 *att, or_stats *st) {
    v3 n = vload(h->normal), p = vload(h->point);
    if (st && m->type >= 0 && m->type < 5) st->scatters[m->type]++;
    switch (m->type) {
    case OR_LAMBERTIAN: { /* material.rs:41-54 */
        v3 dir = vadd(n, vnorm(random_in_unit_sphere(rng, s11, st)));
        if (vis_zero(dir)) dir = n;
        *no = p;
        *nd = vnorm(dir);
        *att = m->tex < 0 ? m->albedo : texture_value(sc, m->tex, h->u, h->v, p);
        return 1;
    }
    case OR_METAL: { /* material.rs:63-76 */
        v3 refl = vreflect(rd, n);
        v3 dir = m->fuzz == 0.0 ? refl : vadd(refl, vscale(random_in_unit_sphere(rng, s11, st), m->fuzz));
        *no = p;
        *nd = vnorm(dir);
        *att = m->tex < 0 ? m->albedo : texture_value(sc, m->tex, h->u, h->v, p);
        return 1;
    }
    case OR_DIELECTRIC: { /* material.rs:92-115, reflectance :84-88 */
        double ratio = h->front_face ? 1.0 / m->ior : m->ior;
        double cos_theta = vdot(vneg(rd), n);
        double sin_theta = sqrt(1.0 - cos_theta * cos_theta);
        int refl = ratio * sin_theta > 1.0;
        if (!refl) {
            double r0 = (1.0 - ratio) / (1.0 + ratio);
            r0 = r0 * r0;
            double x = 1.0 - cos_theta;
            double x5 = x * ((x * x) * (x * x)); /* powi(5) by repeated squaring */
            double refl_p = r0 + (1.0 - r0) * x5;
            refl = refl_p > or_gen_f64(rng);
        }
        v3 dir = refl ? vreflect(rd, n) : vrefract(rd, n, ratio);
        *no = p;
        *nd = vnorm(dir);
        *att = V(1.0, 1.0, 1.0);
        return 1;
    }
    default: return 0; /* DiffuseLight / EmptyMaterial: Material::scatter default None */
    }
}
static v3 emitted(const or_scene *sc, const mat_t *m, const or_hit *h) { /* material.rs:124-128, 22-31 */
    if (m->type != OR_DIFFUSE_LIGHT) return V(0.0, 0.0, 0.0);
    return m->tex < 0 ? m->emit : texture_value(sc, m->tex, h->u, h->v, vload(h->point));
}
/* Scene::background: src/world/mod.rs:199-202 (ignores the JSON value) */
static v3 background(v3 d) {
    double t = 0.5 * (d.y + 1.0);
    return vadd(vscale(V(1.0, 1.0, 1.0), 1.0 - t), vscale(V(0.5, 0.7, 1.0), t));
}

/* ray_color: src/renderer/mod.rs:23-45 — recursive, product order
 * attenuation ⊙ ray_color(child) kept literally. */
static v3 ray_color_rec(const or_scene *sc, v3 o, v3 d, uint32_t depth, uint64_t *rng, double s11,
                        or_stats *st) {
    or_hit h;
    double oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
    if (!or_closest_hit(sc, oo, dd, 0.001, INFINITY, &h, st)) return background(d);
    if (depth == 0) return V(0.0, 0.0, 0.0);
    const mat_t *m = &sc->mats[h.material];
    v3 no, nd, att;
    if (scatter(sc, m, d, &h, rng, s11, &no, &nd, &att, st))
        return vprod(att, ray_color_rec(sc, no, nd, depth - 1, rng, s11, st));
    return emitted(sc, m, &h);
}
void or_ray_color(const or_scene *sc, const double o[3], const double d[3], uint32_t depth,
                  uint64_t *rng_state, double out[3], or_stats *st) {
    double s11 = or_uniform_incl_scale(-1.0, 1.0);
    vstore(out, ray_color_rec(sc, vload(o), vload(d), depth, rng_state, s11, st));
}

/* trace_pixel_samples: src/renderer/mod.rs:151-155, rays from
 * MultisamplerRayCaster::next (ray_caster.rs:103-118): u then v per sample. */
static v3 trace_pixel(const or_scene *sc, const or_caster *k, uint32_t x, uint32_t y, uint32_t spp,
                      uint32_t depth, uint64_t seed, double s11, or_stats *st) {
    v3 acc = V(0.0, 0.0, 0.0);
    uint64_t pixel = (uint64_t)x + (uint64_t)y * k->width;
    for (uint32_t s = 0; s < spp; s++) {
        uint64_t rng = or_sample_key(seed, pixel, s);
        double u = or_gen_f64(&rng);
        double v = or_gen_f64(&rng);
        double o[3], d[3];
        or_caster_ray(k, (double)x + u, (double)y + v, o, d);
        if (st) st->samples++;
        acc = vadd(acc, ray_color_rec(sc, vload(o), vload(d), depth, &rng, s11, st));
    }
    return vdivs(acc, (double)spp);
}
void or_trace_pixel(const or_scene *sc, const or_caster *k, uint32_t x, uint32_t y, uint32_t spp,
                    uint32_t depth, uint64_t seed, double out[3], or_stats *st) {
    vstore(out, trace_pixel(sc, k, x, y, spp, depth, seed, or_uniform_incl_scale(-1.0, 1.0), st));
}

/* ---- threaded driver (src/renderer/mod.rs:66-125 shape) ---------------- */
typedef struct {
    const or_scene *sc;
    const or_caster *k;
    uint32_t spp, depth;
    uint64_t seed;
    const uint32_t *pixels;
    size_t npix, chunk;
    double *out;
    atomic_size_t next;
    or_stats stats;
    pthread_mutex_t lock;
    int want_stats;
} job_t;

static void *worker(void *arg) {
    job_t *j = arg;
    or_stats local;
    memset(&local, 0, sizeof local);
    double s11 = or_uniform_incl_scale(-1.0, 1.0);
    for (;;) {
        size_t c = atomic_fetch_add(&j->next, 1);
        size_t lo = c * j->chunk;
        if (lo >= j->npix) break;
        size_t hi = lo + j->chunk < j->npix ? lo + j->chunk : j->npix;
        for (size_t i = lo; i < hi; i++) {
            uint32_t idx = j->pixels[i];
            uint32_t x = idx % j->k->width, y = idx / j->k->width;
            v3 c3 = trace_pixel(j->sc, j->k, x, y, j->spp, j->depth, j->seed, s11,
                                j->want_stats ? &local : NULL);
            vstore(j->out + 3 * i, c3);
        }
    }
    if (j->want_stats) {
        pthread_mutex_lock(&j->lock);
        uint64_t *a = (uint64_t *)&j->stats, *b = (uint64_t *)&local;
        for (size_t q = 0; q < sizeof(or_stats) / 8; q++) a[q] += b[q];
        pthread_mutex_unlock(&j->lock);
    }
    return NULL;
}

int or_render(const or_scene *sc, const or_caster *k, uint32_t spp, uint32_t depth, uint64_t seed,
              const uint32_t *pixels, size_t npix, int threads, double *out, or_stats *st) {
    if (threads < 1) threads = 1;
    job_t j;
    memset(&j, 0, sizeof j);
    j.sc = sc;
    j.k = k;
    j.spp = spp;
    j.depth = depth;
    j.seed = seed;
    j.pixels = pixels;
    j.npix = npix;
    j.chunk = npix / (size_t)threads / 8; /* mod.rs:74 */
    if (j.chunk == 0) j.chunk = 1;
    j.out = out;
    atomic_init(&j.next, 0);
    j.want_stats = st != NULL;
    pthread_mutex_init(&j.lock, NULL);
    pthread_t *tid = malloc(sizeof(pthread_t) * threads);
    int started = 0;
    if (tid)
        while (started < threads && pthread_create(&tid[started], NULL, worker, &j) == 0) started++;
    if (started == 0) worker(&j); /* no thread could start: the caller's thread pulls every chunk */
    for (int i = 0; i < started; i++) pthread_join(tid[i], NULL);
    free(tid);
    pthread_mutex_destroy(&j.lock);
    if (st) *st = j.stats;
    return 0;
}
