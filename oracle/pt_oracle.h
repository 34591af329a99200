/*
 * pt_oracle.h — CPU restatement of the rs-pathtracing per-pixel sample path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker for the MI355X HIP
 * path: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load it.  The product (rs-pathtracing_amd/) never links or calls it.
 *
 * Every function restates the reference Rust code it cites (paths relative to
 * the reference checkout), in f64, with the same operation order, so that the
 * HIP kernel (compiled with -ffp-contract=off) can be compared bit for bit.
 *
 * Pinning status:
 *   - transforms, camera basis, AABB transform: pinned by the reference's own
 *     unit tests (tests/test_oracle_reference_kats.py);
 *   - primitive intersections, scatter, ray_color: hand-derived known answers
 *     and an independent numpy restatement (tests/golden/);
 *   - anything that consumes random numbers: the reference draws from an
 *     unseedable rand::thread_rng, so image-level parity against the
 *     reference binary is UNPINNED (statistical only).  The oracle replaces
 *     the stream with a documented counter-based SplitMix64 stream and keeps
 *     rand 0.8's float conversions exactly.
 */
#ifndef PT_ORACLE_H
#define PT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* shape kinds (src/world/shapes/mod.rs, src/world/shapes/ray_marching.rs) */
#define OR_SPHERE 0
#define OR_RECT 1
#define OR_CUBE 2
#define OR_MARCH 3
#define OR_TORUS 4

/* ray-marched implicit functions (src/world/shapes/ray_marching.rs) */
#define OR_FUNC_HEART 0
#define OR_FUNC_SINE 1
#define OR_FUNC_STAR 2
#define OR_FUNC_DUPIN 3
#define OR_FUNC_HUNTS 4
#define OR_FUNC_CUSHION 5

/* materials (src/world/material.rs) */
#define OR_LAMBERTIAN 0
#define OR_METAL 1
#define OR_DIELECTRIC 2
#define OR_DIFFUSE_LIGHT 3
#define OR_EMPTY 4

typedef struct {
    int32_t type, material, inverse_normal, depth;
    int32_t func, pad0;
    double translate[3], rotate[3], scale[3];
    double x0, y0, x1, y1, step;
    double fa, fb, fc, fd, fr; /* ray-marched function: a, b, c, d, sphere_radius */
    double radius, tube_radius; /* Torus */
} or_shape_in;

/* textures (src/world/texture.rs) */
#define OR_TEX_SOLID 0
#define OR_TEX_CHECKER 1
#define OR_TEX_UVCHECKER 2
#define OR_TEX_NOISE 3
#define OR_TEX_IMAGE 4

typedef struct {
    int32_t type;
    int32_t tex; /* -1: SolidColor in albedo / emit; else the root texture node */
    double albedo[3];
    double fuzz;
    double ior;
    double emit[3];
} or_material_in;

/* texture tree node: checker kinds pick child odd/even; image: aux = image index */
typedef struct {
    int32_t type, odd, even, aux;
    double c[3]; /* colour | CheckerTexture multipliers | UVChecker multipliers | noise scale */
} or_texture_in;

typedef struct {
    int32_t type, material, inverse_normal, depth, func, pad0;
    double direct[16], inverse[16];
    double x0, y0, x1, y1, step;
    double fa, fb, fc, fd, fr;
    double radius, tube_radius;
} or_shape_out;

typedef struct {
    double t;
    double point[3];
    double normal[3];
    int32_t front_face, shape, material, pad0;
    double u, v; /* RayHit u, v (texture coordinates) */
} or_hit;

typedef struct {
    uint64_t shape_tests[4];   /* leaf tests per shape kind                 */
    uint64_t march_steps;      /* Heart march inner iterations               */
    uint64_t march_bounds;     /* Heart bound (ellipsoid) solves             */
    uint64_t bounces;          /* closest-hit queries                        */
    uint64_t rejection_tries;  /* random_in_unit_sphere attempts            */
    uint64_t samples;          /* camera samples                             */
    uint64_t scatters[5];      /* per material kind                          */
} or_stats;

typedef struct or_scene or_scene;

typedef struct {
    double position[3], direction[3], up[3], right[3];
    double fov, focal_length;
} or_camera;

typedef struct {
    double position[3], right[3], up[3], left_top[3];
    double pixel_resolution;
    uint32_t width, height;
} or_caster;

/* ---- scene ------------------------------------------------------------ */
or_scene *or_scene_new(const or_shape_in *shapes, int n, const or_material_in *mats, int nm,
                       int random_spheres, uint64_t scene_seed);
void or_scene_free(or_scene *s);
/* Non-solid textures: the node array (pre-order per material, as the JSON
 * lists them) and the images they reference (RGBA8, row-major).  The k-th
 * NoiseTexture node draws its Perlin tables from stream k of seed. */
void or_scene_set_textures(or_scene *s, const or_texture_in *tex, int ntex, uint64_t seed);
int or_scene_add_image(or_scene *s, uint32_t width, uint32_t height, const uint8_t *rgba);
/* Perlin::new tables of stream k (perm: 3 x 256, ranvec: 256 x 3) and Perlin::turb(p, 7). */
void or_perlin_tables(uint64_t seed, uint32_t k, int32_t perm[768], double ranvec[768]);
double or_perlin_turb(uint64_t seed, uint32_t k, const double p[3]);
/* Texture::value of node `tex` at (u, v, p). */
void or_texture_value(const or_scene *s, int tex, double u, double v, const double p[3], double out[3]);
int or_scene_num_shapes(const or_scene *s);
int or_scene_num_materials(const or_scene *s);
void or_scene_get_shape(const or_scene *s, int i, or_shape_out *out);
void or_scene_get_material(const or_scene *s, int i, or_material_in *out);
/* Switch closest-hit to the reference's BvhNode traversal (src/world/shapes/mod.rs:620-729),
 * built with a seeded axis stream; default is the ShapeCollection linear scan. */
void or_scene_use_bvh(or_scene *s, int enable, uint64_t seed);

/* ---- algebra (src/algebra/transform.rs) -------------------------------- */
void or_transform_new(const double t[3], const double r[3], const double s[3], double direct[16],
                      double inverse[16]);
void or_rotate(const double r[3], double out[16]);
void or_mat_mul(const double a[16], const double b[16], double out[16]);
void or_aabb_transform(const double mn[3], const double mx[3], const double m[16], double out_mn[3],
                       double out_mx[3]);

/* ---- camera (src/camera/mod.rs, src/camera/ray_caster.rs) -------------- */
void or_camera_new(const double pos[3], const double dir[3], const double up[3], double focal_length,
                   double fov_radians, or_camera *out);
double or_to_radians(double deg);
void or_caster_new(const or_camera *c, uint32_t width, uint32_t height, or_caster *out);
void or_caster_ray(const or_caster *k, double x, double y, double origin[3], double dir[3]);

/* ---- rng (rand 0.8 float conversions over a SplitMix64 stream) --------- */
uint64_t or_mix64(uint64_t z);
uint64_t or_sample_key(uint64_t seed, uint64_t pixel, uint64_t sample);
uint64_t or_rng_next(uint64_t *state);
double or_gen_f64(uint64_t *state);
double or_uniform_incl_scale(double lo, double hi);
double or_gen_range_incl(uint64_t *state, double lo, double hi);

/* ---- Torus (src/world/shapes/mod.rs:429-476; algebra/equation.rs:17-67) --- */
/* solve_quantic_equation on real coefficients: roots re[4], im[4] in its order */
void or_solve_quartic(double a, double b, double c, double d, double e, double re[4], double im[4]);

/* ---- path -------------------------------------------------------------- */
int or_shape_hit(const or_scene *s, int shape, const double o[3], const double d[3], double min_t,
                 double max_t, or_hit *out);
int or_closest_hit(const or_scene *s, const double o[3], const double d[3], double min_t,
                   double max_t, or_hit *out, or_stats *st);
void or_ray_color(const or_scene *s, const double o[3], const double d[3], uint32_t depth,
                  uint64_t *rng_state, double out[3], or_stats *st);
void or_trace_pixel(const or_scene *s, const or_caster *k, uint32_t x, uint32_t y, uint32_t spp,
                    uint32_t depth, uint64_t seed, double out[3], or_stats *st);
/* Threaded renderer in the shape of step_by_step (src/renderer/mod.rs:66-125):
 * pixels (indices x + y*w) are cut into chunks of w*h/threads/8 and pulled by
 * `threads` workers.  out is npix*3 doubles (per-pixel mean). */
int or_render(const or_scene *s, const or_caster *k, uint32_t spp, uint32_t depth, uint64_t seed,
              const uint32_t *pixels, size_t npix, int threads, double *out, or_stats *st);

#ifdef __cplusplus
}
#endif
#endif
