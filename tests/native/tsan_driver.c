/* tsan_driver.c — ThreadSanitizer run of the oracle's threaded renderer
 * (or_render: step_by_step-shaped workers pulling pixel chunks from an atomic
 * counter, src/renderer/mod.rs:66-125), built with -fsanitize=thread by
 * `make -C oracle tsan` (scripts/san.sh).  A small scene with every material
 * kind, a ray-marched Heart and the ~480 random spheres is rendered with 8
 * threads in both traversal modes (linear scan, the reference's BvhNode) and
 * with 1 thread; the three frames must be bit-identical.  Test infrastructure
 * only; exit status 0 when the frames agree (TSan reports make it non-zero). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/pt_oracle.h"

static or_shape_in shape(int type, int material, double tx, double ty, double tz, double s) {
    or_shape_in r;
    memset(&r, 0, sizeof r);
    r.type = type;
    r.material = material;
    r.translate[0] = tx, r.translate[1] = ty, r.translate[2] = tz;
    r.scale[0] = r.scale[1] = r.scale[2] = s;
    r.depth = 4;
    return r;
}

int main(void) {
    or_material_in m[6];
    memset(m, 0, sizeof m);
    for (int i = 0; i < 6; i++) m[i].tex = -1;
    m[0].type = OR_LAMBERTIAN, m[0].albedo[0] = 0.5, m[0].albedo[1] = 0.5, m[0].albedo[2] = 0.5;
    m[1].type = OR_METAL, m[1].albedo[0] = 0.7, m[1].albedo[1] = 0.6, m[1].albedo[2] = 0.5, m[1].fuzz = 0.1;
    m[2].type = OR_DIELECTRIC, m[2].ior = 1.5;
    m[3].type = OR_DIFFUSE_LIGHT, m[3].emit[0] = m[3].emit[1] = m[3].emit[2] = 4.0;
    m[4].type = OR_LAMBERTIAN, m[4].albedo[0] = 0.65, m[4].albedo[1] = 0.05, m[4].albedo[2] = 0.05;
    m[5].type = OR_EMPTY;
    or_shape_in s[7];
    s[0] = shape(OR_SPHERE, 0, 0, -1000, 0, 1000);
    s[1] = shape(OR_SPHERE, 1, 4, 1, 0, 1);
    s[2] = shape(OR_SPHERE, 2, 0, 1, 0, 1);
    s[3] = shape(OR_CUBE, 4, -4, 1, 0, 0.8);
    s[3].rotate[1] = 20;
    s[4] = shape(OR_RECT, 3, -2, 5, -2, 1);
    s[4].x0 = 0, s[4].x1 = 4, s[4].y0 = 0, s[4].y1 = 4, s[4].rotate[0] = 90;
    s[5] = shape(OR_MARCH, 4, 2, 1.2, 3, 1);
    s[5].func = OR_FUNC_HEART, s[5].step = 0.01, s[5].rotate[0] = -90;
    s[6] = shape(OR_SPHERE, 5, -1, 0.5, 3, 0.5);
    or_scene *sc = or_scene_new(s, 7, m, 6, 1, 3);
    if (!sc) {
        fprintf(stderr, "or_scene_new failed\n");
        return 1;
    }
    const double pos[3] = {13, 2, 3}, dir[3] = {-13, -2, -3}, up[3] = {0, 1, 0};
    or_camera cam;
    or_camera_new(pos, dir, up, 10.0, or_to_radians(20.0), &cam);
    const uint32_t w = 96, h = 54, spp = 2, depth = 8;
    or_caster k;
    or_caster_new(&cam, w, h, &k);
    const size_t n = (size_t)w * h;
    uint32_t *px = malloc(n * sizeof *px);
    double *a = malloc(n * 3 * sizeof *a), *b = malloc(n * 3 * sizeof *b), *c = malloc(n * 3 * sizeof *c);
    if (!px || !a || !b || !c) return 1;
    for (size_t i = 0; i < n; i++) px[i] = (uint32_t)i;
    or_stats st;
    or_render(sc, &k, spp, depth, 9, px, n, 8, a, &st);  /* linear scan, 8 workers, per-thread stats merged */
    or_render(sc, &k, spp, depth, 9, px, n, 1, b, NULL);
    or_scene_use_bvh(sc, 1, 7);
    or_render(sc, &k, spp, depth, 9, px, n, 8, c, NULL); /* the reference's BvhNode traversal */
    const int same_ab = memcmp(a, b, n * 3 * sizeof *a) == 0, same_ac = memcmp(a, c, n * 3 * sizeof *a) == 0;
    double mean = 0;
    for (size_t i = 0; i < n * 3; i++) mean += a[i];
    printf("tsan_driver: %zu pixels, mean %.6f, samples %llu, 8 vs 1 threads %s, linear vs BVH %s\n", n,
           mean / (double)(n * 3), (unsigned long long)st.samples, same_ab ? "equal" : "DIFFER",
           same_ac ? "equal" : "DIFFER");
    or_scene_free(sc);
    free(px), free(a), free(b), free(c);
    return same_ab && same_ac && st.samples == (unsigned long long)n * spp ? 0 : 1;
}
