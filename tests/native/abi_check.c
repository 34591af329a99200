/* abi_check.c — a plain C caller of include/rs_pathtracing.h (gcc, the header
 * and the .so only: what a C or Rust-FFI user of the boundary compiles).
 *
 *   abi_check layout                 sizeof / offsetof of every boundary struct as
 *                                    this compiler lays it out == pt_abi_layout
 *   abi_check legacy <scene.json>    old callers, `reserved` = 0 where struct_size now
 *                                    sits: 0.1.0's 16-byte struct at the very end of a
 *                                    readable page, the next page PROT_NONE, so a read
 *                                    past it faults, must load the scene (with an
 *                                    ImageTexture, through the built-in reader); 0.2.0's
 *                                    32-byte struct with an image loader set loads it
 *                                    without calling the loader (0 cannot tell the two
 *                                    apart: ABI 4); the current struct calls its loader;
 *                                    a 16-byte struct (struct_size 16) loads without
 *                                    reading past it; a struct_size below 16 is refused
 *   abi_check render <scene.json> <w> <h> <spp> <depth> <seed> <out.f64>
 *                                    Scene::from_json -> ThreadPoolRenderer::new ->
 *                                    start_rendering -> render_step (blocking) through
 *                                    the C-ABI on the GPU; writes the w*h*3 frame
 *
 * Exit status 0 on success; messages on stderr.  Test infrastructure
 * (tests/test_abi.py, tests/test_gpu_renderer.py). */
#define _GNU_SOURCE
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#include "../../include/rs_pathtracing.h"

static char *read_file(const char *path, size_t *len) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *b = malloc((size_t)n + 1);
    if (b && fread(b, 1, (size_t)n, f) != (size_t)n) {
        free(b);
        b = NULL;
    }
    fclose(f);
    if (b) {
        b[n] = 0;
        *len = (size_t)n;
    }
    return b;
}

static int check(const char *what, int which, const uint32_t *mine, int n) {
    uint32_t lib[64];
    int got = pt_abi_layout(which, lib, 64);
    if (got != n) {
        fprintf(stderr, "%s: library reports %d values, this compiler %d\n", what, got, n);
        return 1;
    }
    for (int k = 0; k < n; k++)
        if (lib[k] != mine[k]) {
            fprintf(stderr, "%s: value %d: library %u, this compiler %u\n", what, k, lib[k], mine[k]);
            return 1;
        }
    printf("%s: %u bytes, %d fields match\n", what, mine[0], n - 1);
    return 0;
}

#define OFF(T, f) (uint32_t) offsetof(T, f)

static int do_layout(void) {
    if (pt_abi_version() != PT_ABI_VERSION) {
        fprintf(stderr, "ABI version: library %u, header %d\n", pt_abi_version(), PT_ABI_VERSION);
        return 1;
    }
    const uint32_t so[] = {sizeof(pt_scene_opts), OFF(pt_scene_opts, random_spheres), OFF(pt_scene_opts, struct_size),
                           OFF(pt_scene_opts, seed), OFF(pt_scene_opts, load_image), OFF(pt_scene_opts, image_user)};
    const uint32_t ca[] = {sizeof(pt_camera), OFF(pt_camera, position), OFF(pt_camera, direction), OFF(pt_camera, up),
                           OFF(pt_camera, right), OFF(pt_camera, fov), OFF(pt_camera, focal_length)};
    const uint32_t sh[] = {sizeof(pt_shape_info), OFF(pt_shape_info, type), OFF(pt_shape_info, material),
                           OFF(pt_shape_info, inverse_normal), OFF(pt_shape_info, depth), OFF(pt_shape_info, func),
                           OFF(pt_shape_info, pad0), OFF(pt_shape_info, direct), OFF(pt_shape_info, inverse),
                           OFF(pt_shape_info, x0), OFF(pt_shape_info, y0), OFF(pt_shape_info, x1), OFF(pt_shape_info, y1),
                           OFF(pt_shape_info, step), OFF(pt_shape_info, a), OFF(pt_shape_info, b), OFF(pt_shape_info, c),
                           OFF(pt_shape_info, d), OFF(pt_shape_info, sphere_radius), OFF(pt_shape_info, radius),
                           OFF(pt_shape_info, tube_radius)};
    const uint32_t ma[] = {sizeof(pt_material_info), OFF(pt_material_info, type), OFF(pt_material_info, texture),
                           OFF(pt_material_info, albedo), OFF(pt_material_info, fuzz), OFF(pt_material_info, ior),
                           OFF(pt_material_info, emit)};
    const uint32_t hi[] = {sizeof(pt_hit), OFF(pt_hit, t), OFF(pt_hit, point), OFF(pt_hit, normal),
                           OFF(pt_hit, front_face), OFF(pt_hit, shape), OFF(pt_hit, material), OFF(pt_hit, pad0)};
    const uint32_t ck[] = {sizeof(pt_checkpoint), OFF(pt_checkpoint, width), OFF(pt_checkpoint, height),
                           OFF(pt_checkpoint, samples_number), OFF(pt_checkpoint, samples_done),
                           OFF(pt_checkpoint, rank), OFF(pt_checkpoint, world), OFF(pt_checkpoint, depth),
                           OFF(pt_checkpoint, reserved), OFF(pt_checkpoint, seed), OFF(pt_checkpoint, scene_key),
                           OFF(pt_checkpoint, count)};
    int bad = 0;
    bad |= check("pt_scene_opts", PT_ABI_SCENE_OPTS, so, (int)(sizeof so / sizeof so[0]));
    bad |= check("pt_camera", PT_ABI_CAMERA, ca, (int)(sizeof ca / sizeof ca[0]));
    bad |= check("pt_shape_info", PT_ABI_SHAPE_INFO, sh, (int)(sizeof sh / sizeof sh[0]));
    bad |= check("pt_material_info", PT_ABI_MATERIAL_INFO, ma, (int)(sizeof ma / sizeof ma[0]));
    bad |= check("pt_hit", PT_ABI_HIT, hi, (int)(sizeof hi / sizeof hi[0]));
    bad |= check("pt_checkpoint", PT_ABI_CHECKPOINT, ck, (int)(sizeof ck / sizeof ck[0]));
    if (pt_abi_layout(99, NULL, 0) != PT_ERR_INVALID) {
        fprintf(stderr, "unknown struct id accepted\n");
        bad = 1;
    }
    return bad;
}

/* the options struct of 0.1.0 / 0.2.0: 32 bytes, `reserved` always 0 */
typedef struct {
    uint32_t random_spheres;
    uint32_t reserved;
    uint64_t seed;
    pt_image_loader load_image;
    void *image_user;
} opts_v02;

/* an image loader that answers every file with a 2x2 RGBA8 image and counts its calls */
static const uint8_t tiny_rgba[16] = {255, 0, 0, 255, 0, 255, 0, 255, 0, 0, 255, 255, 255, 255, 255, 255};
static int counting_loader(void *user, const char *filename, uint32_t *w, uint32_t *h, const uint8_t **rgba8) {
    (void)filename;
    ++*(int *)user;
    *w = 2;
    *h = 2;
    *rgba8 = tiny_rgba;
    return PT_OK;
}

static int do_legacy(const char *path) {
    size_t len = 0;
    char *json = read_file(path, &len);
    if (!json) {
        fprintf(stderr, "cannot read %s\n", path);
        return 1;
    }
    const long pg = sysconf(_SC_PAGESIZE);
    char *mem = mmap(NULL, (size_t)pg * 2, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (mem == MAP_FAILED || mprotect(mem + pg, (size_t)pg, PROT_NONE) != 0) {
        fprintf(stderr, "mmap / mprotect failed\n");
        return 1;
    }
    int calls = 0;
    /* 0.1.0: the 16 bytes {random_spheres, reserved = 0, seed} against the page end */
    uint32_t *o10 = (uint32_t *)(mem + pg - 16);
    o10[0] = 1;
    o10[1] = 0;
    *(uint64_t *)(o10 + 2) = 7;
    pt_scene *s = NULL;
    int rc = pt_scene_create_from_json(json, len, (const pt_scene_opts *)o10, &s);
    if (rc != PT_OK) {
        fprintf(stderr, "0.1.0 opts: status %d: %s\n", rc, pt_last_error());
        return 1;
    }
    printf("0.1.0 opts: %d shapes, %d materials\n", pt_scene_num_shapes(s), pt_scene_num_materials(s));
    pt_scene_destroy(s);
    /* 0.2.0: the 32-byte struct with a loader and reserved = 0 (ABI 4: the loader is not read) */
    opts_v02 *o = (opts_v02 *)(mem + pg - sizeof(opts_v02));
    o->random_spheres = 1;
    o->reserved = 0;
    o->seed = 7;
    o->load_image = counting_loader;
    o->image_user = &calls;
    s = NULL;
    rc = pt_scene_create_from_json(json, len, (const pt_scene_opts *)o, &s);
    if (rc != PT_OK) {
        fprintf(stderr, "0.2.0 opts: status %d: %s\n", rc, pt_last_error());
        return 1;
    }
    if (calls != 0) {
        fprintf(stderr, "0.2.0 opts (struct_size 0): the loader was read and called\n");
        return 1;
    }
    printf("0.2.0 opts: %d shapes, loader not called\n", pt_scene_num_shapes(s));
    pt_scene_destroy(s);
    /* the current struct with its loader: called */
    pt_scene_opts withl = PT_SCENE_OPTS_INIT;
    withl.seed = 7;
    withl.load_image = counting_loader;
    withl.image_user = &calls;
    s = NULL;
    rc = pt_scene_create_from_json(json, len, &withl, &s);
    if (rc != PT_OK || calls == 0) {
        fprintf(stderr, "current opts with a loader: status %d, %d loader calls: %s\n", rc, calls, pt_last_error());
        return 1;
    }
    printf("current opts: loader called %d times\n", calls);
    pt_scene_destroy(s);
    /* the 16 bytes {random_spheres, struct_size = 16, seed} against the page end: no loader is read */
    uint32_t *o16 = (uint32_t *)(mem + pg - 16);
    o16[0] = 1;
    o16[1] = 16;
    *(uint64_t *)(o16 + 2) = 7;
    s = NULL;
    rc = pt_scene_create_from_json(json, len, (const pt_scene_opts *)o16, &s);
    if (rc != PT_OK) {
        fprintf(stderr, "16-byte opts: status %d: %s\n", rc, pt_last_error());
        return 1;
    }
    printf("16-byte opts: %d shapes\n", pt_scene_num_shapes(s));
    pt_scene_destroy(s);
    /* a struct_size that cannot hold even {random_spheres, struct_size, seed} */
    o16[1] = 8;
    s = NULL;
    rc = pt_scene_create_from_json(json, len, (const pt_scene_opts *)o16, &s);
    if (rc != PT_ERR_INVALID || s) {
        fprintf(stderr, "struct_size 8 accepted (status %d)\n", rc);
        return 1;
    }
    printf("struct_size 8 refused: %s\n", pt_last_error());
    /* the current struct, through the initializer */
    pt_scene_opts cur = PT_SCENE_OPTS_INIT;
    cur.seed = 7;
    rc = pt_scene_create_from_json(json, len, &cur, &s);
    if (rc != PT_OK) {
        fprintf(stderr, "current opts: status %d: %s\n", rc, pt_last_error());
        return 1;
    }
    printf("current opts: %d shapes\n", pt_scene_num_shapes(s));
    pt_scene_destroy(s);
    munmap(mem, (size_t)pg * 2);
    free(json);
    return 0;
}

static int do_render(int argc, char **argv) {
    if (argc < 9) {
        fprintf(stderr, "usage: abi_check render <scene.json> <w> <h> <spp> <depth> <seed> <out.f64>\n");
        return 2;
    }
    size_t len = 0;
    char *json = read_file(argv[2], &len);
    if (!json) return 1;
    const uint32_t w = (uint32_t)atoi(argv[3]), h = (uint32_t)atoi(argv[4]), spp = (uint32_t)atoi(argv[5]),
                   depth = (uint32_t)atoi(argv[6]);
    const uint64_t seed = strtoull(argv[7], NULL, 10);
    pt_scene_opts o = PT_SCENE_OPTS_INIT;
    o.seed = 1;
    pt_scene *s = NULL;
    pt_renderer *r = NULL;
    pt_camera cam;
    double *rgb = calloc((size_t)w * h * 3, sizeof(double));
    int rc = pt_scene_create_from_json(json, len, &o, &s);
    if (rc == PT_OK) rc = pt_scene_camera(s, &cam);
    if (rc == PT_OK) rc = pt_renderer_create(s, -1, depth, &r);
    if (rc == PT_OK) rc = pt_render_start(r, &cam, w, h, spp, seed);
    if (rc == PT_OK) rc = pt_render_step(r, rgb, 1);
    if (rc != 1) {
        fprintf(stderr, "render: status %d: %s\n", rc, pt_last_error());
        return 1;
    }
    FILE *f = fopen(argv[8], "wb");
    if (!f || fwrite(rgb, sizeof(double), (size_t)w * h * 3, f) != (size_t)w * h * 3) return 1;
    fclose(f);
    pt_renderer_destroy(r);
    pt_scene_destroy(s);
    free(rgb);
    free(json);
    printf("rendered %ux%u at %u spp\n", w, h, spp);
    return 0;
}

/* A rank's running sums through a checkpoint file and back (host only). */
static int do_checkpoint(const char *path) {
    pt_checkpoint c;
    memset(&c, 0, sizeof c);
    c.width = 100;
    c.height = 37;
    c.samples_number = 64;
    c.samples_done = 24;
    c.rank = 1;
    c.world = 2;
    c.depth = 50;
    c.seed = 7;
    c.scene_key = 0x0123456789abcdefull;
    c.count = (uint64_t)pt_shard_tiles(c.width, c.height, c.rank, c.world) * 256 * 3;
    double *sums = malloc(c.count * sizeof(double)), *back = malloc(c.count * sizeof(double));
    for (uint64_t i = 0; i < c.count; i++) sums[i] = (double)i * 0.1 - 3.0;
    int rc = pt_checkpoint_save(path, &c, sums);
    pt_checkpoint d;
    if (rc == PT_OK) rc = pt_checkpoint_load(path, &d, back, c.count);
    if (rc != PT_OK || memcmp(&c, &d, sizeof c) || memcmp(sums, back, c.count * sizeof(double))) {
        fprintf(stderr, "round trip: status %d: %s\n", rc, pt_last_error());
        return 1;
    }
    printf("checkpoint round trip: %llu sums\n", (unsigned long long)c.count);
    FILE *f = fopen(path, "r+b");
    if (!f || fseek(f, 8 + 56 + 8 * 1000 + 3, SEEK_SET) != 0 || fputc(0x5a, f) == EOF || fclose(f) != 0) return 1;
    rc = pt_checkpoint_load(path, &d, back, c.count);
    if (rc != PT_ERR_IO || back[1000] != 0.0) {
        fprintf(stderr, "corrupt file: status %d\n", rc);
        return 1;
    }
    printf("corrupt file refused: %s\n", pt_last_error());
    free(sums);
    free(back);
    return 0;
}

int main(int argc, char **argv) {
    if (argc >= 3 && !strcmp(argv[1], "checkpoint")) return do_checkpoint(argv[2]);
    if (argc >= 2 && !strcmp(argv[1], "layout")) return do_layout();
    if (argc >= 3 && !strcmp(argv[1], "legacy")) return do_legacy(argv[2]);
    if (argc >= 2 && !strcmp(argv[1], "render")) return do_render(argc, argv);
    fprintf(stderr, "usage: abi_check layout | legacy <scene.json> | render ...\n");
    return 2;
}
