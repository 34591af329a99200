// pt_api.cpp — the C-ABI (include/rs_pathtracing.h).  No exception escapes:
// each entry point catches, stores a thread-local message and returns a
// status.  The renderer owns one HIP stream on its device; start_rendering
// queues the frame as bands of tile rows, each closed by an event, so a
// non-blocking render_step can hand back finished bands while the rest of the
// frame is still on the GPU (src/renderer/step_by_step.rs:101-121).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <new>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/rs_pathtracing.h"
#include "pt_accel.hpp"
#include "pt_kernel.hpp"
#include "pt_scene.hpp"

using namespace pt;

namespace {
thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}
int hip_fail(hipError_t e, const char *what) {
    return fail(PT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
#define HIP_TRY(expr)                                  \
    do {                                               \
        hipError_t e_ = (expr);                        \
        if (e_ != hipSuccess) return hip_fail(e_, #expr); \
    } while (0)

uint32_t tiles_x_of(uint32_t w) { return (w + TILE - 1) / TILE; }
uint32_t tiles_y_of(uint32_t h) { return (h + TILE - 1) / TILE; }

}  // namespace

namespace {
template <class T>
struct DevBuf {
    T *p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    hipError_t alloc(size_t n) { return hipMalloc(&p, (n ? n : 1) * sizeof(T)); }
};
}  // namespace

struct pt_scene {
    Scene s;
};

struct pt_renderer {
    pt_scene *scene = nullptr;
    int device = 0;
    uint32_t depth = 0;
    hipStream_t stream = nullptr;
    DeviceScene ds;
    WaveWorkspace ws;  // wavefront engine state (scenes with ray-marched shapes)
    double s11 = 0;

    // frame in flight
    bool started = false;
    uint32_t width = 0, height = 0;
    double *d_frame = nullptr;
    size_t frame_cap = 0;
    struct Band {
        uint32_t row0, row1;
        hipEvent_t ev;
        bool copied;
    };
    std::vector<Band> bands;
};

extern "C" {

const char *pt_last_error(void) { return g_err.c_str(); }
const char *pt_version(void) { return "rs-pathtracing-amd 0.2.0 (gfx950, f64 megakernel + wavefront march engine)"; }

uint64_t pt_sample_key(uint64_t seed, uint64_t pixel, uint64_t sample) { return sample_key(seed, pixel, sample); }

int pt_scene_create_from_json(const char *json, size_t len, const pt_scene_opts *opts, pt_scene **out) {
    if (!json || !out) return fail(PT_ERR_INVALID, "null argument");
    *out = nullptr;
    bool rs = opts ? opts->random_spheres != 0 : true;
    uint64_t seed = opts ? opts->seed : 1;
    ImageSource img;
    if (opts) {
        img.load = opts->load_image;
        img.user = opts->image_user;
    }
    try {
        pt_scene *s = new pt_scene;
        try {
            s->s = scene_from_json(json, len, rs, seed, img);
        } catch (...) {
            delete s;
            throw;
        }
        *out = s;
        return PT_OK;
    } catch (const SceneError &e) {
        return fail(e.code, e.msg);
    } catch (const std::bad_alloc &) {
        return fail(PT_ERR_INVALID, "out of memory");
    } catch (const std::exception &e) {
        return fail(PT_ERR_INVALID, e.what());
    }
}

void pt_scene_destroy(pt_scene *s) { delete s; }

int pt_scene_camera(const pt_scene *s, pt_camera *out) {
    if (!s || !out) return fail(PT_ERR_INVALID, "null argument");
    *out = s->s.camera;
    return PT_OK;
}
int pt_scene_num_shapes(const pt_scene *s) { return s ? (int)s->s.shapes.size() : fail(PT_ERR_INVALID, "null scene"); }
int pt_scene_num_materials(const pt_scene *s) {
    return s ? (int)s->s.materials.size() : fail(PT_ERR_INVALID, "null scene");
}
int pt_scene_get_shape(const pt_scene *s, int i, pt_shape_info *o) {
    if (!s || !o || i < 0 || i >= (int)s->s.shapes.size()) return fail(PT_ERR_INVALID, "shape index out of range");
    const HostShape &h = s->s.shapes[i];
    std::memset(o, 0, sizeof *o);
    o->type = h.type;
    o->material = h.material;
    o->inverse_normal = h.inverse_normal;
    o->depth = h.depth;
    o->func = h.func;
    std::memcpy(o->direct, h.direct, sizeof o->direct);
    std::memcpy(o->inverse, h.inverse, sizeof o->inverse);
    o->x0 = h.x0;
    o->y0 = h.y0;
    o->x1 = h.x1;
    o->y1 = h.y1;
    o->step = h.step;
    o->a = h.fa;
    o->b = h.fb;
    o->c = h.fc;
    o->d = h.fd;
    o->sphere_radius = h.fr;
    o->radius = h.radius;
    o->tube_radius = h.tube_radius;
    return PT_OK;
}
int pt_scene_get_material(const pt_scene *s, int i, pt_material_info *o) {
    if (!s || !o || i < 0 || i >= (int)s->s.materials.size())
        return fail(PT_ERR_INVALID, "material index out of range");
    const HostMaterial &m = s->s.materials[i];
    std::memset(o, 0, sizeof *o);
    o->type = m.type;
    o->texture = m.tex;
    for (int k = 0; k < 3; k++) {
        o->albedo[k] = m.albedo[k];
        o->emit[k] = m.emit[k];
    }
    o->fuzz = m.fuzz;
    o->ior = m.ior;
    return PT_OK;
}

int pt_camera_new(const double position[3], const double direction[3], const double up[3], double focal_length,
                  double fov_radians, pt_camera *out) {
    if (!position || !direction || !up || !out) return fail(PT_ERR_INVALID, "null argument");
    camera_new(position, direction, up, focal_length, fov_radians, out);
    return PT_OK;
}

// ------------------------------------------------------------- renderer
int pt_renderer_create(pt_scene *scene, int device, uint32_t depth, pt_renderer **out) {
    if (!scene || !out) return fail(PT_ERR_INVALID, "null argument");
    *out = nullptr;
    if (depth > 64) return fail(PT_ERR_UNSUPPORTED, "depth > 64 is not supported on the GPU path");
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count == 0) return fail(PT_ERR_HIP, "no HIP device available (the GPU path has no CPU fallback)");
    if (device < 0) HIP_TRY(hipGetDevice(&device));
    if (device >= count) return fail(PT_ERR_INVALID, "device ordinal out of range");
    HIP_TRY(hipSetDevice(device));
    pt_renderer *r = new (std::nothrow) pt_renderer;
    if (!r) return fail(PT_ERR_INVALID, "out of memory");
    r->scene = scene;
    r->device = device;
    r->depth = depth;
    r->s11 = uniform_incl_scale(-1.0, 1.0);
    std::vector<DShape> hs;
    std::vector<DMaterial> hm;
    for (auto &s : scene->s.shapes) hs.push_back(to_device(s));
    for (auto &m : scene->s.materials) hm.push_back(to_device(m));
    if (hm.empty()) hm.push_back(DMaterial{});
    Accel acc = build_accel(scene->s, scene->s.json_shapes);
    hipError_t err = hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking);
    auto upload = [&err](auto **dst, const auto &vec) {
        using T = typename std::remove_reference<decltype(vec)>::type::value_type;
        size_t n = vec.empty() ? 1 : vec.size();
        if (err == hipSuccess) err = hipMalloc((void **)dst, n * sizeof(T));
        if (err == hipSuccess && !vec.empty())
            err = hipMemcpy(*dst, vec.data(), vec.size() * sizeof(T), hipMemcpyHostToDevice);
    };
    upload(&r->ds.shapes, hs);
    upload(&r->ds.mats, hm);
    upload(&r->ds.nodes, acc.cnodes);
    upload(&r->ds.leaf, acc.leaf);
    upload(&r->ds.lin, acc.lin);
    upload(&r->ds.march, acc.march);
    upload(&r->ds.boxes, acc.boxes);
    const Scene &S = scene->s;
    if (!S.textures.empty()) {
        upload(&r->ds.tex, S.textures);
        upload(&r->ds.perlin, S.perlins);
        upload(&r->ds.images, S.images);
        upload(&r->ds.pixels, S.pixels);
    }
    if (err != hipSuccess) {
        pt_renderer_destroy(r);
        return hip_fail(err, "uploading the scene");
    }
    r->ds.nshapes = (int)hs.size();
    r->ds.nmats = (int)hm.size();
    r->ds.nnodes = acc.nodes_per_octant();  // nodes per octant layout
    r->ds.nlin = (int)acc.lin.size();
    r->ds.nmarch = (int)acc.march.size();
    r->ds.ext = S.textures.empty() ? 0 : 1;
    for (const auto &h : S.shapes)
        if (h.type == TORUS) r->ds.ext = 1;
    r->ds.fkind = 0;  // Heart-only kernel builds unless another function is marched
    for (const auto &h : r->scene->s.shapes)
        if (h.type == MARCH && h.func != 0) r->ds.fkind = -1;
    *out = r;
    return PT_OK;
}

static void release_bands(pt_renderer *r) {
    for (auto &b : r->bands) (void)hipEventDestroy(b.ev);
    r->bands.clear();
}

void pt_renderer_destroy(pt_renderer *r) {
    if (!r) return;
    (void)hipSetDevice(r->device);
    if (r->stream) (void)hipStreamSynchronize(r->stream);
    release_bands(r);
    if (r->d_frame) (void)hipFree(r->d_frame);
    if (r->ds.shapes) (void)hipFree(r->ds.shapes);
    if (r->ds.mats) (void)hipFree(r->ds.mats);
    if (r->ds.nodes) (void)hipFree(r->ds.nodes);
    if (r->ds.leaf) (void)hipFree(r->ds.leaf);
    if (r->ds.lin) (void)hipFree(r->ds.lin);
    if (r->ds.march) (void)hipFree(r->ds.march);
    if (r->ds.boxes) (void)hipFree(r->ds.boxes);
    if (r->ds.tex) (void)hipFree(r->ds.tex);
    if (r->ds.perlin) (void)hipFree(r->ds.perlin);
    if (r->ds.images) (void)hipFree(r->ds.images);
    if (r->ds.pixels) (void)hipFree(r->ds.pixels);
    if (r->stream) (void)hipStreamSynchronize(r->stream);
    wave_workspace_free(&r->ws);
    if (r->stream) (void)hipStreamDestroy(r->stream);
    delete r;
}

static FrameParams frame_params(const pt_renderer *r, const pt_camera &cam, uint32_t w, uint32_t h, uint32_t spp,
                                uint64_t seed) {
    FrameParams P;
    std::memset(&P, 0, sizeof P);
    caster_params(cam, w, h, &P);
    P.s11 = r->s11;
    P.seed = seed;
    P.width = w;
    P.height = h;
    P.spp = spp;
    P.depth = r->depth;
    P.rank = 0;
    P.world = 1;
    P.tiles_x = tiles_x_of(w);
    return P;
}

int pt_render_start(pt_renderer *r, const pt_camera *cam, uint32_t w, uint32_t h, uint32_t spp, uint64_t seed) {
    if (!r || !cam) return fail(PT_ERR_INVALID, "null argument");
    if (w == 0 || h == 0 || spp == 0) return fail(PT_ERR_INVALID, "width, height and samples_number must be > 0");
    HIP_TRY(hipSetDevice(r->device));
    if (r->started) {  // a new frame replaces the one in flight
        HIP_TRY(hipStreamSynchronize(r->stream));
        release_bands(r);
    }
    size_t bytes = (size_t)w * h * 3 * sizeof(double);
    if (bytes > r->frame_cap) {
        if (r->d_frame) HIP_TRY(hipFree(r->d_frame));
        r->d_frame = nullptr;
        r->frame_cap = 0;
        HIP_TRY(hipMalloc(&r->d_frame, bytes));
        r->frame_cap = bytes;
    }
    FrameParams P = frame_params(r, *cam, w, h, spp, seed);
    uint32_t ty = tiles_y_of(h);
    uint32_t band = ty >= 8 ? ty / 8 : 1;  // ~8 progressive bands per frame
    for (uint32_t t0 = 0; t0 < ty; t0 += band) {
        uint32_t t1 = t0 + band < ty ? t0 + band : ty;
        P.tile_begin = t0 * P.tiles_x;
        P.tile_count = (t1 - t0) * P.tiles_x;
        HIP_TRY(launch_render(r->ds, P, r->d_frame, r->stream, &r->ws));
        pt_renderer::Band b;
        b.row0 = t0 * TILE;
        b.row1 = t1 * TILE < h ? t1 * TILE : h;
        b.copied = false;
        HIP_TRY(hipEventCreateWithFlags(&b.ev, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(b.ev, r->stream));
        r->bands.push_back(b);
    }
    r->width = w;
    r->height = h;
    r->started = true;
    return PT_OK;
}

int pt_render_step(pt_renderer *r, double *rgb, int blocking) {
    if (!r || !rgb) return fail(PT_ERR_INVALID, "null argument");
    if (!r->started) return fail(PT_ERR_STATE, "render_step before start_rendering");
    HIP_TRY(hipSetDevice(r->device));
    bool done = true;
    for (auto &b : r->bands) {
        if (b.copied) continue;
        if (blocking) {
            HIP_TRY(hipEventSynchronize(b.ev));
        } else {
            hipError_t q = hipEventQuery(b.ev);
            if (q == hipErrorNotReady) {
                (void)hipGetLastError();
                done = false;
                continue;
            }
            if (q != hipSuccess) return hip_fail(q, "hipEventQuery");
        }
        size_t off = (size_t)b.row0 * r->width * 3;
        size_t n = (size_t)(b.row1 - b.row0) * r->width * 3;
        HIP_TRY(hipMemcpy(rgb + off, r->d_frame + off, n * sizeof(double), hipMemcpyDeviceToHost));
        b.copied = true;
    }
    if (done) {
        release_bands(r);
        r->started = false;
        return 1;
    }
    return 0;
}

int pt_render_stop(pt_renderer *r) {
    if (!r) return fail(PT_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(r->device));
    HIP_TRY(hipStreamSynchronize(r->stream));
    release_bands(r);
    r->started = false;
    return PT_OK;
}

uint32_t pt_shard_tiles(uint32_t w, uint32_t h, uint32_t rank, uint32_t world) {
    if (world == 0 || rank >= world) return 0;
    uint32_t total = tiles_x_of(w) * tiles_y_of(h);
    return rank < total ? (total - rank + world - 1) / world : 0;
}

int pt_render_device(pt_renderer *r, const pt_camera *cam, uint32_t w, uint32_t h, uint32_t spp, uint64_t seed,
                     uint32_t rank, uint32_t world, double *d_out, void *stream) {
    if (!r || !cam || !d_out) return fail(PT_ERR_INVALID, "null argument");
    if (w == 0 || h == 0 || spp == 0) return fail(PT_ERR_INVALID, "width, height and samples_number must be > 0");
    if (world == 0 || rank >= world) return fail(PT_ERR_INVALID, "rank must be < world");
    HIP_TRY(hipSetDevice(r->device));
    FrameParams P = frame_params(r, *cam, w, h, spp, seed);
    P.rank = rank;
    P.world = world;
    P.compact = world > 1 ? 1 : 0;
    P.tile_begin = 0;
    P.tile_count = pt_shard_tiles(w, h, rank, world);
    // any HIP stream, 0 being the null stream as everywhere in HIP (pt_unshard_device
    // takes the same handle, so a caller's render -> gather -> unshard stays ordered)
    hipStream_t st = (hipStream_t)stream;
    HIP_TRY(launch_render(r->ds, P, d_out, st, &r->ws));
    return PT_OK;
}

int pt_unshard_device(const double *g, uint32_t w, uint32_t h, uint32_t world, double *frame, void *stream) {
    if (!g || !frame || world == 0) return fail(PT_ERR_INVALID, "bad argument");
    HIP_TRY(launch_unshard(g, w, h, world, frame, (hipStream_t)stream));
    return PT_OK;
}

// ---------------------------------------------------------------- probes

int pt_closest_hit(pt_renderer *r, const double *rays, size_t n, double min_t, double max_t, pt_hit *out) {
    if (!r || (n && (!rays || !out))) return fail(PT_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(r->device));
    DevBuf<double> dr;
    DevBuf<pt_hit> dh;
    HIP_TRY(dr.alloc(n * 6));
    HIP_TRY(dh.alloc(n));
    HIP_TRY(hipMemcpy(dr.p, rays, n * 6 * sizeof(double), hipMemcpyHostToDevice));
    HIP_TRY(launch_closest_hit(r->ds, dr.p, n, min_t, max_t, dh.p, r->stream));
    HIP_TRY(hipStreamSynchronize(r->stream));
    HIP_TRY(hipMemcpy(out, dh.p, n * sizeof(pt_hit), hipMemcpyDeviceToHost));
    return PT_OK;
}

int pt_ray_color(pt_renderer *r, const double *rays, uint64_t *states, size_t n, uint32_t depth, double *out) {
    if (!r || (n && (!rays || !states || !out))) return fail(PT_ERR_INVALID, "null argument");
    if (depth > 64) return fail(PT_ERR_UNSUPPORTED, "depth > 64 is not supported on the GPU path");
    HIP_TRY(hipSetDevice(r->device));
    DevBuf<double> dr, dout;
    DevBuf<uint64_t> ds;
    HIP_TRY(dr.alloc(n * 6));
    HIP_TRY(ds.alloc(n));
    HIP_TRY(dout.alloc(n * 3));
    HIP_TRY(hipMemcpy(dr.p, rays, n * 6 * sizeof(double), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(ds.p, states, n * sizeof(uint64_t), hipMemcpyHostToDevice));
    HIP_TRY(launch_ray_color(r->ds, dr.p, ds.p, n, depth, r->s11, dout.p, r->stream));
    HIP_TRY(hipStreamSynchronize(r->stream));
    HIP_TRY(hipMemcpy(out, dout.p, n * 3 * sizeof(double), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(states, ds.p, n * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return PT_OK;
}

int pt_trace_pixel_samples(pt_renderer *r, const pt_camera *cam, uint32_t w, uint32_t h, uint32_t spp, uint64_t seed,
                           const uint32_t *pixels, size_t n, double *out) {
    if (!r || !cam || (n && (!pixels || !out))) return fail(PT_ERR_INVALID, "null argument");
    if (w == 0 || h == 0 || spp == 0) return fail(PT_ERR_INVALID, "width, height and samples_number must be > 0");
    for (size_t i = 0; i < n; i++)
        if (pixels[i] >= (uint64_t)w * h) return fail(PT_ERR_INVALID, "pixel index out of range");
    HIP_TRY(hipSetDevice(r->device));
    FrameParams P = frame_params(r, *cam, w, h, spp, seed);
    DevBuf<uint32_t> dp;
    DevBuf<double> dout;
    HIP_TRY(dp.alloc(n));
    HIP_TRY(dout.alloc(n * 3));
    HIP_TRY(hipMemcpy(dp.p, pixels, n * sizeof(uint32_t), hipMemcpyHostToDevice));
    HIP_TRY(launch_trace_pixels(r->ds, P, dp.p, n, dout.p, r->stream));
    HIP_TRY(hipStreamSynchronize(r->stream));
    HIP_TRY(hipMemcpy(out, dout.p, n * 3 * sizeof(double), hipMemcpyDeviceToHost));
    return PT_OK;
}

int pt_count_work(pt_renderer *r, const pt_camera *cam, uint32_t w, uint32_t h, uint32_t spp, uint64_t seed,
                  const uint32_t *pixels, size_t n, uint64_t *counters) {
    static_assert(C_COUNT == PT_NUM_COUNTERS, "counter list matches the header");
    if (!r || !cam || !counters || (n && !pixels)) return fail(PT_ERR_INVALID, "null argument");
    if (w == 0 || h == 0 || spp == 0) return fail(PT_ERR_INVALID, "width, height and samples_number must be > 0");
    for (size_t i = 0; i < n; i++)
        if (pixels[i] >= (uint64_t)w * h) return fail(PT_ERR_INVALID, "pixel index out of range");
    HIP_TRY(hipSetDevice(r->device));
    FrameParams P = frame_params(r, *cam, w, h, spp, seed);
    DevBuf<uint32_t> dp;
    DevBuf<unsigned long long> dc;
    HIP_TRY(dp.alloc(n));
    HIP_TRY(dc.alloc(C_COUNT));
    HIP_TRY(hipMemcpy(dp.p, pixels, n * sizeof(uint32_t), hipMemcpyHostToDevice));
    HIP_TRY(hipMemsetAsync(dc.p, 0, C_COUNT * sizeof(unsigned long long), r->stream));
    HIP_TRY(launch_count_work(r->ds, P, dp.p, n, dc.p, r->stream));
    HIP_TRY(hipStreamSynchronize(r->stream));
    HIP_TRY(hipMemcpy(counters, dc.p, C_COUNT * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return PT_OK;
}

int pt_march_jobs(pt_renderer *r, const double *jobs, size_t n, double *t_out, int32_t *status, uint32_t *iters) {
    if (!r || (n && (!jobs || !t_out || !status || !iters))) return fail(PT_ERR_INVALID, "null argument");
    if (n == 0) return PT_OK;
    HIP_TRY(hipSetDevice(r->device));
    DevBuf<double> dj, dt;
    DevBuf<int32_t> ds;
    DevBuf<uint32_t> di;
    HIP_TRY(dj.alloc(n * 8));
    HIP_TRY(dt.alloc(n));
    HIP_TRY(ds.alloc(n));
    HIP_TRY(di.alloc(n));
    HIP_TRY(hipMemcpyAsync(dj.p, jobs, n * 8 * sizeof(double), hipMemcpyHostToDevice, r->stream));
    HIP_TRY(launch_march_probe(dj.p, n, dt.p, ds.p, di.p, r->stream));
    HIP_TRY(hipMemcpyAsync(t_out, dt.p, n * sizeof(double), hipMemcpyDeviceToHost, r->stream));
    HIP_TRY(hipMemcpyAsync(status, ds.p, n * sizeof(int32_t), hipMemcpyDeviceToHost, r->stream));
    HIP_TRY(hipMemcpyAsync(iters, di.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, r->stream));
    HIP_TRY(hipStreamSynchronize(r->stream));
    return PT_OK;
}

int pt_kernel_timing(pt_renderer *r, int enable, double *ms, uint32_t *launches, size_t nkinds) {
    if (!r) return fail(PT_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(r->device));
    double m[K_KINDS];
    uint32_t l[K_KINDS];
    HIP_TRY(timer_collect(r->ws.timer, m, l));
    for (size_t k = 0; k < nkinds && k < (size_t)K_KINDS; k++) {
        if (ms) ms[k] = m[k];
        if (launches) launches[k] = l[k];
    }
    if (enable && !r->ws.timer) r->ws.timer = timer_new();
    if (!enable && r->ws.timer) {
        timer_free(r->ws.timer);
        r->ws.timer = nullptr;
    }
    return PT_OK;
}

int pt_wave_diag(pt_renderer *r, int enable, uint64_t *out, size_t n) {
    if (!r) return fail(PT_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(r->device));
    HIP_TRY(hipStreamSynchronize(r->stream));
    if (out && n && r->ws.diag) HIP_TRY(hipMemcpy(out, r->ws.diag, (n < 40 ? n : 40) * 8, hipMemcpyDeviceToHost));
    if (enable && !r->ws.diag) HIP_TRY(hipMalloc(&r->ws.diag, 40 * 8));
    if (r->ws.diag) HIP_TRY(hipMemset(r->ws.diag, 0, 40 * 8));
    if (!enable && r->ws.diag) {
        HIP_TRY(hipFree(r->ws.diag));
        r->ws.diag = nullptr;
    }
    return PT_OK;
}

int pt_profile_phases(pt_renderer *r, const pt_camera *cam, uint32_t w, uint32_t h, uint32_t spp, uint64_t seed,
                      uint64_t *out) {
    if (!r || !cam || !out) return fail(PT_ERR_INVALID, "null argument");
    if (r->depth > 8) return fail(PT_ERR_UNSUPPORTED, "phase profiling supports depth <= 8");
    HIP_TRY(hipSetDevice(r->device));
    FrameParams P = frame_params(r, *cam, w, h, spp, seed);
    P.tile_count = pt_shard_tiles(w, h, 0, 1);
    DevBuf<double> frame;
    DevBuf<unsigned long long> acc;
    HIP_TRY(frame.alloc((size_t)w * h * 3));
    HIP_TRY(acc.alloc(10));
    HIP_TRY(hipMemsetAsync(acc.p, 0, 10 * sizeof(unsigned long long), r->stream));
    HIP_TRY(launch_render_timed(r->ds, P, frame.p, acc.p, r->stream));
    HIP_TRY(hipStreamSynchronize(r->stream));
    HIP_TRY(hipMemcpy(out, acc.p, 10 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return PT_OK;
}

// Display encode (src/bin/main.rs:281-289): f64::clamp keeps NaN, `as u8`
// saturates NaN to 0.
int pt_encode_rgba8(const double *rgb, size_t npix, uint8_t *rgba) {
    if (npix && (!rgb || !rgba)) return fail(PT_ERR_INVALID, "null argument");
    for (size_t i = 0; i < npix; i++) {
        for (int c = 0; c < 3; c++) {
            double v = std::sqrt(rgb[i * 3 + c]);
            if (v < 0.0) v = 0.0;
            if (v > 0.999) v = 0.999;
            double s = v * 256.0;
            rgba[i * 4 + c] = std::isnan(s) ? 0 : (uint8_t)s;
        }
        rgba[i * 4 + 3] = 255;
    }
    return PT_OK;
}

}  // extern "C"
