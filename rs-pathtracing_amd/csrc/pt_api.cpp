// pt_api.cpp — the C-ABI (include/rs_pathtracing.h).  No exception escapes:
// each entry point catches, stores a thread-local message and returns a
// status.  The renderer owns one HIP stream on its device; start_rendering
// queues the frame as bands of tile rows, each closed by an event, so a
// non-blocking render_step can hand back finished bands while the rest of the
// frame is still on the GPU (src/renderer/step_by_step.rs:101-121).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstddef>
#include <cstring>
#include <new>
#include <string>
#include <thread>
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
// the smallest band of a progressive frame, in samples (enough paths to fill the device)
constexpr uint64_t BAND_MIN_SAMPLES = (uint64_t)1 << 24;

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

// One device of a renderer: its own copy of the scene, wavefront workspace
// and stream.  A single-device renderer has one; a multi-device
// renderer (pt_renderer_create_multi) deals the frame's tiles to several,
// rank g = gpus[g], and gathers the shards on gpus[0].
struct GpuShare {
    int device = 0;
    hipStream_t stream = nullptr;
    DeviceScene ds;
    WaveWorkspace ws;
    double *d_shard = nullptr;  // compact tile shard of a multi-device frame (ranks >= 1)
    size_t shard_cap = 0;
    hipEvent_t shard_ev = nullptr;  // a band's shard copy to gpus[0] is done
};

struct pt_renderer {
    pt_scene *scene = nullptr;
    uint32_t depth = 0;
    double s11 = 0;
    std::vector<GpuShare> gpus;  // gpus[0] holds the frame

    // frame in flight (render_start .. render_step)
    bool started = false;
    uint32_t width = 0, height = 0;
    double *d_frame = nullptr;  // w*h*3 on gpus[0]
    size_t frame_cap = 0;
    uint8_t *d_rgba = nullptr;  // w*h*4 display encode of d_frame, on gpus[0]
    size_t rgba_cap = 0;
    double *d_gather = nullptr;  // multi-device: world shards back to back, on gpus[0]
    size_t gather_cap = 0;
    int peer_pairs = 0, peer_enabled = 0;  // distinct (gpus[0], gpus[k]) device pairs; with peer access both ways
    int fault_accel_alloc = 0;  // test hook (option "fault_accel_alloc"): this renderer's next BVH rebuild fails
    // A progressive frame is a list of bands of tile rows.  A feeder thread
    // queues them on the device(s), keeping two bands ahead of the GPU (one
    // running, one queued), so the device never idles between bands and
    // stop_rendering only has to drain at most two of them.
    struct Band {
        uint32_t t0, t1;      // tile rows
        uint32_t row0, row1;  // pixel rows
        hipEvent_t ev;        // recorded on gpus[0].stream once the band is queued
        bool copied;
    };
    std::vector<Band> bands;
    FrameParams frame{};
    std::thread feeder;
    std::atomic<bool> stop_req{false};
    std::atomic<uint32_t> bands_queued{0};  // bands [0, n) are queued (their events recorded)
    std::atomic<int> feed_rc{0};            // the feeder's failure status (feed_err holds the message)
    std::string feed_err;
    // The progressive frame's stop flag (FrameParams::stop), host-mapped and
    // coherent so the kernels see pt_render_stop's store at once: while it is
    // set, a queued launch of the frame does no work, so the stop returns
    // after the launches already running instead of two whole bands.  Frames
    // queued by pt_render_device / pt_render_frame_device carry no flag.
    int *h_stop = nullptr;
    const int *d_stop = nullptr;

    int device() const { return gpus[0].device; }
    hipStream_t stream() const { return gpus[0].stream; }
};

extern "C" {

const char *pt_last_error(void) { return g_err.c_str(); }
__attribute__((visibility("hidden"))) void pt_set_last_error(const char *msg) { g_err = msg ? msg : ""; }  // for pt_image.cpp
#ifndef PT_SRC_SHA
#define PT_SRC_SHA "unknown"
#endif
const char *pt_version(void) {
    return "rs-pathtracing-amd 0.4.2 (gfx950, f64 megakernel + wavefront march engine; src " PT_SRC_SHA ")";
}
uint32_t pt_abi_version(void) { return PT_ABI_VERSION; }

int pt_abi_layout(int which, uint32_t *out, size_t n) {
    std::vector<size_t> v;
#define PT_F(T, f) v.push_back(offsetof(T, f))
    switch (which) {
    case PT_ABI_SCENE_OPTS:
        v.push_back(sizeof(pt_scene_opts));
        PT_F(pt_scene_opts, random_spheres), PT_F(pt_scene_opts, struct_size), PT_F(pt_scene_opts, seed);
        PT_F(pt_scene_opts, load_image), PT_F(pt_scene_opts, image_user);
        break;
    case PT_ABI_CAMERA:
        v.push_back(sizeof(pt_camera));
        PT_F(pt_camera, position), PT_F(pt_camera, direction), PT_F(pt_camera, up), PT_F(pt_camera, right);
        PT_F(pt_camera, fov), PT_F(pt_camera, focal_length);
        break;
    case PT_ABI_SHAPE_INFO:
        v.push_back(sizeof(pt_shape_info));
        PT_F(pt_shape_info, type), PT_F(pt_shape_info, material), PT_F(pt_shape_info, inverse_normal);
        PT_F(pt_shape_info, depth), PT_F(pt_shape_info, func), PT_F(pt_shape_info, pad0);
        PT_F(pt_shape_info, direct), PT_F(pt_shape_info, inverse);
        PT_F(pt_shape_info, x0), PT_F(pt_shape_info, y0), PT_F(pt_shape_info, x1), PT_F(pt_shape_info, y1);
        PT_F(pt_shape_info, step), PT_F(pt_shape_info, a), PT_F(pt_shape_info, b), PT_F(pt_shape_info, c);
        PT_F(pt_shape_info, d), PT_F(pt_shape_info, sphere_radius), PT_F(pt_shape_info, radius);
        PT_F(pt_shape_info, tube_radius);
        break;
    case PT_ABI_MATERIAL_INFO:
        v.push_back(sizeof(pt_material_info));
        PT_F(pt_material_info, type), PT_F(pt_material_info, texture), PT_F(pt_material_info, albedo);
        PT_F(pt_material_info, fuzz), PT_F(pt_material_info, ior), PT_F(pt_material_info, emit);
        break;
    case PT_ABI_HIT:
        v.push_back(sizeof(pt_hit));
        PT_F(pt_hit, t), PT_F(pt_hit, point), PT_F(pt_hit, normal), PT_F(pt_hit, front_face);
        PT_F(pt_hit, shape), PT_F(pt_hit, material), PT_F(pt_hit, pad0);
        break;
    case PT_ABI_CHECKPOINT:
        v.push_back(sizeof(pt_checkpoint));
        PT_F(pt_checkpoint, width), PT_F(pt_checkpoint, height), PT_F(pt_checkpoint, samples_number);
        PT_F(pt_checkpoint, samples_done), PT_F(pt_checkpoint, rank), PT_F(pt_checkpoint, world);
        PT_F(pt_checkpoint, depth), PT_F(pt_checkpoint, reserved), PT_F(pt_checkpoint, seed);
        PT_F(pt_checkpoint, scene_key), PT_F(pt_checkpoint, count);
        break;
    default:
        return fail(PT_ERR_INVALID, "pt_abi_layout: unknown struct " + std::to_string(which));
    }
#undef PT_F
    if (n && !out) return fail(PT_ERR_INVALID, "null argument");
    for (size_t k = 0; k < n && k < v.size(); k++) out[k] = (uint32_t)v[k];
    return (int)v.size();
}

uint64_t pt_sample_key(uint64_t seed, uint64_t pixel, uint64_t sample) { return sample_key(seed, pixel, sample); }

int pt_scene_create_from_json(const char *json, size_t len, const pt_scene_opts *opts, pt_scene **out) {
    if (!json || !out) return fail(PT_ERR_INVALID, "null argument");
    *out = nullptr;
    // struct_size versions the options (header): no byte at or past
    // opts + struct_size is read; 0 is a 0.1.0 (16-byte struct) or 0.2.0
    // (32-byte) caller with `reserved` = 0 in this field, which 0 cannot tell
    // apart, so only the 16 bytes both have are read (no image loader)
    const size_t osz = !opts ? 0 : (opts->struct_size ? opts->struct_size : (size_t)PT_SCENE_OPTS_LEGACY_SIZE);
    if (opts && osz < PT_SCENE_OPTS_MIN_SIZE)
        return fail(PT_ERR_INVALID, "pt_scene_opts.struct_size " + std::to_string(osz) +
                                        " is below the 16 bytes of {random_spheres, struct_size, seed}");
    bool rs = opts ? opts->random_spheres != 0 : true;
    uint64_t seed = opts ? opts->seed : 1;
    ImageSource img;
    if (opts && osz >= offsetof(pt_scene_opts, load_image) + sizeof(opts->load_image)) img.load = opts->load_image;
    if (opts && osz >= offsetof(pt_scene_opts, image_user) + sizeof(opts->image_user)) img.user = opts->image_user;
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
}  // extern "C"

namespace {

void free_share(GpuShare &g) {
    (void)hipSetDevice(g.device);
    if (g.stream) (void)hipStreamSynchronize(g.stream);
    DeviceScene &d = g.ds;
    void *bufs[] = {d.shapes, d.mats, d.nodes, d.qnodes, d.leaf, d.lin, d.march, d.boxes, d.tex, d.perlin,
                    d.images, d.pixels, d.guard};
    for (void *p : bufs)
        if (p) (void)hipFree(p);
    d = DeviceScene{};
    if (g.d_shard) (void)hipFree(g.d_shard);
    g.d_shard = nullptr;
    g.shard_cap = 0;
    wave_workspace_free(&g.ws);
    if (g.shard_ev) (void)hipEventDestroy(g.shard_ev);
    g.shard_ev = nullptr;
    if (g.stream) (void)hipStreamDestroy(g.stream);
    g.stream = nullptr;
}

// The acceleration structure on one device: octant-threaded BVH nodes, leaf
// shape ids, the wave-uniform and marched lists and the padded boxes.  A new
// structure is first staged in buffers of its own (stage_accel); only when
// every device has staged it are the old buffers swapped out and freed
// (commit_accel), so a failed upload leaves every device on its old, complete
// structure.
struct StagedAccel {
    DNodeC *nodes = nullptr;
    DQGrid *qnodes = nullptr;
    int32_t *leaf = nullptr, *lin = nullptr, *march = nullptr;
    DBox *boxes = nullptr;
    int nnodes = 0, nlin = 0, nmarch = 0;
    float bvh_bound = 0.f;
};

// Test hook (renderer option "fault_accel_alloc" = n, kept per renderer): the
// n-th device allocation of that renderer's next BVH rebuild fails as if the
// device were out of memory.  `fault` is the renderer's counter (null when
// creating a renderer: no hook).

void free_staged(int device, StagedAccel &a) {
    (void)hipSetDevice(device);
    void *bufs[] = {a.nodes, a.qnodes, a.leaf, a.lin, a.march, a.boxes};
    for (void *p : bufs)
        if (p) (void)hipFree(p);
    a = StagedAccel{};
}

int stage_accel(int device, const Accel &acc, StagedAccel *out, int *fault = nullptr) {
    StagedAccel a;
    hipError_t err = hipSetDevice(device);
    auto upload = [&err, fault](auto **dst, const auto &vec) {
        using T = typename std::remove_reference<decltype(vec)>::type::value_type;
        size_t n = vec.empty() ? 1 : vec.size();
        if (err == hipSuccess && fault && *fault > 0 && (*fault)-- == 1) err = hipErrorOutOfMemory;
        if (err == hipSuccess) err = hipMalloc((void **)dst, n * sizeof(T));
        if (err == hipSuccess && !vec.empty())
            err = hipMemcpy(*dst, vec.data(), vec.size() * sizeof(T), hipMemcpyHostToDevice);
    };
    upload(&a.nodes, acc.cnodes);
    upload(&a.leaf, acc.leaf);
    upload(&a.lin, acc.lin);
    upload(&a.march, acc.march);
    upload(&a.boxes, acc.boxes);
    if (err == hipSuccess && !acc.qnodes.empty()) {  // the grid, then the quantized layouts
        DQGrid g{};
        for (int k = 0; k < 3; k++) g.g0[k] = acc.qg0[k], g.gs[k] = acc.qgs[k];
        g.bound = acc.qbound;
        const size_t nb = acc.qnodes.size() * sizeof(DNodeQ);
        if (fault && *fault > 0 && (*fault)-- == 1) err = hipErrorOutOfMemory;
        // (one node of padding past the last layout, then the one-shape leaves' records: qleaf_offset)
        const size_t ro = qleaf_offset(acc.nodes_per_octant()), rb = acc.qleaves.size() * sizeof(DLeafRec);
        if (err == hipSuccess) err = hipMalloc((void **)&a.qnodes, ro + rb);
        if (err == hipSuccess) err = hipMemset((char *)(a.qnodes + 1) + nb, 0, sizeof(DNodeQ));
        if (err == hipSuccess) err = hipMemcpy(a.qnodes, &g, sizeof g, hipMemcpyHostToDevice);
        if (err == hipSuccess) err = hipMemcpy(a.qnodes + 1, acc.qnodes.data(), nb, hipMemcpyHostToDevice);
        if (err == hipSuccess && rb)
            err = hipMemcpy((char *)a.qnodes + ro, acc.qleaves.data(), rb, hipMemcpyHostToDevice);
    }
    if (err != hipSuccess) {
        free_staged(device, a);
        return hip_fail(err, "uploading the acceleration structure");
    }
    a.nnodes = acc.nodes_per_octant();  // nodes per octant layout
    a.nlin = (int)acc.lin.size();
    a.nmarch = (int)acc.march.size();
    a.bvh_bound = acc.bvh_bound;
    *out = a;
    return PT_OK;
}

// Swaps a staged structure in; the old one is freed once the device's queued
// work (which may still read it) is done.
int commit_accel(GpuShare &g, StagedAccel &a) {
    HIP_TRY(hipSetDevice(g.device));
    HIP_TRY(hipDeviceSynchronize());
    DeviceScene &d = g.ds;
    StagedAccel old{d.nodes, d.qnodes, d.leaf, d.lin, d.march, d.boxes, d.nnodes, d.nlin, d.nmarch, d.bvh_bound};
    d.nodes = a.nodes;
    d.qnodes = a.qnodes;
    d.leaf = a.leaf;
    d.lin = a.lin;
    d.march = a.march;
    d.boxes = a.boxes;
    d.nnodes = a.nnodes;
    d.nlin = a.nlin;
    d.nmarch = a.nmarch;
    d.bvh_bound = a.bvh_bound;
    a = StagedAccel{};
    free_staged(g.device, old);
    return PT_OK;
}

// Uploads the realized scene to one device and creates its stream.
int init_share(GpuShare &g, int device, const Scene &S, const Accel &acc, const std::vector<DShape> &hs,
               const std::vector<DMaterial> &hm) {
    g.device = device;
    HIP_TRY(hipSetDevice(device));
    hipError_t err = hipStreamCreateWithFlags(&g.stream, hipStreamNonBlocking);
    auto upload = [&err](auto **dst, const auto &vec) {
        using T = typename std::remove_reference<decltype(vec)>::type::value_type;
        size_t n = vec.empty() ? 1 : vec.size();
        if (err == hipSuccess) err = hipMalloc((void **)dst, n * sizeof(T));
        if (err == hipSuccess && !vec.empty())
            err = hipMemcpy(*dst, vec.data(), vec.size() * sizeof(T), hipMemcpyHostToDevice);
    };
    upload(&g.ds.shapes, hs);
    upload(&g.ds.mats, hm);
    if (!S.textures.empty()) {
        upload(&g.ds.tex, S.textures);
        upload(&g.ds.perlin, S.perlins);
        upload(&g.ds.images, S.images);
        upload(&g.ds.pixels, S.pixels);
    }
    if (err == hipSuccess) err = hipEventCreateWithFlags(&g.shard_ev, hipEventDisableTiming);
    // device counters: [0] march guard drops, [1] stop-gated launches that found the frame stopped, [2] of those,
    // launches that still had work (pt_render_stop_stats)
    if (err == hipSuccess) err = hipMalloc((void **)&g.ds.guard, 4 * sizeof(unsigned long long));
    if (err == hipSuccess) err = hipMemset(g.ds.guard, 0, 4 * sizeof(unsigned long long));
    if (err != hipSuccess) return hip_fail(err, "uploading the scene");
    StagedAccel a;
    if (int rc = stage_accel(device, acc, &a)) return rc;
    if (int rc = commit_accel(g, a)) return rc;
    g.ws.tune = tuning_defaults();
    g.ds.diag = g.ws.tune.diag;
    g.ds.nshapes = (int)hs.size();
    g.ds.nmats = (int)hm.size();
    g.ds.ext = S.textures.empty() ? 0 : 1;
    for (const auto &h : S.shapes)
        if (h.type == TORUS) g.ds.ext = 1;
    g.ds.fkind = 0;  // Heart-only kernel builds unless another function is marched
    for (const auto &h : S.shapes)
        if (h.type == MARCH && h.func != 0) g.ds.fkind = -1;
    return PT_OK;
}

void release_bands(pt_renderer *r) {
    for (auto &b : r->bands) (void)hipEventDestroy(b.ev);
    r->bands.clear();
}

int sync_all(pt_renderer *r) {
    for (auto &g : r->gpus) {
        HIP_TRY(hipSetDevice(g.device));
        HIP_TRY(hipStreamSynchronize(g.stream));
    }
    return PT_OK;
}

FrameParams frame_params(const pt_renderer *r, const pt_camera &cam, uint32_t w, uint32_t h, uint32_t spp,
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

// The part [*i0, *i1) of rank's tile list whose logical tiles lie in [a, b):
// logical tile k belongs to rank k % world at list index k / world.
void rank_range(uint32_t a, uint32_t b, uint32_t rank, uint32_t world, uint32_t *i0, uint32_t *i1) {
    *i0 = a > rank ? (a - rank + world - 1) / world : 0;
    *i1 = b > rank ? (b - rank + world - 1) / world : 0;
}

template <class T>
int grow(T **p, size_t *cap, size_t n) {
    const size_t bytes = n * sizeof(T);
    if (bytes <= *cap) return PT_OK;
    if (*p) HIP_TRY(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    HIP_TRY(hipMalloc((void **)p, bytes));
    *cap = bytes;
    return PT_OK;
}

// Buffers of a frame on the renderer's devices (world > 1: the shards and the
// gather buffer), and the fork: the other devices' streams start after
// everything queued so far on gpus[0]'s stream.
int frame_prologue(pt_renderer *r, uint32_t w, uint32_t h) {
    const uint32_t world = (uint32_t)r->gpus.size();
    if (world == 1) return PT_OK;
    GpuShare &g0 = r->gpus[0];
    const size_t per = pt_shard_tiles(w, h, 0, world);
    HIP_TRY(hipSetDevice(g0.device));
    if (int rc = grow(&r->d_gather, &r->gather_cap, (size_t)world * per * TILE * TILE * 3)) return rc;
    HIP_TRY(hipEventRecord(g0.shard_ev, g0.stream));
    for (uint32_t k = 1; k < world; k++) {
        GpuShare &g = r->gpus[k];
        HIP_TRY(hipSetDevice(g.device));
        if (int rc = grow(&g.d_shard, &g.shard_cap, per * TILE * TILE * 3)) return rc;
        HIP_TRY(hipStreamWaitEvent(g.stream, g0.shard_ev, 0));
    }
    return PT_OK;
}

// Queues tile rows [t0, t1) of the frame: every device renders its tiles of
// the band (world > 1: into its compact shard, then copied to gpus[0] over
// the peer link), gpus[0] un-interleaves the band into d_frame, encodes it
// into d_rgba (if given) and records `ev` (if given).
int enqueue_band(pt_renderer *r, const FrameParams &P0, double *d_frame, uint8_t *d_rgba, uint32_t t0, uint32_t t1,
                 hipEvent_t ev) {
    const uint32_t world = (uint32_t)r->gpus.size();
    const uint32_t w = P0.width, h = P0.height, tx = P0.tiles_x;
    GpuShare &g0 = r->gpus[0];
    const size_t per = pt_shard_tiles(w, h, 0, world);
    const uint32_t row0 = t0 * TILE, row1 = t1 * TILE < h ? t1 * TILE : h;
    for (uint32_t k = 0; k < world; k++) {
        GpuShare &g = r->gpus[k];
        HIP_TRY(hipSetDevice(g.device));
        FrameParams P = P0;
        P.rank = k;
        P.world = world;
        P.compact = world > 1 ? 1 : 0;
        uint32_t i0, i1;
        rank_range(t0 * tx, t1 * tx, k, world, &i0, &i1);
        P.tile_begin = i0;
        P.tile_count = i1 - i0;
        double *dst = world == 1 ? d_frame : (k == 0 ? r->d_gather : g.d_shard);
        HIP_TRY(launch_render(g.ds, P, dst, g.stream, &g.ws));
        if (k > 0) {
            if (i1 > i0) {
                const size_t off = (size_t)i0 * TILE * TILE * 3, n = (size_t)(i1 - i0) * TILE * TILE * 3;
                HIP_TRY(hipMemcpyPeerAsync(r->d_gather + (size_t)k * per * TILE * TILE * 3 + off, g0.device,
                                           g.d_shard + off, g.device, n * sizeof(double), g.stream));
            }
            HIP_TRY(hipEventRecord(g.shard_ev, g.stream));
            HIP_TRY(hipSetDevice(g0.device));
            HIP_TRY(hipStreamWaitEvent(g0.stream, g.shard_ev, 0));
        }
    }
    HIP_TRY(hipSetDevice(g0.device));
    if (world > 1) HIP_TRY(launch_unshard(r->d_gather, w, h, world, d_frame, g0.stream, row0, row1));
    if (d_rgba) HIP_TRY(launch_encode_rgba8(d_frame, (size_t)row0 * w, (size_t)row1 * w, d_rgba, g0.stream));
    if (ev) HIP_TRY(hipEventRecord(ev, g0.stream));
    return PT_OK;
}

// The feeder thread of a progressive frame: queues band b once band b - 2 is
// done, until the frame is queued or stop_rendering asks it to stop.
void feed_bands(pt_renderer *r) {
    const size_t n = r->bands.size();
    for (size_t b = 0; b < n; b++) {
        if (r->stop_req.load()) return;
        if (b >= 2) {
            (void)hipSetDevice(r->device());
            hipError_t e = hipEventSynchronize(r->bands[b - 2].ev);
            if (e != hipSuccess) {
                r->feed_err = std::string("hipEventSynchronize: ") + hipGetErrorString(e);
                r->feed_rc.store(PT_ERR_HIP);
                return;
            }
            if (r->stop_req.load()) return;
        }
        const auto &B = r->bands[b];
        if (int rc = enqueue_band(r, r->frame, r->d_frame, r->d_rgba, B.t0, B.t1, B.ev)) {
            r->feed_err = g_err;  // this thread's message
            r->feed_rc.store(rc);
            return;
        }
        r->bands_queued.store((uint32_t)(b + 1));
    }
}

void join_feeder(pt_renderer *r) {
    if (r->feeder.joinable()) r->feeder.join();
}

// Peer access between gpus[0] (which holds the frame) and every other distinct
// device, both ways, so hipMemcpyPeerAsync of a shard goes device to device
// over xGMI instead of staging through the host.  A pair the hardware cannot
// reach stays on the staged copy (still correct).
int enable_peers(pt_renderer *r) {
    const int d0 = r->gpus[0].device;
    std::vector<int> seen;
    for (size_t k = 1; k < r->gpus.size(); k++) {
        const int dk = r->gpus[k].device;
        if (dk == d0 || std::find(seen.begin(), seen.end(), dk) != seen.end()) continue;
        seen.push_back(dk);
        r->peer_pairs++;
        int a = 0, b = 0;
        HIP_TRY(hipDeviceCanAccessPeer(&a, dk, d0));
        HIP_TRY(hipDeviceCanAccessPeer(&b, d0, dk));
        if (!a || !b) continue;
        bool ok = true;
        for (int way = 0; way < 2; way++) {
            HIP_TRY(hipSetDevice(way == 0 ? dk : d0));
            const hipError_t e = hipDeviceEnablePeerAccess(way == 0 ? d0 : dk, 0);
            // "already enabled" is success; any other error leaves this pair on the staged
            // hipMemcpyPeerAsync (still correct): clear the error and carry on
            if (e != hipSuccess) (void)hipGetLastError();
            ok = ok && (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled);
        }
        if (ok) r->peer_enabled++;
    }
    return PT_OK;
}

int create_renderer(pt_scene *scene, const std::vector<int> &devices, uint32_t depth, pt_renderer **out) {
    *out = nullptr;
    if (depth > 64) return fail(PT_ERR_UNSUPPORTED, "depth > 64 is not supported on the GPU path");
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count == 0) return fail(PT_ERR_HIP, "no HIP device available (the GPU path has no CPU fallback)");
    for (int d : devices)
        if (d < 0 || d >= count) return fail(PT_ERR_INVALID, "device ordinal out of range");
    pt_renderer *r = new (std::nothrow) pt_renderer;
    if (!r) return fail(PT_ERR_INVALID, "out of memory");
    r->scene = scene;
    r->depth = depth;
    r->s11 = uniform_incl_scale(-1.0, 1.0);
    try {
        std::vector<DShape> hs;
        std::vector<DMaterial> hm;
        for (auto &s : scene->s.shapes) hs.push_back(to_device(s));
        for (auto &m : scene->s.materials) hm.push_back(to_device(m));
        if (hm.empty()) hm.push_back(DMaterial{});
        const Accel acc = build_accel(scene->s, scene->s.json_shapes, tuning_defaults().bvh_leaf);
        r->gpus.resize(devices.size());
        for (size_t k = 0; k < devices.size(); k++) {
            if (int rc = init_share(r->gpus[k], devices[k], scene->s, acc, hs, hm)) {
                pt_renderer_destroy(r);
                return rc;
            }
        }
    } catch (const std::bad_alloc &) {
        pt_renderer_destroy(r);
        return fail(PT_ERR_INVALID, "out of memory");
    }
    if (int rc = enable_peers(r)) {
        pt_renderer_destroy(r);
        return rc;
    }
    (void)hipSetDevice(devices[0]);
    {
        void *dp = nullptr;
        hipError_t e = hipHostMalloc((void **)&r->h_stop, sizeof(int),
                                     hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess) {
            __atomic_store_n(r->h_stop, 0, __ATOMIC_SEQ_CST);
            e = hipHostGetDevicePointer(&dp, r->h_stop, 0);
        }
        if (e != hipSuccess) {
            pt_renderer_destroy(r);
            return hip_fail(e, "allocating the stop flag");
        }
        r->d_stop = (const int *)dp;
    }
    *out = r;
    return PT_OK;
}

}  // namespace

extern "C" {

int pt_renderer_create(pt_scene *scene, int device, uint32_t depth, pt_renderer **out) {
    if (!scene || !out) return fail(PT_ERR_INVALID, "null argument");
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
        return fail(PT_ERR_HIP, "no HIP device available (the GPU path has no CPU fallback)");
    if (device < 0) HIP_TRY(hipGetDevice(&device));
    return create_renderer(scene, {device}, depth, out);
}

int pt_renderer_create_multi(pt_scene *scene, const int *devices, int ngpu, uint32_t depth, pt_renderer **out) {
    if (!scene || !out) return fail(PT_ERR_INVALID, "null argument");
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
        return fail(PT_ERR_HIP, "no HIP device available (the GPU path has no CPU fallback)");
    if (ngpu <= 0) {
        if (devices) return fail(PT_ERR_INVALID, "ngpu must be > 0 when devices are listed");
        ngpu = count;
    }
    std::vector<int> dv((size_t)ngpu);
    for (int k = 0; k < ngpu; k++) dv[k] = devices ? devices[k] : k;
    return create_renderer(scene, dv, depth, out);
}

int pt_renderer_set_option(pt_renderer *r, const char *name, int64_t value) {
    if (!r || !name) return fail(PT_ERR_INVALID, "null argument");
    if (r->started) return fail(PT_ERR_STATE, "options cannot change while a frame is in flight");
    if (!std::strcmp(name, "bvh_leaf") && value != r->gpus[0].ws.tune.bvh_leaf) {
        // the BVH is rebuilt with the new leaf size on every device
        Tuning t = r->gpus[0].ws.tune;
        if (tuning_set(&t, name, value) != PT_OK)
            return fail(PT_ERR_INVALID, "bvh_leaf out of range (1..16): " + std::to_string((long long)value));
        std::vector<StagedAccel> staged(r->gpus.size());
        auto drop = [&] {
            for (size_t k = 0; k < staged.size(); k++) free_staged(r->gpus[k].device, staged[k]);
        };
        try {
            const Accel acc = build_accel(r->scene->s, r->scene->s.json_shapes, t.bvh_leaf);
            // every device stages the new tree before any device lets go of the old one
            for (size_t k = 0; k < r->gpus.size(); k++)
                if (int rc = stage_accel(r->gpus[k].device, acc, &staged[k], &r->fault_accel_alloc)) {
                    drop();
                    return rc;
                }
        } catch (const std::exception &e) {
            drop();
            return fail(PT_ERR_INVALID, std::string("rebuilding the BVH: ") + e.what());
        }
        for (size_t k = 0; k < r->gpus.size(); k++)
            if (int rc = commit_accel(r->gpus[k], staged[k])) {
                drop();  // the devices before k run the new tree, k and after the old one: both complete
                return rc;
            }
    }
    if (!std::strcmp(name, "fault_accel_alloc")) {  // test hook of this renderer, see stage_accel
        if (value < 0 || value > 64) return fail(PT_ERR_INVALID, "fault_accel_alloc out of range (0..64)");
        r->fault_accel_alloc = (int)value;
        return PT_OK;
    }
    for (auto &g : r->gpus) {
        Tuning t = g.ws.tune;
        if (tuning_set(&t, name, value) != PT_OK)
            return fail(PT_ERR_INVALID, std::string("unknown option or value out of range: ") + name + " = " +
                                            std::to_string((long long)value));
        // the workspace may be in use by a frame queued on any stream
        HIP_TRY(hipSetDevice(g.device));
        HIP_TRY(hipDeviceSynchronize());
        g.ws.tune = t;
        g.ds.diag = t.diag;
    }
    return PT_OK;
}

int pt_renderer_get_option(const pt_renderer *r, const char *name, int64_t *value) {
    if (!r || !name || !value) return fail(PT_ERR_INVALID, "null argument");
    if (!std::strcmp(name, "bvh_nodes")) {  // read-only state
        *value = r->gpus[0].ds.nnodes;
        return PT_OK;
    }
    if (tuning_get(r->gpus[0].ws.tune, name, value) != PT_OK) return fail(PT_ERR_INVALID, std::string("unknown option: ") + name);
    return PT_OK;
}

const char *pt_option_name(int index) {
    int n = 0;
    while (TUNING_NAMES[n]) n++;
    return index >= 0 && index < n ? TUNING_NAMES[index] : nullptr;
}

int pt_renderer_peer_access(const pt_renderer *r, int *pairs, int *enabled) {
    if (!r) return fail(PT_ERR_INVALID, "null renderer");
    if (pairs) *pairs = r->peer_pairs;
    if (enabled) *enabled = r->peer_enabled;
    return PT_OK;
}

int pt_renderer_num_devices(const pt_renderer *r) { return r ? (int)r->gpus.size() : fail(PT_ERR_INVALID, "null renderer"); }

void pt_renderer_destroy(pt_renderer *r) {
    if (!r) return;
    if (r->started) (void)pt_render_stop(r);
    join_feeder(r);
    (void)sync_all(r);
    release_bands(r);
    if (!r->gpus.empty()) {
        (void)hipSetDevice(r->device());
        if (r->d_frame) (void)hipFree(r->d_frame);
        if (r->d_rgba) (void)hipFree(r->d_rgba);
        if (r->d_gather) (void)hipFree(r->d_gather);
    }
    for (auto &g : r->gpus) free_share(g);
    if (r->h_stop) (void)hipHostFree(r->h_stop);
    delete r;
}

int pt_render_start(pt_renderer *r, const pt_camera *cam, uint32_t w, uint32_t h, uint32_t spp, uint64_t seed) {
    if (!r || !cam) return fail(PT_ERR_INVALID, "null argument");
    if (w == 0 || h == 0 || spp == 0) return fail(PT_ERR_INVALID, "width, height and samples_number must be > 0");
    if (r->started) {  // a new frame replaces the one in flight (the reference stops it first, main.rs:268)
        if (int rc = pt_render_stop(r)) return rc;
    }
    HIP_TRY(hipSetDevice(r->device()));
    if (int rc = grow(&r->d_frame, &r->frame_cap, (size_t)w * h * 3)) return rc;
    if (int rc = grow(&r->d_rgba, &r->rgba_cap, (size_t)w * h * 4)) return rc;
    if (int rc = frame_prologue(r, w, h)) return rc;
    r->frame = frame_params(r, *cam, w, h, spp, seed);
    r->frame.stop = r->d_stop;
    // ~8 bands of whole tile rows, each a pass of the engine over 1/8 of the frame, but no band under
    // BAND_MIN_SAMPLES: a band of the reference GUI's 1-spp preview at 1600x900 (main.rs:264) would otherwise be
    // 160k samples, a chain of ~260 launches that each find a few paths (a 78 ms frame, round 5).  The stop
    // latency does not depend on the band size (stop_gate runs at every chunk start and compaction).
    const uint32_t ty = tiles_y_of(h);
    const uint64_t row_samples = (uint64_t)tiles_x_of(w) * TILE * TILE * spp;
    const uint32_t min_rows = (uint32_t)((BAND_MIN_SAMPLES + row_samples - 1) / row_samples);
    uint32_t band = ty >= 8 ? ty / 8 : 1;
    if (band < min_rows) band = min_rows < ty ? min_rows : ty;
    release_bands(r);
    for (uint32_t t0 = 0; t0 < ty; t0 += band) {
        pt_renderer::Band b;
        b.t0 = t0;
        b.t1 = t0 + band < ty ? t0 + band : ty;
        b.row0 = t0 * TILE;
        b.row1 = b.t1 * TILE < h ? b.t1 * TILE : h;
        b.copied = false;
        hipError_t e = hipEventCreateWithFlags(&b.ev, hipEventDisableTiming);
        if (e != hipSuccess) {
            release_bands(r);
            return hip_fail(e, "hipEventCreateWithFlags");
        }
        r->bands.push_back(b);
    }
    r->width = w;
    r->height = h;
    r->stop_req.store(false);
    r->bands_queued.store(0);
    r->feed_rc.store(0);
    r->feed_err.clear();
    try {
        r->feeder = std::thread(feed_bands, r);
    } catch (const std::exception &ex) {
        release_bands(r);
        return fail(PT_ERR_INVALID, std::string("cannot start the band feeder: ") + ex.what());
    }
    r->started = true;
    return PT_OK;
}

// Renderer::render_step: copy every band finished since the last call into
// rgb (linear f64) and / or rgba (display encode); 1 once the frame is complete.
int pt_render_step_rgba8(pt_renderer *r, double *rgb, uint8_t *rgba, int blocking) {
    if (!r || (!rgb && !rgba)) return fail(PT_ERR_INVALID, "null argument");
    if (!r->started) return fail(PT_ERR_STATE, "render_step before start_rendering");
    HIP_TRY(hipSetDevice(r->device()));
    if (blocking) join_feeder(r);  // every band queued (or the feeder failed)
    if (r->feed_rc.load()) {
        join_feeder(r);
        const int rc = r->feed_rc.load();
        const std::string msg = r->feed_err;
        (void)pt_render_stop(r);
        return fail(rc, "queueing the frame: " + msg);
    }
    const uint32_t queued = r->bands_queued.load();
    bool done = true;
    for (uint32_t k = 0; k < r->bands.size(); k++) {
        auto &b = r->bands[k];
        if (b.copied) continue;
        if (k >= queued) {  // not queued yet (non-blocking only)
            done = false;
            continue;
        }
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
        const size_t p0 = (size_t)b.row0 * r->width, np = (size_t)(b.row1 - b.row0) * r->width;
        if (rgb) HIP_TRY(hipMemcpy(rgb + p0 * 3, r->d_frame + p0 * 3, np * 3 * sizeof(double), hipMemcpyDeviceToHost));
        if (rgba) HIP_TRY(hipMemcpy(rgba + p0 * 4, r->d_rgba + p0 * 4, np * 4, hipMemcpyDeviceToHost));
        b.copied = true;
    }
    if (done) {
        join_feeder(r);
        release_bands(r);
        r->started = false;
        return 1;
    }
    return 0;
}

int pt_render_step(pt_renderer *r, double *rgb, int blocking) {
    if (!r || !rgb) return fail(PT_ERR_INVALID, "null argument");
    return pt_render_step_rgba8(r, rgb, nullptr, blocking);
}

// Renderer::stop_rendering: the feeder queues no further band and the stop
// flag turns the frame's queued launches into no-ops, so the wait is for the
// launches already running; the flag is cleared once the streams are idle
// and the frame is forgotten.
int pt_render_stop(pt_renderer *r) {
    if (!r) return fail(PT_ERR_INVALID, "null argument");
    r->stop_req.store(true);
    const bool flag = r->started && r->h_stop;
    if (flag) __atomic_store_n(r->h_stop, 1, __ATOMIC_SEQ_CST);
    join_feeder(r);
    int rc = sync_all(r);
    if (flag) __atomic_store_n(r->h_stop, 0, __ATOMIC_SEQ_CST);
    release_bands(r);
    r->started = false;
    return rc;
}

uint32_t pt_shard_tiles(uint32_t w, uint32_t h, uint32_t rank, uint32_t world) {
    if (world == 0 || rank >= world) return 0;
    uint32_t total = tiles_x_of(w) * tiles_y_of(h);
    return rank < total ? (total - rank + world - 1) / world : 0;
}

int pt_render_device(pt_renderer *r, const pt_camera *cam, uint32_t w, uint32_t h, uint32_t spp, uint64_t seed,
                     uint32_t rank, uint32_t world, double *d_out, void *stream) {
    return pt_render_device_samples(r, cam, w, h, spp, seed, rank, world, 0, spp, d_out, stream);
}

int pt_render_device_samples(pt_renderer *r, const pt_camera *cam, uint32_t w, uint32_t h, uint32_t spp,
                             uint64_t seed, uint32_t rank, uint32_t world, uint32_t s_begin, uint32_t s_end,
                             double *d_out, void *stream) {
    if (!r || !cam || !d_out) return fail(PT_ERR_INVALID, "null argument");
    if (w == 0 || h == 0 || spp == 0) return fail(PT_ERR_INVALID, "width, height and samples_number must be > 0");
    if (world == 0 || rank >= world) return fail(PT_ERR_INVALID, "rank must be < world");
    if (s_begin >= s_end || s_end > spp)
        return fail(PT_ERR_INVALID, "sample window must satisfy 0 <= s_begin < s_end <= samples_number");
    if (r->started) return fail(PT_ERR_STATE, "a progressive frame is in flight (render_step it to the end or stop it)");
    GpuShare &g = r->gpus[0];
    HIP_TRY(hipSetDevice(g.device));
    FrameParams P = frame_params(r, *cam, w, h, spp, seed);
    P.rank = rank;
    P.world = world;
    P.compact = world > 1 ? 1 : 0;
    P.tile_begin = 0;
    P.tile_count = pt_shard_tiles(w, h, rank, world);
    P.s_begin = s_begin;
    P.s_end = s_end;
    // any HIP stream of the renderer's (first) device, 0 being the null stream
    // as everywhere in HIP (pt_unshard_device takes the same handle, so a
    // caller's render -> gather -> unshard stays ordered)
    HIP_TRY(launch_render(g.ds, P, d_out, (hipStream_t)stream, &g.ws));
    return PT_OK;
}

int pt_render_frame_device(pt_renderer *r, const pt_camera *cam, uint32_t w, uint32_t h, uint32_t spp, uint64_t seed,
                           double *d_frame, void *stream) {
    if (!r || !cam || !d_frame) return fail(PT_ERR_INVALID, "null argument");
    if (w == 0 || h == 0 || spp == 0) return fail(PT_ERR_INVALID, "width, height and samples_number must be > 0");
    if (r->started) return fail(PT_ERR_STATE, "a progressive frame is in flight (render_step it to the end or stop it)");
    GpuShare &g0 = r->gpus[0];
    HIP_TRY(hipSetDevice(g0.device));
    hipStream_t st = (hipStream_t)stream;
    // the frame runs on the renderer's streams, after everything queued on st;
    // st resumes when the frame is in d_frame
    HIP_TRY(hipEventRecord(g0.shard_ev, st));
    HIP_TRY(hipStreamWaitEvent(g0.stream, g0.shard_ev, 0));
    const FrameParams P = frame_params(r, *cam, w, h, spp, seed);
    if (int rc = frame_prologue(r, w, h)) return rc;
    if (int rc = enqueue_band(r, P, d_frame, nullptr, 0, tiles_y_of(h), nullptr)) return rc;
    HIP_TRY(hipSetDevice(g0.device));
    HIP_TRY(hipEventRecord(g0.shard_ev, g0.stream));
    HIP_TRY(hipStreamWaitEvent(st, g0.shard_ev, 0));
    return PT_OK;
}

int pt_unshard_device(int device, const double *g, uint32_t w, uint32_t h, uint32_t world, double *frame,
                      void *stream) {
    if (!g || !frame || world == 0) return fail(PT_ERR_INVALID, "bad argument");
    if (device >= 0) HIP_TRY(hipSetDevice(device));
    HIP_TRY(launch_unshard(g, w, h, world, frame, (hipStream_t)stream));
    return PT_OK;
}

int pt_encode_rgba8_device(int device, const double *d_rgb, size_t npix, uint8_t *d_rgba, void *stream) {
    if (npix && (!d_rgb || !d_rgba)) return fail(PT_ERR_INVALID, "null argument");
    if (((uintptr_t)d_rgba & 3u) != 0) return fail(PT_ERR_INVALID, "rgba must be 4-byte aligned");
    if (device >= 0) HIP_TRY(hipSetDevice(device));
    HIP_TRY(launch_encode_rgba8(d_rgb, 0, npix, d_rgba, (hipStream_t)stream));
    return PT_OK;
}

// ---------------------------------------------------------------- probes

int pt_closest_hit(pt_renderer *r, const double *rays, size_t n, double min_t, double max_t, pt_hit *out) {
    if (!r || (n && (!rays || !out))) return fail(PT_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(r->device()));
    DevBuf<double> dr;
    DevBuf<pt_hit> dh;
    HIP_TRY(dr.alloc(n * 6));
    HIP_TRY(dh.alloc(n));
    HIP_TRY(hipMemcpy(dr.p, rays, n * 6 * sizeof(double), hipMemcpyHostToDevice));
    HIP_TRY(launch_closest_hit(r->gpus[0].ds, dr.p, n, min_t, max_t, dh.p, r->stream()));
    HIP_TRY(hipStreamSynchronize(r->stream()));
    HIP_TRY(hipMemcpy(out, dh.p, n * sizeof(pt_hit), hipMemcpyDeviceToHost));
    return PT_OK;
}

int pt_ray_color(pt_renderer *r, const double *rays, uint64_t *states, size_t n, uint32_t depth, double *out) {
    if (!r || (n && (!rays || !states || !out))) return fail(PT_ERR_INVALID, "null argument");
    if (depth > 64) return fail(PT_ERR_UNSUPPORTED, "depth > 64 is not supported on the GPU path");
    HIP_TRY(hipSetDevice(r->device()));
    DevBuf<double> dr, dout;
    DevBuf<uint64_t> ds;
    HIP_TRY(dr.alloc(n * 6));
    HIP_TRY(ds.alloc(n));
    HIP_TRY(dout.alloc(n * 3));
    HIP_TRY(hipMemcpy(dr.p, rays, n * 6 * sizeof(double), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(ds.p, states, n * sizeof(uint64_t), hipMemcpyHostToDevice));
    HIP_TRY(launch_ray_color(r->gpus[0].ds, dr.p, ds.p, n, depth, r->s11, dout.p, r->stream()));
    HIP_TRY(hipStreamSynchronize(r->stream()));
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
    HIP_TRY(hipSetDevice(r->device()));
    FrameParams P = frame_params(r, *cam, w, h, spp, seed);
    DevBuf<uint32_t> dp;
    DevBuf<double> dout;
    HIP_TRY(dp.alloc(n));
    HIP_TRY(dout.alloc(n * 3));
    HIP_TRY(hipMemcpy(dp.p, pixels, n * sizeof(uint32_t), hipMemcpyHostToDevice));
    HIP_TRY(launch_trace_pixels(r->gpus[0].ds, P, dp.p, n, dout.p, r->stream()));
    HIP_TRY(hipStreamSynchronize(r->stream()));
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
    HIP_TRY(hipSetDevice(r->device()));
    FrameParams P = frame_params(r, *cam, w, h, spp, seed);
    DevBuf<uint32_t> dp;
    DevBuf<unsigned long long> dc;
    HIP_TRY(dp.alloc(n));
    HIP_TRY(dc.alloc(C_COUNT));
    HIP_TRY(hipMemcpy(dp.p, pixels, n * sizeof(uint32_t), hipMemcpyHostToDevice));
    HIP_TRY(hipMemsetAsync(dc.p, 0, C_COUNT * sizeof(unsigned long long), r->stream()));
    HIP_TRY(launch_count_work(r->gpus[0].ds, P, dp.p, n, dc.p, r->stream()));
    HIP_TRY(hipStreamSynchronize(r->stream()));
    HIP_TRY(hipMemcpy(counters, dc.p, C_COUNT * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return PT_OK;
}

int pt_march_jobs(pt_renderer *r, const double *jobs, size_t n, double *t_out, int32_t *status, uint32_t *iters) {
    if (!r || (n && (!jobs || !t_out || !status || !iters))) return fail(PT_ERR_INVALID, "null argument");
    if (n == 0) return PT_OK;
    HIP_TRY(hipSetDevice(r->device()));
    DevBuf<double> dj, dt;
    DevBuf<int32_t> ds;
    DevBuf<uint32_t> di;
    HIP_TRY(dj.alloc(n * 8));
    HIP_TRY(dt.alloc(n));
    HIP_TRY(ds.alloc(n));
    HIP_TRY(di.alloc(n));
    HIP_TRY(hipMemcpyAsync(dj.p, jobs, n * 8 * sizeof(double), hipMemcpyHostToDevice, r->stream()));
    HIP_TRY(launch_march_probe(dj.p, n, dt.p, ds.p, di.p, r->stream()));
    HIP_TRY(hipMemcpyAsync(t_out, dt.p, n * sizeof(double), hipMemcpyDeviceToHost, r->stream()));
    HIP_TRY(hipMemcpyAsync(status, ds.p, n * sizeof(int32_t), hipMemcpyDeviceToHost, r->stream()));
    HIP_TRY(hipMemcpyAsync(iters, di.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, r->stream()));
    HIP_TRY(hipStreamSynchronize(r->stream()));
    return PT_OK;
}

int pt_march_guard_drops(pt_renderer *r, uint64_t *count) {
    if (!r || !count) return fail(PT_ERR_INVALID, "null argument");
    if (r->started) return fail(PT_ERR_STATE, "a progressive frame is in flight (render_step it to the end or stop it)");
    uint64_t total = 0;
    for (auto &g : r->gpus) {
        HIP_TRY(hipSetDevice(g.device));
        HIP_TRY(hipDeviceSynchronize());  // frames on any stream of the device
        unsigned long long n = 0;
        HIP_TRY(hipMemcpy(&n, g.ds.guard, sizeof n, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemset(g.ds.guard, 0, sizeof n));
        total += n;
    }
    *count = total;
    return PT_OK;
}

int pt_render_stop_stats(pt_renderer *r, uint64_t *skipped, uint64_t *worked) {
    if (!r || !skipped || !worked) return fail(PT_ERR_INVALID, "null argument");
    if (r->started) return fail(PT_ERR_STATE, "a progressive frame is in flight (render_step it to the end or stop it)");
    uint64_t s = 0, w = 0;
    for (auto &g : r->gpus) {
        HIP_TRY(hipSetDevice(g.device));
        HIP_TRY(hipDeviceSynchronize());
        unsigned long long c[2] = {0, 0};
        HIP_TRY(hipMemcpy(c, g.ds.guard + 1, sizeof c, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemset(g.ds.guard + 1, 0, sizeof c));
        s += c[0];
        w += c[1];
    }
    *skipped = s;
    *worked = w;
    return PT_OK;
}

int pt_kernel_timing(pt_renderer *r, int enable, double *ms, uint32_t *launches, size_t nkinds) {
    if (!r) return fail(PT_ERR_INVALID, "null argument");
    // the band feeder pushes into the timer and may queue timed launches
    if (r->started) return fail(PT_ERR_STATE, "a progressive frame is in flight (render_step it to the end or stop it)");
    HIP_TRY(hipSetDevice(r->device()));
    double m[K_KINDS];
    uint32_t l[K_KINDS];
    HIP_TRY(timer_collect(r->gpus[0].ws.timer, m, l));
    for (size_t k = 0; k < nkinds && k < (size_t)K_KINDS; k++) {
        if (ms) ms[k] = m[k];
        if (launches) launches[k] = l[k];
    }
    if (enable && !r->gpus[0].ws.timer) r->gpus[0].ws.timer = timer_new();
    if (!enable && r->gpus[0].ws.timer) {
        timer_free(r->gpus[0].ws.timer);
        r->gpus[0].ws.timer = nullptr;
    }
    return PT_OK;
}

int pt_wave_diag(pt_renderer *r, int enable, uint64_t *out, size_t n) {
    if (!r) return fail(PT_ERR_INVALID, "null argument");
    // the band feeder may queue launches that use the diag buffer
    if (r->started) return fail(PT_ERR_STATE, "a progressive frame is in flight (render_step it to the end or stop it)");
    if (enable && !PT_WAVE_DIAG)
        return fail(PT_ERR_UNSUPPORTED, "wave diagnostics are compiled out of this build (make EXTRA=-DPT_WAVE_DIAG=1)");
    HIP_TRY(hipSetDevice(r->device()));
    HIP_TRY(hipStreamSynchronize(r->stream()));
    if (out && n && r->gpus[0].ws.diag) HIP_TRY(hipMemcpy(out, r->gpus[0].ws.diag, (n < 64 ? n : 64) * 8, hipMemcpyDeviceToHost));
    if (enable && !r->gpus[0].ws.diag) HIP_TRY(hipMalloc(&r->gpus[0].ws.diag, 64 * 8));
    if (r->gpus[0].ws.diag) HIP_TRY(hipMemset(r->gpus[0].ws.diag, 0, 64 * 8));
    if (!enable && r->gpus[0].ws.diag) {
        HIP_TRY(hipFree(r->gpus[0].ws.diag));
        r->gpus[0].ws.diag = nullptr;
    }
    return PT_OK;
}

int pt_profile_phases(pt_renderer *r, const pt_camera *cam, uint32_t w, uint32_t h, uint32_t spp, uint64_t seed,
                      uint64_t *out) {
    if (!r || !cam || !out) return fail(PT_ERR_INVALID, "null argument");
    if (r->depth > 8) return fail(PT_ERR_UNSUPPORTED, "phase profiling supports depth <= 8");
    HIP_TRY(hipSetDevice(r->device()));
    FrameParams P = frame_params(r, *cam, w, h, spp, seed);
    P.tile_count = pt_shard_tiles(w, h, 0, 1);
    DevBuf<double> frame;
    DevBuf<unsigned long long> acc;
    HIP_TRY(frame.alloc((size_t)w * h * 3));
    HIP_TRY(acc.alloc(10));
    HIP_TRY(hipMemsetAsync(acc.p, 0, 10 * sizeof(unsigned long long), r->stream()));
    HIP_TRY(launch_render_timed(r->gpus[0].ds, P, frame.p, acc.p, r->stream()));
    HIP_TRY(hipStreamSynchronize(r->stream()));
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
