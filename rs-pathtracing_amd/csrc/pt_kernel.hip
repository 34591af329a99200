// pt_kernel.hip — MI355X (gfx950) kernels of the sample path.
//
// render_tiles: the megakernel.  One workgroup = one 16x16 pixel tile,
// 4 wave64s of 8x8 pixels each (adjacent pixels share a wave, so primary rays
// and their first bounces stay coherent); one pixel per lane, its spp camera
// samples traced in order and summed in f64 in registers; one write of the
// per-pixel mean.  Tiles are dealt round-robin to ranks (tile k -> k % world)
// so multi-GPU shards balance the Heart-heavy region.
#include <hip/hip_runtime.h>

#include "pt_device.hpp"
#include "pt_kernel.hpp"

#include <cstdlib>
#include <cstring>

constexpr int DEFAULT_WAVES = 4;  // C5 (100k spheres, compact BVH): 2 waves 845-849, 3: 1044, 4: 1109 M samples/s

namespace pt {

using dev::Ray;
using dev::V3;

// WAVES = minimum waves per SIMD the register allocation must allow
// (__launch_bounds__' second argument): 2 -> <= 256 VGPRs, 3 -> <= 168, 4 -> <= 128, 5 -> <= 102.
template <int NW, int WAVES, int FK = march::F_ANY>
__global__ __launch_bounds__(256, WAVES) void render_tiles(dev::Scene sc, FrameParams P, double *__restrict__ out) {
    if (P.stop) {  // progressive frames: one read of the host-mapped stop flag per block
        __shared__ int halt;
        if (threadIdx.x == 0) {
            halt = dev::stopped(P.stop);
            if (halt) dev::note_stop(sc.guard, false);
        }
        __syncthreads();
        if (halt) return;
    }
    const uint32_t ti = P.tile_begin + blockIdx.x;  // index in this rank's tile list
    const uint32_t k = dev::tile_position(P.rank + ti * P.world, P.tiles_x, P.world);  // global tile id
    const uint32_t tx = k % P.tiles_x, ty = k / P.tiles_x;
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const uint32_t lx = ((w & 1u) << 3) | (l & 7u), ly = ((w >> 1) << 3) | (l >> 3);
    const uint32_t x = tx * TILE + lx, y = ty * TILE + ly;
    double *dst = P.compact ? out + ((size_t)ti * (TILE * TILE) + ly * TILE + lx) * 3
                            : out + ((size_t)y * P.width + x) * 3;
    if (x >= P.width || y >= P.height) {
        if (P.compact) dst[0] = dst[1] = dst[2] = 0.0;
        return;
    }
    V3 c = dev::trace_pixel<NW, false, false, FK>(sc, P, x, y);
    dst[0] = c.x;
    dst[1] = c.y;
    dst[2] = c.z;
}

// Rows [y0, y1) of the frame from the gathered rank shards (rank-major, each
// padded to per_rank tiles): 48 B moved per pixel, HBM-bound.
__global__ __launch_bounds__(256) void unshard(const double *__restrict__ g, uint32_t width, uint32_t y0, uint32_t y1,
                                               uint32_t world, uint32_t tiles_x, uint32_t per_rank,
                                               double *__restrict__ frame) {
    const size_t i = (size_t)y0 * width + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)y1 * width) return;
    uint32_t x = (uint32_t)(i % width), y = (uint32_t)(i / width);
    uint32_t k = dev::tile_logical((y / TILE) * tiles_x + x / TILE, tiles_x, world);
    uint32_t rank = k % world, ti = k / world;
    const double *s = g + (((size_t)rank * per_rank + ti) * (TILE * TILE) + (y % TILE) * TILE + x % TILE) * 3;
    frame[i * 3 + 0] = s[0];
    frame[i * 3 + 1] = s[1];
    frame[i * 3 + 2] = s[2];
}

// Display encode of the GUI loop (src/bin/main.rs:281-289, main_raylib.rs:239-247):
// per channel sqrt -> f64::clamp(0, 0.999) -> *256 -> `as u8`, alpha 255.
// f64::clamp passes NaN through and the saturating `as u8` cast maps NaN to 0
// (and anything >= 256 to 255, which the clamp already prevents).  One pixel
// per lane: 24 B read, 4 B written, HBM-bound.
__device__ __forceinline__ uint32_t encode_channel(double c) {
    double v = sqrt(c);
    v = v < 0.0 ? 0.0 : v;  // Rust's clamp: if self < min { min }; if self > max { max }
    v = v > 0.999 ? 0.999 : v;
    const double s = v * 256.0;
    return s != s ? 0u : (uint32_t)s;  // NaN -> 0; 0 <= s < 256 otherwise
}
__global__ __launch_bounds__(256) void encode_rgba8(const double *__restrict__ rgb, size_t p0, size_t p1,
                                                    uint32_t *__restrict__ rgba) {
    const size_t i = p0 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p1) return;
    const uint32_t r = encode_channel(rgb[i * 3 + 0]), g = encode_channel(rgb[i * 3 + 1]),
                   b = encode_channel(rgb[i * 3 + 2]);
    rgba[i] = r | (g << 8) | (b << 16) | (255u << 24);  // bytes R, G, B, A in memory order
}

__global__ __launch_bounds__(256) void closest_hit_probe(dev::Scene sc, const double *__restrict__ rays, size_t n, double min_t,
                                  double max_t, pt_hit *__restrict__ out) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Ray r;
    r.o = dev::v3(rays[i * 6 + 0], rays[i * 6 + 1], rays[i * 6 + 2]);
    r.d = dev::v3(rays[i * 6 + 3], rays[i * 6 + 4], rays[i * 6 + 5]);
    double t;
    int who = dev::closest<false, true>(sc, r, min_t, max_t, &t);
    pt_hit h = {};
    h.shape = who;
    h.material = -1;
    if (who >= 0) {
        dev::Hit hh = dev::finish(sc.shapes[who], r, t);
        h.t = t;
        h.point[0] = hh.p.x;
        h.point[1] = hh.p.y;
        h.point[2] = hh.p.z;
        h.normal[0] = hh.n.x;
        h.normal[1] = hh.n.y;
        h.normal[2] = hh.n.z;
        h.front_face = hh.front ? 1 : 0;
        h.material = sc.shapes[who].material;
    }
    out[i] = h;
}

// Probes of textured scenes keep textured attenuation values in `vals`:
// lane i, level k, component c at vals[(k * 3 + c) * n + i].
template <int NW>
__global__ __launch_bounds__(256) void ray_color_probe(dev::Scene sc, const double *__restrict__ rays, uint64_t *__restrict__ states,
                                size_t n, uint32_t depth, double s11, double *__restrict__ out, double *vals) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Ray r;
    r.o = dev::v3(rays[i * 6 + 0], rays[i * 6 + 1], rays[i * 6 + 2]);
    r.d = dev::v3(rays[i * 6 + 3], rays[i * 6 + 4], rays[i * 6 + 5]);
    dev::Rng rng{states[i]};
    V3 c = vals ? dev::ray_color<NW, true>(sc, r, depth, rng, s11, vals + i, n) : dev::ray_color<NW>(sc, r, depth, rng, s11);
    states[i] = rng.s;
    out[i * 3 + 0] = c.x;
    out[i * 3 + 1] = c.y;
    out[i * 3 + 2] = c.z;
}

template <int NW>
__global__ __launch_bounds__(256) void trace_pixels_probe(dev::Scene sc, FrameParams P, const uint32_t *__restrict__ pixels, size_t n,
                                   double *__restrict__ out, double *vals) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t idx = pixels[i];
    V3 c = vals ? dev::trace_pixel<NW, false, false, march::F_ANY, true>(sc, P, idx % P.width, idx / P.width, nullptr,
                                                                         nullptr, vals + i, n)
                : dev::trace_pixel<NW>(sc, P, idx % P.width, idx / P.width);
    out[i * 3 + 0] = c.x;
    out[i * 3 + 1] = c.y;
    out[i * 3 + 2] = c.z;
}

// Diagnostic build: the same path with per-lane event counters (STATS), summed
// with one 64-bit atomic per counter per lane.  Only pt_count_work uses it.
template <int NW>
__global__ __launch_bounds__(256) void count_work(dev::Scene sc, FrameParams P, const uint32_t *__restrict__ pixels, size_t n,
                           unsigned long long *__restrict__ ctr, double *vals) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Ctr c;
    for (int k = 0; k < C_COUNT; k++) c.c[k] = 0;
    uint32_t idx = pixels[i];
    if (vals)
        dev::trace_pixel<NW, true, false, march::F_ANY, true>(sc, P, idx % P.width, idx / P.width, &c, nullptr,
                                                              vals + i, n);
    else
        dev::trace_pixel<NW, true>(sc, P, idx % P.width, idx / P.width, &c);
    for (int k = 0; k < C_COUNT; k++)
        if (c.c[k]) atomicAdd(&ctr[k], (unsigned long long)c.c[k]);
}

// The skipping march alone on explicit object-space jobs (8 doubles each:
// step, passes, o[3], d[3], unused): t, status (1 hit / 0 miss) and iteration
// count, for checking the device build of pt_march.hpp against the host's.
__global__ __launch_bounds__(256) void march_probe(const double *__restrict__ jobs, size_t n, double *__restrict__ t_out,
                                                   int32_t *__restrict__ status, uint32_t *__restrict__ iters) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double *j = jobs + i * 8;
    march::MarchState m;
    int st = march::M_MISS;
    uint32_t k = 0;
    march::FParams F{};
    F.func = march::F_HEART;
    if (march::march_begin(F, j[0], (int)j[1], j[2], j[3], j[4], j[5], j[6], j[7], &m)) {
        march::MarchStats ms{0, 0, 0, 0};
        while ((st = march::march_step<false>(m, &ms)) == march::M_RUNNING) k++;
    }
    t_out[i] = m.t;
    status[i] = st == march::M_DONE ? 1 : (st == march::M_GUARD ? 2 : 0);
    iters[i] = k;
}

// Diagnostic build: render_tiles with wave-level phase timing; lane 0 of each
// wave adds its wave's stamps (the same for every lane: s_memtime is scalar).
__global__ __launch_bounds__(256, 2) void render_tiles_timed(dev::Scene sc, FrameParams P, double *__restrict__ out,
                                                             unsigned long long *__restrict__ acc) {
    const uint32_t ti = P.tile_begin + blockIdx.x;
    const uint32_t k = dev::tile_position(P.rank + ti * P.world, P.tiles_x, P.world);
    const uint32_t tx = k % P.tiles_x, ty = k / P.tiles_x;
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const uint32_t lx = ((w & 1u) << 3) | (l & 7u), ly = ((w >> 1) << 3) | (l >> 3);
    const uint32_t x = tx * TILE + lx, y = ty * TILE + ly;
    dev::PhaseTimes pt = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    V3 c = dev::v3(0.0, 0.0, 0.0);
    if (x < P.width && y < P.height) c = dev::trace_pixel<4, false, true>(sc, P, x, y, nullptr, &pt);
    if (P.compact == 0 && x < P.width && y < P.height) {
        double *dst = out + ((size_t)y * P.width + x) * 3;
        dst[0] = c.x;
        dst[1] = c.y;
        dst[2] = c.z;
    }
    // per-lane pass counts: sum and max; wave-level times from the lane that
    // kept the wave alive longest (largest stamp total; lowest such lane)
    unsigned long long tot = pt.trace + pt.march + pt.select + pt.finish + pt.scatter + pt.restart, mx = tot;
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long v = __shfl_xor(mx, o, 64);
        mx = v > mx ? v : mx;
    }
    const unsigned long long bal = __ballot(tot == mx);
    if (l == (uint32_t)__ffsll((long long)bal) - 1) {
        atomicAdd(&acc[0], (unsigned long long)pt.trace);
        atomicAdd(&acc[1], (unsigned long long)pt.march);
        atomicAdd(&acc[2], (unsigned long long)pt.select);
        atomicAdd(&acc[3], (unsigned long long)(pt.finish + pt.scatter + pt.restart));
        atomicAdd(&acc[7], (unsigned long long)pt.finish);
        atomicAdd(&acc[8], (unsigned long long)pt.scatter);
        atomicAdd(&acc[9], (unsigned long long)pt.restart);
    }
    atomicAdd(&acc[4], (unsigned long long)pt.passes);
    atomicAdd(&acc[5], (unsigned long long)pt.march_passes);
    atomicMax(&acc[6], (unsigned long long)pt.passes);
}

// ------------------------------------------------------------- launchers
static dev::Scene dscene(const DeviceScene &s) {
    dev::Scene d;
    d.shapes = s.shapes;
    d.mats = s.mats;
    d.nodes = s.nodes;
    d.qnodes = s.qnodes;
    d.leaf = s.leaf;
    d.lin = s.lin;
    d.march = s.march;
    d.boxes = s.boxes;
    d.tex = s.tex;
    d.perlin = s.perlin;
    d.images = s.images;
    d.pixels = s.pixels;
    d.ext = s.ext;
    d.nnodes = s.nnodes;
    d.bvh_bound = s.bvh_bound;
    d.nlin = s.nlin;
    d.nmarch = s.nmarch;
    d.nmats = s.nmats;
    d.diag = s.diag;
    d.guard = s.guard;
    return d;
}

// Attenuation-stack width by depth: one 32-bit material id per bounce.
#define PT_DISPATCH_NW(depth, CALL)        \
    do {                                   \
        if ((depth) <= 8) {                \
            constexpr int NW = 4;          \
            CALL;                          \
        } else if ((depth) <= 16) {        \
            constexpr int NW = 8;          \
            CALL;                          \
        } else if ((depth) <= 32) {        \
            constexpr int NW = 16;         \
            CALL;                          \
        } else {                           \
            constexpr int NW = 32;         \
            CALL;                          \
        }                                  \
    } while (0)

// ------------------------------------------------------------- tuning
const char *const TUNING_NAMES[] = {"engine", "mega_waves", "diag", "wf_slots", "wf_paths", "wf_min_chunks",
                                    "wf_bounce_waves", "wf_march_slice", "wf_walk", "bvh_leaf", nullptr};

static int64_t *tuning_field(Tuning *t, const char *name, int64_t *lo, int64_t *hi, int **iv) {
    struct F {
        const char *n;
        int Tuning::*i;
        int64_t lo, hi;
    };
    static const F fs[] = {
        {"engine", &Tuning::engine, 0, 2},
        {"mega_waves", &Tuning::mega_waves, 2, 5},
        {"diag", &Tuning::diag, 0, 1},
        {"wf_slots", &Tuning::wf_slots, 1, WaveWorkspace::MAX_SLOTS},
        {"wf_min_chunks", &Tuning::wf_min_chunks, 1, 4096},
        {"wf_bounce_waves", &Tuning::wf_bounce_waves, 2, 8},
        {"wf_march_slice", &Tuning::wf_march_slice, 0, 1 << 20},
        {"wf_walk", &Tuning::wf_walk, 0, 8},
        {"bvh_leaf", &Tuning::bvh_leaf, 1, 16},
    };
    *iv = nullptr;
    if (!name) return nullptr;
    if (!strcmp(name, "wf_paths")) {  // (0 = by depth; 1..255 refused in tuning_set)
        *lo = 0;
        *hi = (int64_t)1 << 28;
        return &t->wf_paths;
    }
    for (const F &f : fs)
        if (!strcmp(name, f.n)) {
            *lo = f.lo;
            *hi = f.hi;
            *iv = &(t->*(f.i));
            return nullptr;
        }
    return nullptr;
}

int tuning_set(Tuning *t, const char *name, int64_t v) {
    int64_t lo = 0, hi = 0;
    int *iv = nullptr;
    int64_t *lv = tuning_field(t, name, &lo, &hi, &iv);
    if (!lv && !iv) return PT_ERR_INVALID;
    if (v < lo || v > hi) return PT_ERR_INVALID;
    if (!strcmp(name, "wf_bounce_waves") && !(v == 2 || v == 3 || v == 4 || v == 5 || v == 6 || v == 8))
        return PT_ERR_INVALID;
    if (!strcmp(name, "wf_walk") && !(v == 0 || v == 4 || v == 5 || v == 6 || v == 8)) return PT_ERR_INVALID;
    if (!strcmp(name, "wf_paths") && v > 0 && v < 256) return PT_ERR_INVALID;
    if (lv) *lv = v;
    else *iv = (int)v;
    return PT_OK;
}

int tuning_get(const Tuning &t0, const char *name, int64_t *v) {
    Tuning t = t0;
    int64_t lo = 0, hi = 0;
    int *iv = nullptr;
    int64_t *lv = tuning_field(&t, name, &lo, &hi, &iv);
    if (!lv && !iv) return PT_ERR_INVALID;
    *v = lv ? *lv : (int64_t)*iv;
    return PT_OK;
}

Tuning tuning_defaults() { return Tuning{}; }

hipError_t launch_render_wave(const dev::Scene &sc, const FrameParams &P, double *out, hipStream_t st,
                              WaveWorkspace *ws, int fkind);

// Frames of at least this many samples take the wavefront engine even
// without ray-marched shapes: on C5 (100k spheres, BVH) it runs 1394 against
// the megakernel's 1026 M samples/s (the path state is dense by position and
// the bounce waves stay full where the megakernel's lanes idle on finished
// paths and unequal BVH walks); below it the per-chunk launches cost more
// than they save.
constexpr uint64_t WAVE_MIN_SAMPLES = 1ull << 22;

static bool use_wavefront(const DeviceScene &s, const FrameParams &P, WaveWorkspace *ws) {
    if (s.ext) return true;  // textures / Torus: the extended builds live in the wavefront engine
    const int engine = ws ? ws->tune.engine : 1;
    if (engine == 1) return false;
    if (engine == 2) return ws != nullptr;
    const uint64_t samples = (uint64_t)P.tile_count * TILE * TILE * P.spp;
    return ws != nullptr && (s.diag & 1) == 0 && (s.nmarch > 0 || samples >= WAVE_MIN_SAMPLES);
}

hipError_t launch_render(const DeviceScene &s, const FrameParams &P, double *out, hipStream_t st,
                         WaveWorkspace *ws) {
    if (P.tile_count == 0) return hipSuccess;
    if (P.s_begin > 0 || (P.s_end && P.s_end < P.spp)) {
        // a sample window: only the wavefront engine keeps running sums across launches
        if (!ws || P.s_begin >= (P.s_end ? P.s_end : P.spp)) return hipErrorInvalidValue;
        return launch_render_wave(dscene(s), P, out, st, ws, s.fkind);
    }
    if (use_wavefront(s, P, ws)) return launch_render_wave(dscene(s), P, out, st, ws, s.fkind);
    KernelTimer *tm = ws ? ws->timer : nullptr;
    hipError_t e0 = timer_begin(tm, st, K_MEGA);
    if (e0 != hipSuccess) return e0;
    if (P.depth <= 8 && s.fkind == march::F_HEART) {
        // Heart-only (or no marched shape): the single-function build
        // megakernel register budget (Tuning::mega_waves); depths > 8 use the
        // 2-wave build: their attenuation stacks are wider
        switch (ws ? ws->tune.mega_waves : DEFAULT_WAVES) {
        case 2: render_tiles<4, 2, march::F_HEART><<<P.tile_count, 256, 0, st>>>(dscene(s), P, out); break;
        case 3: render_tiles<4, 3, march::F_HEART><<<P.tile_count, 256, 0, st>>>(dscene(s), P, out); break;
        case 5: render_tiles<4, 5, march::F_HEART><<<P.tile_count, 256, 0, st>>>(dscene(s), P, out); break;
        default: render_tiles<4, 4, march::F_HEART><<<P.tile_count, 256, 0, st>>>(dscene(s), P, out); break;
        }
    } else if (P.depth <= 8) {
        render_tiles<4, 2><<<P.tile_count, 256, 0, st>>>(dscene(s), P, out);
    } else {
        PT_DISPATCH_NW(P.depth, (render_tiles<NW, 2><<<P.tile_count, 256, 0, st>>>(dscene(s), P, out)));
    }
    e0 = hipGetLastError();
    if (e0 != hipSuccess) return e0;
    return timer_end(tm, st);
}

hipError_t launch_unshard(const double *g, uint32_t width, uint32_t height, uint32_t world, double *frame,
                          hipStream_t st, uint32_t y0, uint32_t y1) {
    uint32_t tiles_x = (width + TILE - 1) / TILE, tiles_y = (height + TILE - 1) / TILE;
    uint32_t total = tiles_x * tiles_y;
    uint32_t per_rank = (total + world - 1) / world;
    if (y1 > height) y1 = height;
    if (y0 >= y1) return hipSuccess;
    size_t npix = (size_t)width * (y1 - y0);
    unshard<<<(unsigned)((npix + 255) / 256), 256, 0, st>>>(g, width, y0, y1, world, tiles_x, per_rank, frame);
    return hipGetLastError();
}

hipError_t launch_encode_rgba8(const double *rgb, size_t p0, size_t p1, uint8_t *rgba, hipStream_t st) {
    if (p1 <= p0) return hipSuccess;
    encode_rgba8<<<(unsigned)((p1 - p0 + 255) / 256), 256, 0, st>>>(rgb, p0, p1, (uint32_t *)rgba);
    return hipGetLastError();
}

hipError_t launch_closest_hit(const DeviceScene &s, const double *rays, size_t n, double min_t, double max_t,
                              pt_hit *out, hipStream_t st) {
    if (!n) return hipSuccess;
    closest_hit_probe<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(dscene(s), rays, n, min_t, max_t, out);
    return hipGetLastError();
}

// Stream-ordered scratch for the probes' textured attenuation values (textured
// scenes only): n lanes x (depth + 1) levels x 3 doubles.
struct ProbeVals {
    double *p = nullptr;
    hipStream_t st;
    hipError_t alloc(const DeviceScene &s, size_t n, uint32_t depth) {
        if (!s.ext) return hipSuccess;
        return hipMallocAsync((void **)&p, n * (depth + 1) * 3 * sizeof(double), st);
    }
    ~ProbeVals() {
        if (p) (void)hipFreeAsync(p, st);
    }
};

hipError_t launch_ray_color(const DeviceScene &s, const double *rays, uint64_t *states, size_t n, uint32_t depth,
                            double s11, double *out, hipStream_t st) {
    if (!n) return hipSuccess;
    ProbeVals vals{nullptr, st};
    hipError_t e = vals.alloc(s, n, depth);
    if (e != hipSuccess) return e;
    PT_DISPATCH_NW(depth, (ray_color_probe<NW><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(
                              dscene(s), rays, states, n, depth, s11, out, vals.p)));
    return hipGetLastError();
}

hipError_t launch_trace_pixels(const DeviceScene &s, const FrameParams &P, const uint32_t *pixels, size_t n,
                               double *out, hipStream_t st) {
    if (!n) return hipSuccess;
    ProbeVals vals{nullptr, st};
    hipError_t e = vals.alloc(s, n, P.depth);
    if (e != hipSuccess) return e;
    PT_DISPATCH_NW(P.depth, (trace_pixels_probe<NW><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(
                                dscene(s), P, pixels, n, out, vals.p)));
    return hipGetLastError();
}

hipError_t launch_count_work(const DeviceScene &s, const FrameParams &P, const uint32_t *pixels, size_t n,
                             unsigned long long *ctr, hipStream_t st) {
    if (!n) return hipSuccess;
    ProbeVals vals{nullptr, st};
    hipError_t e = vals.alloc(s, n, P.depth);
    if (e != hipSuccess) return e;
    PT_DISPATCH_NW(P.depth, (count_work<NW><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(dscene(s), P, pixels, n,
                                                                                         ctr, vals.p)));
    return hipGetLastError();
}

hipError_t launch_march_probe(const double *jobs, size_t n, double *t, int32_t *status, uint32_t *iters,
                              hipStream_t st) {
    if (n == 0) return hipSuccess;
    march_probe<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(jobs, n, t, status, iters);
    return hipGetLastError();
}

hipError_t launch_render_timed(const DeviceScene &s, const FrameParams &P, double *out, unsigned long long *acc,
                               hipStream_t st) {
    if (P.tile_count == 0) return hipSuccess;
    if (s.ext) return hipErrorNotSupported;  // the timing build has no extended (texture / Torus) build
    render_tiles_timed<<<P.tile_count, 256, 0, st>>>(dscene(s), P, out, acc);
    return hipGetLastError();
}

}  // namespace pt
