// pt_kernel.hpp — host-side launchers of the HIP kernels (pt_kernel.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/rs_pathtracing.h"
#include "pt_types.hpp"

namespace pt {

struct DeviceScene {
    DShape *shapes = nullptr;
    DMaterial *mats = nullptr;
    DNodeC *nodes = nullptr;
    DQGrid *qnodes = nullptr;  // the quantized layouts after their grid (large trees only; else null)
    int32_t *leaf = nullptr, *lin = nullptr, *march = nullptr;
    DBox *boxes = nullptr;
    DTexture *tex = nullptr;  // non-solid textures (null when the scene has none)
    DPerlin *perlin = nullptr;
    DImage *images = nullptr;
    uint8_t *pixels = nullptr;
    int nshapes = 0, nmats = 0, nnodes = 0, nlin = 0, nmarch = 0;
    float bvh_bound = 0.f;  // Accel::bvh_bound
    int ext = 0;    // non-solid textures or a Torus: the extended (EXT) kernel builds
    int fkind = 0;  // 0: every marched shape is a Heart (or none) -> Heart-only kernel builds; -1: any
    int diag = 0;  // Tuning::diag (timing ablation), copied here for the probes
    unsigned long long *guard = nullptr;  // device counter of marches dropped by the march guard
};

// Device workspace of the wavefront engine (pt_wave.hip), grown on demand and
// reused by every frame of a renderer.
// Per-kernel launch timing (pt_kernel_timing): HIP events recorded on the
// launch stream around every render-path kernel while enabled.
// (kind 5 was the wavefront tail kernel until round 6; it now times the per-slot unwind, wf_unwind)
enum KernelKind : int { K_BOUNCE = 0, K_MARCH = 1, K_SELECT = 2, K_REDUCE = 3, K_MEGA = 4, K_UNWIND = 5, K_WALK = 6, K_KINDS = 7 };
struct KernelTimer;
KernelTimer *timer_new();
void timer_free(KernelTimer *t);
hipError_t timer_begin(KernelTimer *t, hipStream_t st, int kind);  // no-op when t is null
hipError_t timer_end(KernelTimer *t, hipStream_t st);
hipError_t timer_collect(KernelTimer *t, double *ms, uint32_t *launches);  // sums since last collect

// Tuning knobs of the render engines (pt_renderer_set_option; the option names
// are the field names).  The defaults are the measured optimum on MI355X
// (DESIGN.md §5); bench.py reports every knob that differs from its default.
struct Tuning {
    int engine = 0;                  // 0 auto (wavefront for a scene that marches or has textures / a Torus, and for any frame of >= 2^22 samples; else the megakernel), 1 megakernel, 2 wavefront
    int mega_waves = 4;              // megakernel register budget, waves per SIMD (2..5)
    int diag = 0;                    // bit 0: skip ray-marched shapes (a timing ablation, not the reference)
    int wf_slots = 2;                // sample chunks in flight, one stream each (1..4)
    int64_t wf_paths = 0;            // path slots per chunk (256 .. 2^28; 0: 48M up to depth 16, else 256M).  Deep
                                     // frames spend a quarter of a chunk in its tail of latency-bound iterations:
                                     // C2 depth 50 48M 1156, 96M 1226, 128M 1230-1241, 160M 1235 M samples/s (~58 GB
                                     // per chunk stream at 128M); at depth 8 128M costs the bounce 3 % (C2 2010 vs
                                     // 2039), C1, C3, C5 unchanged (round 5 r5w-r5y)
    int wf_min_chunks = 1;           // at least this many sample chunks per frame (1..4096)
    int wf_bounce_waves = 3;         // wf_bounce register budget (2, 3, 4, 5, 6, 8)
    int wf_march_slice = 256;        // march-queue run dealt to a block (0 = contiguous share)
    int wf_walk = 5;                 // large-tree scenes without marched shapes: the BVH walk in its own kernel (wf_walk)
                                     // at this register budget, waves per SIMD (4, 5, 6, 8; 0: the walk in the bounce)
    int bvh_leaf = 1;                // shapes per BVH leaf (1..16; C5 677 / 609 / 534 M samples/s at 1 / 2 / 4)
};
Tuning tuning_defaults();  // the measured defaults; a renderer changes them only through pt_renderer_set_option
// 0 on success, PT_ERR_INVALID for an unknown name or a value out of range
int tuning_set(Tuning *t, const char *name, int64_t value);
int tuning_get(const Tuning &t, const char *name, int64_t *value);
extern const char *const TUNING_NAMES[];  // null-terminated

// Diagnostic builds of the wavefront kernels (pt_wave_diag: wave-level s_memtime per bounce section and march
// phase): make EXTRA=-DPT_WAVE_DIAG=1.  In the product build the instrumentation is compiled out of every
// kernel (it is no template parameter of the hot kernels) and pt_wave_diag refuses to enable it.
#ifndef PT_WAVE_DIAG
#define PT_WAVE_DIAG 0
#endif

struct WaveWorkspace {
    Tuning tune;  // this renderer's knobs (both engines read them from here)
    void *base = nullptr;
    size_t bytes = 0;
    unsigned long long *diag = nullptr;  // march-kernel phase diagnostics (pt_wave_diag), when enabled
    KernelTimer *timer = nullptr;         // per-kernel timing (pt_kernel_timing), when enabled
    // chunk pipeline: extra launch streams (chunk c runs on stream c % slots,
    // stream 0 being the caller's) and the events that order them
    static constexpr int MAX_SLOTS = 4;
    hipStream_t side[MAX_SLOTS - 1] = {};
    hipEvent_t fork = nullptr, join[MAX_SLOTS - 1] = {}, reduced = nullptr;
    // recorded on the launch stream after a frame's last use of the workspace;
    // the next frame (on any stream) waits for it
    hipEvent_t done = nullptr;
    bool used = false;
    // the launches' argument blocks of the last frame (pt_wave.hip WfArgs): pinned staging and device copy;
    // args_ev is recorded after the frame's copy (the staging buffer is free once it has run)
    void *args_host = nullptr, *args_dev = nullptr;
    size_t args_bytes = 0;
    hipEvent_t args_ev = nullptr;
    bool args_pending = false;
    int device = -1;
};
void wave_workspace_free(WaveWorkspace *ws);

// Renders this rank's tiles of P into out.  Scenes with ray-marched shapes use
// the wavefront engine (ws required), others the megakernel; the renderer
// option "engine" (1 megakernel, 2 wavefront) forces one.
hipError_t launch_render(const DeviceScene &s, const FrameParams &P, double *out, hipStream_t st,
                         WaveWorkspace *ws);
// rows [y0, y1) of the frame from gathered shards (pt_unshard_device)
hipError_t launch_unshard(const double *gathered, uint32_t width, uint32_t height, uint32_t world, double *frame,
                          hipStream_t st, uint32_t y0 = 0, uint32_t y1 = ~0u);
// display encode of pixels [p0, p1) (pt_encode_rgba8_device); rgba is 4-byte aligned
hipError_t launch_encode_rgba8(const double *rgb, size_t p0, size_t p1, uint8_t *rgba, hipStream_t st);
hipError_t launch_closest_hit(const DeviceScene &s, const double *rays, size_t n, double min_t, double max_t,
                              pt_hit *out, hipStream_t st);
hipError_t launch_ray_color(const DeviceScene &s, const double *rays, uint64_t *states, size_t n, uint32_t depth,
                            double s11, double *out, hipStream_t st);
hipError_t launch_trace_pixels(const DeviceScene &s, const FrameParams &P, const uint32_t *pixels, size_t n,
                               double *out, hipStream_t st);

hipError_t launch_count_work(const DeviceScene &s, const FrameParams &P, const uint32_t *pixels, size_t n,
                             unsigned long long *ctr, hipStream_t st);

hipError_t launch_march_probe(const double *jobs, size_t n, double *t, int32_t *status, uint32_t *iters,
                              hipStream_t st);
hipError_t launch_render_timed(const DeviceScene &s, const FrameParams &P, double *out, unsigned long long *acc,
                               hipStream_t st);

}  // namespace pt
