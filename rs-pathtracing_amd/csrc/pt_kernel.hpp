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
    int32_t *leaf = nullptr, *lin = nullptr, *march = nullptr;
    DBox *boxes = nullptr;
    DTexture *tex = nullptr;  // non-solid textures (null when the scene has none)
    DPerlin *perlin = nullptr;
    DImage *images = nullptr;
    uint8_t *pixels = nullptr;
    int nshapes = 0, nmats = 0, nnodes = 0, nlin = 0, nmarch = 0;
    int ext = 0;    // non-solid textures or a Torus: the extended (EXT) kernel builds
    int fkind = 0;  // 0: every marched shape is a Heart (or none) -> Heart-only kernel builds; -1: any
};

// Device workspace of the wavefront engine (pt_wave.hip), grown on demand and
// reused by every frame of a renderer.
// Per-kernel launch timing (pt_kernel_timing): HIP events recorded on the
// launch stream around every render-path kernel while enabled.
enum KernelKind : int { K_BOUNCE = 0, K_MARCH = 1, K_SELECT = 2, K_REDUCE = 3, K_MEGA = 4, K_KINDS = 5 };
struct KernelTimer;
KernelTimer *timer_new();
void timer_free(KernelTimer *t);
hipError_t timer_begin(KernelTimer *t, hipStream_t st, int kind);  // no-op when t is null
hipError_t timer_end(KernelTimer *t, hipStream_t st);
hipError_t timer_collect(KernelTimer *t, double *ms, uint32_t *launches);  // sums since last collect

struct WaveWorkspace {
    void *base = nullptr;
    size_t bytes = 0;
    unsigned long long *diag = nullptr;  // march-kernel phase diagnostics (pt_wave_diag), when enabled
    KernelTimer *timer = nullptr;         // per-kernel timing (pt_kernel_timing), when enabled
    // chunk pipeline: extra launch streams (chunk c runs on stream c % slots,
    // stream 0 being the caller's) and the events that order them
    static constexpr int MAX_SLOTS = 4;
    hipStream_t side[MAX_SLOTS - 1] = {};
    hipEvent_t fork = nullptr, join[MAX_SLOTS - 1] = {}, reduced = nullptr;
    int device = -1;
};
void wave_workspace_free(WaveWorkspace *ws);

// Renders this rank's tiles of P into out.  Scenes with ray-marched shapes use
// the wavefront engine (ws required), others the megakernel; PT_ENGINE=mega or
// PT_ENGINE=wave in the environment forces one.
hipError_t launch_render(const DeviceScene &s, const FrameParams &P, double *out, hipStream_t st,
                         WaveWorkspace *ws);
hipError_t launch_unshard(const double *gathered, uint32_t width, uint32_t height, uint32_t world, double *frame,
                          hipStream_t st);
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
