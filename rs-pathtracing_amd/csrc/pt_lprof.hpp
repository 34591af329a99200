// pt_lprof.hpp — tuning instrumentation of the wavefront kernels, compiled out
// of the product builds: the bounce kernel's lane profile (PT_LANE_PROF) and
// the march kernel's region timing (PT_MARCH_REGIONS).
//
// Built with -DPT_LANE_PROF (scripts/variants.sh lprof "-DPT_LANE_PROF",
// loaded through PT_AMD_LIB; scripts/bounce_lanes.py reads it), PT_LP(k) at
// profiling point k makes the wave's first active lane add one wave pass and
// the number of active lanes to block-local counters, which the kernel flushes
// to a device array at its end (pt_lane_prof).  Passes per point say how
// often a wave runs that code, lanes per pass how full it is when it does.
// In every other build PT_LP is nothing and the kernels are unchanged.
#pragma once
#include <hip/hip_runtime.h>

#ifdef PT_MARCH_REGIONS
// Tuning builds only: wave wall-clock (s_memtime) spent in each region of
// the march kernel (pt_march.hpp's PT_MREG points), as seen by the wave's
// first active lane, summed over all waves, the same weighted by the lanes
// active at the region's start, and per profiling point of pt_march.hpp
// (PT_MPROF: one per segment, halving level, literal add, ...) the wave
// passes and the lanes active in them (pt_march_regions).
namespace pt {
namespace mreg {
enum { R_ITER, R_POLY, R_PREFIX, R_HALVE, R_ADV, R_LIT, R_REFILL, R_TOTAL, R_N };
enum { P_iters, P_lin_init, P_lit_adds, P_advance_loops, P_evals, P_sir_inside, P_lin_fail_zero, P_lin_fail_q,
       P_lin_fail_tie, P_lin_fail_zone, P_N };
constexpr int G_N = 2 * R_N + 2 * P_N;
__device__ unsigned long long g_acc[G_N];
__shared__ unsigned long long t0[4][R_N], acc[4][R_N], accl[4][R_N], n0[4][R_N], pw[4][P_N], pl[4][P_N];
__device__ __forceinline__ unsigned long long now() {
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
__device__ __forceinline__ bool leader() {
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    return lane == (uint32_t)__builtin_ctzll(__ballot(1));
}
__device__ __forceinline__ void begin(int r) {
    const unsigned long long m = __ballot(1);
    if (leader()) {
        t0[threadIdx.x >> 6][r] = now();
        n0[threadIdx.x >> 6][r] = __popcll(m);
    }
}
__device__ __forceinline__ void end(int r) {
    if (leader()) {
        const unsigned long long dt = now() - t0[threadIdx.x >> 6][r];
        acc[threadIdx.x >> 6][r] += dt;
        accl[threadIdx.x >> 6][r] += dt * n0[threadIdx.x >> 6][r];
    }
}
__device__ __forceinline__ void prof(int k) {
    const unsigned long long m = __ballot(1);
    if (leader()) {
        pw[threadIdx.x >> 6][k] += 1;
        pl[threadIdx.x >> 6][k] += __popcll(m);
    }
}
__device__ __forceinline__ void poly_begin() { begin(R_POLY); }
__device__ __forceinline__ void poly_end() { end(R_POLY); }
__device__ __forceinline__ void prefix_begin() { begin(R_PREFIX); }
__device__ __forceinline__ void prefix_end() { end(R_PREFIX); }
__device__ __forceinline__ void halve_begin() { begin(R_HALVE); }
__device__ __forceinline__ void halve_end() { end(R_HALVE); }
__device__ __forceinline__ void adv_begin() { begin(R_ADV); }
__device__ __forceinline__ void adv_end() { end(R_ADV); }
__device__ __forceinline__ void lit_begin() { begin(R_LIT); }
// wf_march's hooks: per-wave accumulators cleared at the start, the march step
// and the job refill timed, a literal loop (opened inside the step) closed after
// it, and the sums flushed at the end
__device__ __forceinline__ void kernel_begin(unsigned long long *t_kernel) {
    if ((threadIdx.x & 63) == 0) {
        for (int k = 0; k < R_N; k++) t0[threadIdx.x >> 6][k] = acc[threadIdx.x >> 6][k] = accl[threadIdx.x >> 6][k] = 0;
        for (int k = 0; k < P_N; k++) pw[threadIdx.x >> 6][k] = pl[threadIdx.x >> 6][k] = 0;
    }
    *t_kernel = now();
}
__device__ __forceinline__ void step_end() {
    end(R_ITER);
    if (leader() && t0[threadIdx.x >> 6][R_LIT]) {  // a literal loop ran: close it
        const unsigned long long dt = now() - t0[threadIdx.x >> 6][R_LIT];
        acc[threadIdx.x >> 6][R_LIT] += dt;
        accl[threadIdx.x >> 6][R_LIT] += dt * n0[threadIdx.x >> 6][R_LIT];
        t0[threadIdx.x >> 6][R_LIT] = 0;
    }
}
__device__ __forceinline__ void kernel_end(unsigned long long t_kernel) {
    if ((threadIdx.x & 63) == 0) {
        const int w = threadIdx.x >> 6;
        acc[w][R_TOTAL] = now() - t_kernel;
        accl[w][R_TOTAL] = 0;
        for (int k = 0; k < R_N; k++) {
            atomicAdd(&g_acc[k], acc[w][k]);
            atomicAdd(&g_acc[R_N + k], accl[w][k]);
        }
        for (int k = 0; k < P_N; k++) {
            atomicAdd(&g_acc[2 * R_N + k], pw[w][k]);
            atomicAdd(&g_acc[2 * R_N + P_N + k], pl[w][k]);
        }
    }
}
}  // namespace mreg
}  // namespace pt
#define PT_MREG(what) pt::mreg::what()
#define PT_MPROF(field) (pt::mreg::prof(pt::mreg::P_##field))
#define PT_MREG_KERNEL_BEGIN() \
    unsigned long long mreg_t_kernel_; \
    pt::mreg::kernel_begin(&mreg_t_kernel_)
#define PT_MREG_STEP_BEGIN() pt::mreg::begin(pt::mreg::R_ITER)
#define PT_MREG_STEP_END() pt::mreg::step_end()
#define PT_MREG_REFILL_BEGIN() pt::mreg::begin(pt::mreg::R_REFILL)
#define PT_MREG_REFILL_END() pt::mreg::end(pt::mreg::R_REFILL)
#define PT_MREG_KERNEL_END() pt::mreg::kernel_end(mreg_t_kernel_)
#else
#define PT_MREG_KERNEL_BEGIN() ((void)0)
#define PT_MREG_STEP_BEGIN() ((void)0)
#define PT_MREG_STEP_END() ((void)0)
#define PT_MREG_REFILL_BEGIN() ((void)0)
#define PT_MREG_REFILL_END() ((void)0)
#define PT_MREG_KERNEL_END() ((void)0)
#endif


namespace pt {
namespace lprof {
enum Point : int {
    LIVE,         // wf_bounce: a live path after its state load
    SHADE_HIT,    // shade: a hit to shade (not a miss, not depth 0)
    LAMBERT,      // Lambertian scatter
    REJECT_TRY,   // one try of random_in_unit_sphere's rejection loop
    METAL,        // Metal scatter
    DIELECTRIC,   // Dielectric scatter
    EMIT,         // DiffuseLight / EmptyMaterial: the path ends on the hit
    ENDED,        // wf_bounce: a path the shade ended (leaf stored)
    TRACE,        // wf_bounce: a path that traces a new ray
    ULIST_SHAPE,  // one shape of the wave-uniform list
    RECT_ROWS,    // a rectangle's x/y rows (its t was in range)
    UBOX_PASS,    // a uniform-list cube or sphere past its padded world box: the exact test
    BVH_NODE,     // one node of the threaded BVH walk
    BVH_ENTER,    // a node whose box the ray enters (inner node descended or leaf tested)
    BVH_LEAF,     // one leaf shape test
    PRE_SLAB,     // march pre-check: the ray enters a marched shape's padded box
    PRE_JOB,      // march pre-check: a march job record and its queue-order prediction
    ANY_END,      // a depth-0 trace that ends its path (any-hit answer)
    STORE,        // the state stores of every input position
    N_POINTS
};
}  // namespace lprof
}  // namespace pt

#if defined(PT_LANE_PROF)
namespace pt {
namespace lprof {
static __device__ unsigned long long g_counts[2 * N_POINTS];
static __shared__ unsigned long long s_pass[N_POINTS], s_lanes[N_POINTS];
__device__ __forceinline__ void hit(int k) {
    const unsigned long long m = __ballot(1);
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    if (lane == (uint32_t)__builtin_ctzll(m)) {
        atomicAdd(&s_pass[k], 1ull);
        atomicAdd(&s_lanes[k], (unsigned long long)__popcll(m));
    }
}
__device__ __forceinline__ void begin_kernel() {
    if (threadIdx.x < N_POINTS) s_pass[threadIdx.x] = s_lanes[threadIdx.x] = 0;
    __syncthreads();
}
__device__ __forceinline__ void end_kernel() {
    __syncthreads();
    if (threadIdx.x < N_POINTS) {
        atomicAdd(&g_counts[threadIdx.x], s_pass[threadIdx.x]);
        atomicAdd(&g_counts[N_POINTS + threadIdx.x], s_lanes[threadIdx.x]);
    }
}
}  // namespace lprof
}  // namespace pt
#endif
#if defined(PT_LANE_PROF) && defined(__HIP_DEVICE_COMPILE__)
#define PT_LP(k) pt::lprof::hit(pt::lprof::k)
#define PT_LP_BEGIN() pt::lprof::begin_kernel()
#define PT_LP_END() pt::lprof::end_kernel()
#else
#define PT_LP(k) ((void)0)
#define PT_LP_BEGIN() ((void)0)
#define PT_LP_END() ((void)0)
#endif
