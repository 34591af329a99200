// pt_lprof.hpp — lane profile of the bounce kernel (tuning builds only).
//
// Built with -DPT_LANE_PROF (scripts/variants.sh lprof "-DPT_LANE_PROF",
// loaded through PT_AMD_LIB; scripts/bounce_lanes.py reads it), PT_LP(k) at
// profiling point k makes the wave's first active lane add one wave pass and
// the number of active lanes to block-local counters, which the kernel flushes
// to a device array at its end (pt_lane_prof).  Passes per point say how
// often a wave runs that code, lanes per pass how full it is when it does.
// In every other build PT_LP is nothing and the kernels are unchanged.
#pragma once

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
