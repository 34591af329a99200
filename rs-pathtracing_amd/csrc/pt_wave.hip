// pt_wave.hip — wavefront engine for scenes with ray-marched shapes.
//
// The megakernel (pt_kernel.hip) keeps a path in a lane for all of its
// samples.  That is ideal while every lane does the same kind of work, but a
// Heart march (tens of march iterations, ~1k VALU instructions each) runs for
// a handful of lanes at a time and stalls the other 60 of its wave: on cornell
// the megakernel spends >90 % of its wave time with few lanes active.
//
// Here the per-pixel sample loop (renderer/mod.rs:151-155, ray_color :23-45)
// is cut at the closest hit into queue-connected kernels, one bounce per
// launch (iteration `it`):
//
//   wf_bounce(it)  for every live path: shade the pending hit (material,
//                  scatter, next ray — or end the path and store its sample
//                  radiance), then trace the new ray through the uniform list
//                  and the BVH.  A path whose ray enters a marched shape's
//                  bound before its best hit goes to the march queue; the rest
//                  go straight to the next live list.
//   wf_march(it)   persistent lanes that refill themselves from the march
//                  queue: every lane of every wave marches (select + march
//                  iterations, pt_march.hpp) until the queue is drained, so
//                  the march runs with full waves.
//   wf_reduce      per pixel, adds the chunk's sample radiances in sample
//                  order to the running sum (the reference's in-order sum),
//                  and divides by spp after the last chunk.
//   wf_unwind      (chunks of few pixels) each slot's radiance, unwound in
//                  place before wf_reduce, one thread per slot.
//
// Path state lives in HBM, structure-of-arrays, dense by position: bounce
// `it` reads its k-th input from one state set at the position the live list
// names and writes it at position k of the other set (76 B per path), so the
// later kernels read a dense, id-ordered subsequence of the previous bounce's
// outputs (not a sparse one of the chunk's slots).  What a path leaves for
// the per-pixel reduce (leaf radiance, attenuation ids) is kept per slot
// (pixel, sample).  Order-preserving compaction keeps 8x8 pixel blocks
// together in the lists.  Every value is computed by the same device functions, in the
// same per-path order, as the megakernel and the oracle: the frame is
// bit-identical.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <vector>

#include "pt_lprof.hpp"  // tuning instrumentation (compiled out of the product builds)

#include "pt_device.hpp"
#include "pt_kernel.hpp"

namespace pt {

using dev::Ray;
using dev::V3;

// Path state between kernels, structure of arrays, dense by position: the
// bounce kernel of iteration `it` reads path k of its input list at position
// list[k] of one set and writes it at position k of the other (the two sets
// alternate by iteration), so every later kernel reads a dense, id-ordered
// subsequence of the previous bounce's outputs instead of a sparse one of the
// chunk's slots.  The slot id (sample, pixel) travels with the path.
// Blocks of 64 positions (one wave's worth), each field a contiguous run in
// the block: the eight 8-byte fields (ray, best hit t, rng) at 512-byte steps,
// then the three 4-byte ones (who, meta, slot id) at 256-byte steps, 4864 B
// per block.  A wave on 64 consecutive positions reads or writes each field
// as one 512- (256-) byte run, as in plain structure of arrays, but every
// field sits at an immediate offset from one per-lane address: with one array
// per field the loop-invariant field bases of the two sets were 22 SGPR pairs,
// and the bounce kernel spilled 65 SGPRs to VGPR lanes (round 5).
// Who and the attenuation-stack count share one word, and the depth comes from the iteration (72 B of state per
// path; round 5): a live path's depth at bounce `it` is depth - (it - 1) for every path (each bounce before it
// shaded it once and scattered), so only the stack count is state; it shares a word with the pending hit's
// shape: (who + 1) | count << 25 (shapes < 2^24: the BVH's leaf index bound; count <= depth <= 64).
constexpr uint32_t WHO_MASK = (1u << 25) - 1u;
__host__ __device__ __forceinline__ uint32_t pack_who(int who, uint32_t count) {
    return (uint32_t)(who + 1) | (count << 25);
}
__host__ __device__ __forceinline__ int unpack_who(uint32_t w) { return (int)(w & WHO_MASK) - 1; }

struct PathSoA {
    char *base;
    size_t cap;  // a multiple of 64
    static constexpr size_t BYTES = 8 * 8 + 2 * 4;  // per path
    static constexpr uint32_t BLK = 64, BLK_BYTES = (uint32_t)BYTES * BLK;
    enum F8 : int { OX, OY, OZ, DX, DY, DZ, T, RNG };
    enum F4 : int { WHO, SID };
    // the 8-byte fields of position k: d8(k)[f * 64]; the 4-byte ones: d4(k)[f * 64]
    __host__ __device__ double *d8(uint32_t k) const {
        return (double *)(base + (size_t)(k / BLK) * BLK_BYTES) + (k % BLK);
    }
    __host__ __device__ uint32_t *d4(uint32_t k) const {
        return (uint32_t *)(base + (size_t)(k / BLK) * BLK_BYTES + 8 * 8 * BLK) + (k % BLK);
    }
    __host__ __device__ double &t(uint32_t k) const { return d8(k)[T * BLK]; }  // best hit t
    // the word holding the best hit's shape (-1: miss), packed with the stack count (pack_who)
    __host__ __device__ uint32_t &who(uint32_t k) const { return d4(k)[WHO * BLK]; }
};

// Device view of the workspace for one chunk.
struct WfView {
    PathSoA in, out;  // the bounce reads `in` (by list position) and writes `out` (by its input index)
    uint32_t *ids;   // attenuation-id stack: entry k of a path at ids[k * cap + id]
    double *att;     // textured attenuation values (EXT builds): (k * 3 + c) * cap + id
    // per slot, 32 B: an ended path's leaf radiance (x, y, z) and its attenuation-stack depth (u64 bits; wf_reduce
    // unwinds the stack)
    double *leaf;
    uint8_t *status;  // per output position of a bounce: bit 0 path alive, bit 1 needs a march, bit 2 long march
    uint32_t *list, *mq;  // positions (in `out` of the previous / current bounce) of the live paths and march jobs
    // march jobs pre-selected by the bounce kernel (scenes with one ray-marched
    // shape): object-space ray and bound interval per position,
    // 64 B each (o, d, start, end); null when the march kernel selects itself
    double2 *jo;
    // per iteration: [0] the bounce's input count, [1] march-queue count,
    // [2] long-march jobs, [3] unused; word 3 (iteration 0) is the chunk's
    // stop mark (stop_gate): set, the first bounce and wf_reduce do nothing
    uint32_t *cnt;
    double *acc;    // running per-pixel sums (3 per pixel of the tile group)
    uint32_t cap;   // path slots
    uint32_t npix;  // pixels of the tile group (tiles * 256)
    uint32_t s0, ns;  // sample range of the chunk
    uint32_t tile0;   // first tile of the group (index in this rank's tile list)
};

// What a launch of the wavefront kernels reads besides its iteration: the
// scene, the frame and the chunk's view (for one parity of the iteration: the
// two state sets swap roles every bounce).  A frame's blocks, one per (chunk,
// parity), are written to device memory with one copy before its first
// launch, and each kernel takes a pointer to its block (16 bytes of kernel
// arguments instead of 704 by value).  The kernels read the block through
// kargs(): a scalar pointer the compiler cannot see through, taken again at
// the top of every trip of their loops, so each field is a scalar load next to
// its use rather than a value held in an SGPR for the whole kernel (by value,
// the loop-invariant arguments and their derived addresses spilled 60-70
// SGPRs of the bounce builds to VGPR lanes, round 5).
struct WfArgs {
    dev::Scene sc;
    FrameParams P;
    WfView v;
};

template <class T>
__device__ __forceinline__ const T &kargs(const T *p) {
    typedef const __attribute__((address_space(4))) T *cptr;
    cptr q = (cptr)p;
    asm volatile("" : "+s"(q));
    return *(const T *)q;
}

__device__ __forceinline__ uint32_t lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// The attenuation-id stack of a path kept in HBM: a push writes one 32-bit
// id (once, where the recursion would have pushed it); the ids are read back
// only when the path ends (unwind).
struct MemStack {
    uint32_t *base;
    size_t stride;
    int n;
    double *vb;  // textured attenuation values: level k, component c at vb[(k * 3 + c) * stride]
    __device__ __forceinline__ void push_val(V3 a) {
        vb[(size_t)(n * 3 + 0) * stride] = a.x;
        vb[(size_t)(n * 3 + 1) * stride] = a.y;
        vb[(size_t)(n * 3 + 2) * stride] = a.z;
        push(dev::VAL_BIT);
    }
    __device__ __forceinline__ V3 val(int level) const {
        return dev::v3(vb[(size_t)(level * 3 + 0) * stride], vb[(size_t)(level * 3 + 1) * stride],
                       vb[(size_t)(level * 3 + 2) * stride]);
    }
    __device__ __forceinline__ void push(uint32_t id) {
        base[(size_t)n * stride] = id;
        n++;
    }
    __device__ __forceinline__ uint32_t pop() {
        n--;
        return base[(size_t)n * stride];
    }
};

// dev::unwind for an HBM id stack, with the loads batched: the top UB ids are
// loaded together, then their albedos together, then multiplied in the
// recursion's order (top of the stack first, as dev::unwind pops them), so a
// path of n bounces waits for 2*ceil(n/UB) dependent round trips instead of
// 2n.  Textured (EXT) stacks take the generic unwind.
constexpr int UB = 4;
template <bool EXT>
__device__ __forceinline__ V3 unwind_mem(const dev::Scene &sc, MemStack &stk, V3 c) {
    if (EXT) return dev::unwind<false, true>(sc, stk, c);
    while (stk.n > 0) {
        const int m = stk.n < UB ? stk.n : UB;
        uint32_t id[UB];
#pragma unroll
        for (int j = 0; j < UB; j++) id[j] = j < m ? stk.base[(size_t)(stk.n - 1 - j) * stk.stride] : 0u;
        double ax[UB], ay[UB], az[UB];
#pragma unroll
        for (int j = 0; j < UB; j++) {
            const DMaterial &mt = sc.mats[id[j]];
            ax[j] = j < m ? mt.albedo[0] : 1.0;
            ay[j] = j < m ? mt.albedo[1] : 1.0;
            az[j] = j < m ? mt.albedo[2] : 1.0;
        }
#pragma unroll
        for (int j = 0; j < UB; j++)
            if (j < m) c = dev::v3(ax[j] * c.x, ay[j] * c.y, az[j] * c.z);  // Vector3d::product
        stk.n -= m;
    }
    return c;
}

// A path that ends stores its leaf radiance (emitted light, background or 0)
// and its attenuation-stack depth; the per-pixel reduce unwinds the stack
// (the recursion's products, in its order) when it sums the chunk's samples,
// so the bounce kernel's waves never wait for the unwind's dependent loads.
// Non-temporal (read once, by the chunk's reduce): iso bounce -0.6 ms, C2 +0.4 %.
// The leaf and the depth form one 32-byte record per slot (two 16-byte stores): an ended path's write touches
// one line instead of the four of separate x / y / z / depth arrays, where only ~1 lane in 8 ends per bounce
// (C2 iso bounce 226.4 -> 222.0 ms, +1.1..2.8 %, round-4 A/B r4f).
__device__ __forceinline__ void end_path(const WfView &v, uint32_t id, const MemStack &stk, V3 leaf) {
    typedef double d2v __attribute__((ext_vector_type(2)));
    d2v *rec = (d2v *)(v.leaf + (size_t)id * 4);
    __builtin_nontemporal_store((d2v){leaf.x, leaf.y}, rec);
    __builtin_nontemporal_store((d2v){leaf.z, __builtin_bit_cast(double, (uint64_t)(uint32_t)stk.n)}, rec + 1);
}

// A live path's state at output position k: non-temporal stores (the state
// is read back only by the next bounce, after 1.8 GB of other traffic: no
// cache level holds it that long; C2 iso bounce 216.2 -> 211.5 ms, 1792 ->
// 1814 M samples/s; non-temporal loads were slower).
template <typename T>
__device__ __forceinline__ void st_path(T *p, T x) {
    __builtin_nontemporal_store(x, p);
}
template <typename T>
__device__ __forceinline__ T ld_path(const T *p) {
    return *p;
}
// count: the path's attenuation-stack count (stored with who; the depth follows from the iteration)
__device__ __forceinline__ void store_path(const PathSoA &S, uint32_t k, uint32_t id, const Ray &ray, double best,
                                           int who, uint64_t rng, uint32_t count) {
    double *a = S.d8(k);
    uint32_t *b = S.d4(k);
    constexpr uint32_t B = PathSoA::BLK;
    st_path(a + PathSoA::OX * B, ray.o.x);
    st_path(a + PathSoA::OY * B, ray.o.y);
    st_path(a + PathSoA::OZ * B, ray.o.z);
    st_path(a + PathSoA::DX * B, ray.d.x);
    st_path(a + PathSoA::DY * B, ray.d.y);
    st_path(a + PathSoA::DZ * B, ray.d.z);
    st_path(a + PathSoA::T * B, best);
    st_path(b + PathSoA::WHO * B, pack_who(who, count));
    st_path((uint64_t *)a + PathSoA::RNG * B, (uint64_t)rng);
    st_path(b + PathSoA::SID * B, id);
}
// The state of position p: slot id, ray, rng, pending hit (who, t), attenuation-stack count, and the depth
// (depth_it: the depth of every path at this bounce).
__device__ __forceinline__ void load_path(const PathSoA &S, uint32_t p, uint32_t *id, Ray *ray, uint64_t *rng,
                                          uint32_t depth_it, uint32_t *depth, uint32_t *count, int *who,
                                          double *best) {
    const double *a = S.d8(p);
    const uint32_t *b = S.d4(p);
    constexpr uint32_t B = PathSoA::BLK;
    *id = ld_path(b + PathSoA::SID * B);
    ray->o = dev::v3(ld_path(a + PathSoA::OX * B), ld_path(a + PathSoA::OY * B), ld_path(a + PathSoA::OZ * B));
    ray->d = dev::v3(ld_path(a + PathSoA::DX * B), ld_path(a + PathSoA::DY * B), ld_path(a + PathSoA::DZ * B));
    *rng = ld_path((const uint64_t *)a + PathSoA::RNG * B);
    const uint32_t w = ld_path(b + PathSoA::WHO * B);
    *who = unpack_who(w);
    *count = w >> 25;
    *depth = depth_it;
    *best = ld_path(a + PathSoA::T * B);
}

// Pixel of a path slot: slot = (s_local * tiles + ti_local) * 256 + thread-in-tile,
// thread-in-tile laid out as render_tiles' 4 waves of 8x8.
__device__ __forceinline__ void slot_pixel(const FrameParams &P, const WfView &v, uint32_t id, uint32_t *x,
                                           uint32_t *y, uint32_t *s_local, uint32_t *pix_local) {
    const uint32_t within = id % v.npix;
    *s_local = id / v.npix;
    *pix_local = within;
    const uint32_t ti = v.tile0 + within / (TILE * TILE);
    const uint32_t th = within % (TILE * TILE);
    const uint32_t k = dev::tile_position(P.rank + ti * P.world, P.tiles_x, P.world);
    const uint32_t tx = k % P.tiles_x, ty = k / P.tiles_x;
    const uint32_t w = th >> 6, l = th & 63;
    *x = tx * TILE + (((w & 1u) << 3) | (l & 7u));
    *y = ty * TILE + (((w >> 1) << 3) | (l >> 3));
}

// points along a march job's chord whose sign of f predicts a hit (queue
// order only; 0: march -25 %, profiles/r3/ab_round3_experiments.txt)
constexpr int WF_PREDICT = 4;

// One bounce for every live path of iteration `it` (it == 0: camera rays).
// DIAG: wave-level s_memtime cycles per section, each section ended by a
// full s_waitcnt so the memory waits it causes are charged to it (tuning
// only): list load, state loads, shade, unwind, trace, march pre-check,
// stores; summed into diag[36..42].
// SPLIT (the large-tree builds without marched shapes, C5): the kernel only shades and stores the new ray; wf_walk
// traces it after the compaction (Tuning::wf_walk).
template <bool FIRST, int WAVES, int FK = march::F_ANY, bool EXT = false, bool BIGBVH = false, bool SPLIT = false>
__global__ __launch_bounds__(256, WAVES) void wf_bounce(const WfArgs *__restrict__ A, int it,
                                                        unsigned long long *diag = nullptr) {
    // input: the id-sorted list of live paths (iteration 0: every slot)
    uint32_t count;
    {
        const WfArgs &a = kargs(A);
        const WfView &v = a.v;
        count = FIRST ? (v.cnt[3] ? 0u : v.ns * v.npix) : v.cnt[it * 4 + 0];
        // a progressive frame's chunk stopped by stop_gate: this launch must find no work
        if (a.P.stop && blockIdx.x == 0 && threadIdx.x == 0 && v.cnt[3]) dev::note_stop(a.sc.guard, count > 0);
    }
    const uint32_t stride = gridDim.x * blockDim.x;
    const bool DIAG = PT_WAVE_DIAG && diag;  // (a diagnostics build with pt_wave_diag enabled)
    unsigned long long dsec[7] = {0, 0, 0, 0, 0, 0, 0}, tst = 0;
    PT_LP_BEGIN();
#define PT_BSTAMP(k)                                                \
    if (DIAG) {                                                     \
        __builtin_amdgcn_s_waitcnt(0);                              \
        const unsigned long long n_ = __builtin_amdgcn_s_memtime(); \
        dsec[k] += n_ - tst;                                        \
        tst = n_;                                                   \
    }
    for (uint32_t base = blockIdx.x * blockDim.x; base < count; base += stride) {
        if (DIAG) tst = __builtin_amdgcn_s_memtime();
        const WfArgs &a = kargs(A);
        const dev::Scene &sc = a.sc;
        const FrameParams &P = a.P;
        const WfView &v = a.v;
        const uint32_t i = base + threadIdx.x;
        bool live = i < count;
        uint32_t id = 0;
        Ray ray;
        dev::Rng rng{0};
        uint32_t depth = 0;
        MemStack stk{v.ids, (size_t)v.cap, 0, nullptr};
        // pending hit of the path (non-first iterations: from the state)
        int who = -1;
        double best = 0.0;
        if (live) {
            if (FIRST) {
                id = i;
                uint32_t x, y, sl, pl;
                slot_pixel(P, v, id, &x, &y, &sl, &pl);
                if (x >= P.width || y >= P.height || sl >= v.ns) {
                    live = false;
                } else {
                    rng.s = dev::sample_key(P.seed, (uint64_t)x + (uint64_t)y * P.width, v.s0 + sl);
                    ray = dev::camera_ray(P, x, y, rng);
                    depth = P.depth;
                    stk.base = v.ids + id;  // (a second bounce in this launch pushes onto it)
                    if (EXT) stk.vb = v.att + id;
                }
            } else {
                const uint32_t p = v.list[i];
                PT_BSTAMP(0)
                uint32_t count;
                // (every live path has been shaded it - 1 times, each a scatter: its depth is P.depth - (it - 1))
                load_path(v.in, p, &id, &ray, &rng.s, P.depth + 1u - (uint32_t)it, &depth, &count, &who, &best);
                stk.base = v.ids + id;
                stk.n = (int)count;
                if (EXT) stk.vb = v.att + id;
                PT_BSTAMP(1)
            }
        }
        // One bounce of this path: shade the pending hit (the camera ray has
        // none), trace the new ray, and find whether a marched shape's bound
        // starts before its best hit.  (Up to 2-3 bounces per launch for paths
        // needing no march measured +0.8 % / -2.5 %, round 2.)
        bool need_march = false, long_job = false;
        V3 jo_o = dev::v3(0.0, 0.0, 0.0), jo_d = jo_o;  // a march job: the object-space ray and bound interval
        double jo_st = 0.0, jo_en = 0.0;
        if (live) {
            PT_LP(LIVE);
            if (!FIRST) {
                V3 leaf;
                const bool ended = dev::shade<false, FK, EXT>(kargs(A).sc, who, best, ray, depth, stk, rng, P.s11, &leaf);
                PT_BSTAMP(2)
                if (ended) {
                    // the leaf radiance and the stack depth; wf_reduce unwinds
                    // the attenuation stack (end_path)
                    PT_LP(ENDED);
                    end_path(v, id, stk, leaf);
                    live = false;
                    PT_BSTAMP(3)
                }
            }
        }
        if (live && SPLIT) {  // the ray is traced by wf_walk
            best = __builtin_inf();
            who = -1;
        } else if (live) {
            PT_LP(TRACE);
            const V3 inv = dev::v3(1.0 / ray.d.x, 1.0 / ray.d.y, 1.0 / ray.d.z);
            best = __builtin_inf();
            who = -1;
            // the hit of this trace is shaded at depth `depth`: at 0 only hit or
            // miss matters (any hit gives black), so a path with a hit found
            // needs no march either
            const bool any = depth == 0;
            dev::closest_nomarch<false, EXT, BIGBVH>(kargs(A).sc, ray, inv, T_MIN, &best, &who, nullptr, any);
            PT_BSTAMP(4)
            // does any marched shape's bound start before the best hit? (the
            // march kernel marches it)
            for (int k = 0; k < sc.nmarch && !need_march && !(any && who >= 0); k++) {
                const int s = dev::uniform_index(dev::uniform_load(&sc.march[k]));
                const DBox bx = dev::uniform_box(&sc.boxes[s]);
                if (!dev::slab(bx.lo, bx.hi, ray, inv, T_MIN, best)) continue;
                PT_LP(PRE_SLAB);
                const DShape S = dev::uniform_shape(&sc.shapes[s]);
                jo_o = dev::xf_point(S.inv, ray.o);
                jo_d = dev::xf_vector(S.inv, ray.d);
                need_march = march::shape_bound_k<FK>(dev::shape_params(S), jo_o.x, jo_o.y, jo_o.z, jo_d.x, jo_d.y,
                                                      jo_d.z, &jo_st, &jo_en);
            }
            PT_BSTAMP(5)
            if (any && !need_march) {
                PT_LP(ANY_END);
                // its shade would end it at once (mod.rs:24-27, 42-44): black
                // after a hit, the background after a miss; only paths whose
                // answer needs a march go on to the last iteration
                end_path(v, id, stk, who >= 0 ? dev::v3(0.0, 0.0, 0.0) : dev::background(ray.d));
                live = false;
            }
        }
        // The wave's surviving paths (live, or waiting for a march) go to consecutive output positions from the
        // wave's first one, in input (= id) order, and the positions after them get status 0: the ended paths'
        // state is not written, and the next bounce gathers from runs with holes only at wave ends (round 5).
        const uint32_t wbase = base + (threadIdx.x & ~63u);
        const uint64_t keep = __ballot(live);
        const uint32_t k = wbase + (uint32_t)__popcll(keep & ((1ull << (threadIdx.x & 63)) - 1ull));
        if (i < count && (threadIdx.x & 63) >= (uint32_t)__popcll(keep)) v.status[i] = 0u;
        if (need_march && v.jo) {  // the march kernel starts from here (one marched shape)
            PT_LP(PRE_JOB);
            // the 64 B record in four 16-byte non-temporal stores (as eight 8-byte ones: the
            // same time; structure of arrays: slower, round 3 jo2)
            typedef double d2v __attribute__((ext_vector_type(2)));
            d2v *j = (d2v *)(v.jo + (size_t)k * 4);
            __builtin_nontemporal_store((d2v){jo_o.x, jo_o.y}, j + 0);
            __builtin_nontemporal_store((d2v){jo_o.z, jo_d.x}, j + 1);
            __builtin_nontemporal_store((d2v){jo_d.y, jo_d.z}, j + 2);
            __builtin_nontemporal_store((d2v){jo_st, jo_en}, j + 3);
            // queue order only: a march that will cross the surface (a hit: ~3x
            // the iterations of a miss) is predicted by the sign of f at the bound
            // entry and at WF_PREDICT points along the chord (inside is f < 0;
            // measured on captured cornell jobs: every predicted job a hit, 0.2 %
            // of the others)
            const march::FParams F = dev::shape_params(dev::uniform_shape(&sc.shapes[dev::uniform_index(
                dev::uniform_load(&sc.march[0]))]));
            const V3 o = jo_o, d = jo_d;
            const double st = jo_st, en = jo_en;
            long_job = march::shape_f_k<FK>(F, o.x + d.x * st, o.y + d.y * st, o.z + d.z * st) < 0.0;
            const double dt = (en - st) * (1.0 / WF_PREDICT);
#pragma unroll
            for (int q = 0; q < WF_PREDICT; q++) {
                const double tq = st + dt * (q + 0.5);
                long_job = long_job || march::shape_f_k<FK>(F, o.x + d.x * tq, o.y + d.y * tq, o.z + d.z * tq) < 0.0;
            }
        }
        if (i < count) PT_LP(STORE);
        if (i < count && live) {
            store_path(v.out, k, id, ray, best, who, rng.s, (uint32_t)stk.n);
            v.status[k] = live ? (need_march ? (long_job ? 7u : 3u) : 1u) : 0u;
        }
        PT_BSTAMP(6)
    }
#undef PT_BSTAMP
    PT_LP_END();
    if (DIAG && (threadIdx.x & 63) == 0)
        for (int k = 0; k < 7; k++) atomicAdd(&diag[36 + k], dsec[k]);
}

// Order-preserving compaction of the status bytes into the two position lists
// (live paths: bit 0, march jobs: bit 1) in three small launches: per-tile
// counts (16 statuses per thread, one 16-byte load), one scan over the tile
// counts, and an ordered scatter.  Neighbouring pixels stay in neighbouring
// lanes, so the next kernels' structure-of-arrays loads stay coalesced and
// march waves coherent.  March jobs the bounce kernel predicts long (bit 2:
// the ray passes close to the marched shape's centre) go first in the queue,
// each class in id order, so the persistent march grid's tail is made of
// short jobs.
constexpr int CP_ITEMS = 16, CP_BLOCK = 256, CP_TILE = CP_ITEMS * CP_BLOCK;

__device__ __forceinline__ void cp_bits(uint4 q, uint32_t *live, uint32_t *march, uint32_t *lng) {
    // statuses are 0, 1, 3 or 7: bit 0 of each byte = live, bit 1 = march, bit 2 = predicted long
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
    uint32_t l = 0, m = 0, g = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        l += __popc(w[k] & 0x01010101u);
        m += __popc(w[k] & 0x02020202u);
        g += __popc(w[k] & 0x04040404u);
    }
    *live = l;
    *march = m;
    *lng = g;
}

// block-wide exclusive scan of one value per thread (256 threads, 4 waves)
__device__ __forceinline__ uint32_t block_exscan(uint32_t x, uint32_t *total, uint32_t *lds /*4*/) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t inc = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63) lds[wv] = inc;
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if ((uint32_t)k < wv) before += lds[k];
        tot += lds[k];
    }
    __syncthreads();
    *total = tot;
    return before + inc - x;
}

// The thread's 16 statuses; positions at or past the bounce's input count n
// (stale bytes of earlier iterations) read as 0.
__device__ __forceinline__ uint4 cp_load(const uint8_t *__restrict__ st, uint32_t tile, uint32_t n) {
    const uint32_t b = tile * CP_TILE + threadIdx.x * CP_ITEMS;
    if (b >= n) return make_uint4(0u, 0u, 0u, 0u);
    uint4 q = reinterpret_cast<const uint4 *>(st + (size_t)tile * CP_TILE)[threadIdx.x];
    if (n - b < (uint32_t)CP_ITEMS) {
        const uint32_t k = n - b;  // bytes kept: 1 .. 15
        uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t keep = k >= 4u * (j + 1) ? 4u : (k > 4u * j ? k - 4u * j : 0u);
            w[j] &= keep >= 4u ? 0xffffffffu : ((1u << (8u * keep)) - 1u);
        }
        q = make_uint4(w[0], w[1], w[2], w[3]);
    }
    return q;
}

// Tile counts live in three arrays (live, long march, short march) of
// per * 256 words, tile b at (b % per) * 256 + b / per with per =
// ceil(tiles / 256): cp_scan's thread t owns tiles t * per .. t * per + per - 1,
// and with this order a wave's loads of its threads' j-th tiles are 64
// consecutive words.  (Tile-major, each load touched 64 lines: the scan took
// 49 us per launch at 48M-path chunks, 12k tiles.)
struct CpLayout {
    uint32_t per, stride;  // tiles per scan thread, words per class array (per * 256)
    __host__ __device__ static CpLayout of(uint32_t tiles) {
        const uint32_t per = (tiles + CP_BLOCK - 1) / CP_BLOCK;
        return CpLayout{per ? per : 1u, (per ? per : 1u) * CP_BLOCK};
    }
    __device__ uint32_t at(uint32_t b) const { return (b % per) * CP_BLOCK + b / per; }
};

// The compaction kernels cover the tiles of the bounce's input count n (read
// on the device) with at most CP_GRID blocks, each looping over tiles: a late
// iteration's few live paths no longer launch a grid of the chunk's size
// (three launches of ~11k blocks cost ~40 us even with nothing to do, round 5).
constexpr uint32_t CP_GRID = 2048;
__device__ __forceinline__ uint32_t cp_n(const uint32_t *n_dev, uint32_t n_host) { return n_dev ? *n_dev : n_host; }

// per tile: (live, long march, short march) counts
__global__ __launch_bounds__(256) void cp_count(const uint8_t *__restrict__ st, uint32_t *__restrict__ blk, CpLayout L,
                                                const uint32_t *__restrict__ n_dev, uint32_t n_host) {
    __shared__ uint32_t lds[12];
    const uint32_t n = cp_n(n_dev, n_host), nt = (n + CP_TILE - 1) / CP_TILE;
    for (uint32_t tb = blockIdx.x; tb < nt; tb += gridDim.x) {  // (block-uniform)
        const uint4 q = cp_load(st, tb, n);
        uint32_t l, m, g, tl, tg, ts;
        cp_bits(q, &l, &m, &g);
        block_exscan(l, &tl, lds);
        block_exscan(g, &tg, lds + 4);
        block_exscan(m - g, &ts, lds + 8);
        if (threadIdx.x == 0) {
            const uint32_t k = L.at(tb);
            blk[k] = tl;
            blk[L.stride + k] = tg;
            blk[2 * L.stride + k] = ts;
        }
    }
}

// one block: exclusive scan of the tile counts in place; totals go to the
// counters the next kernels read (n_long: where the short march jobs start).
// Each thread owns a contiguous run of `per` tiles (CpLayout: coalesced across
// the wave), loaded into registers up front (every load in flight together)
// when the run is at most SCAN_RUN tiles, and the block scans once.
constexpr int SCAN_RUN = 48;
__global__ __launch_bounds__(256) void cp_scan(uint32_t *__restrict__ blk, uint32_t nblk_max, CpLayout L,
                                               const uint32_t *__restrict__ n_dev, uint32_t n_host,
                                               uint32_t *__restrict__ n_live, uint32_t *__restrict__ n_march,
                                               uint32_t *__restrict__ n_long) {
    __shared__ uint32_t lds[12];
    const uint32_t nt = (cp_n(n_dev, n_host) + CP_TILE - 1) / CP_TILE;
    const uint32_t nblk = nt < nblk_max ? nt : nblk_max;  // the tiles cp_count wrote
    const uint32_t per = L.per;
    const uint32_t b0 = threadIdx.x * per;
    const uint32_t nj = b0 >= nblk ? 0u : (nblk - b0 < per ? nblk - b0 : per);  // this thread's tiles
    uint32_t *bl = blk + threadIdx.x, *bg = bl + L.stride, *bs = bg + L.stride;  // tile j at [j * 256]
    uint32_t sl = 0, sg = 0, ss = 0, tl, tg, ts;
    if (per <= (uint32_t)SCAN_RUN) {  // (block-uniform)
        uint32_t rl[SCAN_RUN], rg[SCAN_RUN], rs[SCAN_RUN];
#pragma unroll
        for (int j = 0; j < SCAN_RUN; j++) {
            const bool ok = (uint32_t)j < nj;
            rl[j] = ok ? bl[j * CP_BLOCK] : 0u;
            rg[j] = ok ? bg[j * CP_BLOCK] : 0u;
            rs[j] = ok ? bs[j * CP_BLOCK] : 0u;
        }
#pragma unroll
        for (int j = 0; j < SCAN_RUN; j++) sl += rl[j], sg += rg[j], ss += rs[j];
        uint32_t cl = block_exscan(sl, &tl, lds), cg = block_exscan(sg, &tg, lds + 4), cs = block_exscan(ss, &ts, lds + 8);
#pragma unroll
        for (int j = 0; j < SCAN_RUN; j++) {
            if ((uint32_t)j < nj) {
                bl[j * CP_BLOCK] = cl;
                bg[j * CP_BLOCK] = cg;
                bs[j * CP_BLOCK] = cs;
            }
            cl += rl[j];
            cg += rg[j];
            cs += rs[j];
        }
    } else {
#pragma unroll 8
        for (uint32_t j = 0; j < nj; j++) {
            sl += bl[j * CP_BLOCK];
            sg += bg[j * CP_BLOCK];
            ss += bs[j * CP_BLOCK];
        }
        uint32_t cl = block_exscan(sl, &tl, lds), cg = block_exscan(sg, &tg, lds + 4), cs = block_exscan(ss, &ts, lds + 8);
#pragma unroll 8
        for (uint32_t j = 0; j < nj; j++) {
            const uint32_t l = bl[j * CP_BLOCK], g = bg[j * CP_BLOCK], h = bs[j * CP_BLOCK];
            bl[j * CP_BLOCK] = cl;
            bg[j * CP_BLOCK] = cg;
            bs[j * CP_BLOCK] = cs;
            cl += l;
            cg += g;
            cs += h;
        }
    }
    if (threadIdx.x == 0) {
        *n_live = tl;
        *n_march = tg + ts;
        *n_long = tg;
    }
}

// Progressive frames only (FrameParams::stop set): at a chunk's start (it < 0)
// and after each compaction, one lane reads the renderer's host-mapped stop
// flag; set, the chunk's stop mark goes up and the compaction's counts go to
// zero, so the chunk's remaining launches find no work.  One host-link read
// per launch, not one per wave of the hot kernels.
__global__ __launch_bounds__(64) void stop_gate(const int *stop, uint32_t *__restrict__ cnt, int it) {
    if (threadIdx.x != 0 || !dev::stopped(stop)) return;
    cnt[3] = 1u;
    if (it >= 0) cnt[(it + 1) * 4 + 0] = cnt[it * 4 + 1] = cnt[it * 4 + 2] = 0u;
}

// The tile's ids are compacted into LDS first (in order), then copied out
// with consecutive lanes on consecutive positions (one thread's 16 statuses
// scattered straight to HBM would touch 64 lines per wave store).
__global__ __launch_bounds__(256) void cp_scatter(const uint8_t *__restrict__ st, const uint32_t *__restrict__ blk,
                                                  CpLayout L, const uint32_t *__restrict__ n_long, uint32_t *__restrict__ live_out,
                                                  uint32_t *__restrict__ march_out, const uint32_t *__restrict__ n_dev,
                                                  uint32_t n_host) {
    __shared__ uint32_t lds[12];
    __shared__ uint32_t ids[CP_TILE];  // the tile's live ids, then its march ids (long, then short)
    const uint32_t n = cp_n(n_dev, n_host), nt = (n + CP_TILE - 1) / CP_TILE;
    for (uint32_t tb = blockIdx.x; tb < nt; tb += gridDim.x) {  // (block-uniform)
        const size_t base = (size_t)tb * CP_TILE + (size_t)threadIdx.x * CP_ITEMS;
        const uint4 q = cp_load(st, tb, n);
        uint32_t l, m, g, tl, tg, ts;
        cp_bits(q, &l, &m, &g);
        uint32_t ol = block_exscan(l, &tl, lds);  // (its barriers also end the previous tile's reads of ids)
        uint32_t og = block_exscan(g, &tg, lds + 4);
        uint32_t os = tg + block_exscan(m - g, &ts, lds + 8);
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int k = 0; k < CP_ITEMS; k++)
            if ((w[k >> 2] >> (8 * (k & 3))) & 1u) ids[ol++] = (uint32_t)(base + k);
        __syncthreads();
        const uint32_t kb = L.at(tb);
        const uint32_t bl = blk[kb], bg = blk[L.stride + kb], bs = *n_long + blk[2 * L.stride + kb];
        for (uint32_t k = threadIdx.x; k < tl; k += CP_BLOCK) live_out[bl + k] = ids[k];
        if (tg + ts == 0) continue;  // (block-uniform)
        __syncthreads();
#pragma unroll
        for (int k = 0; k < CP_ITEMS; k++) {
            const uint32_t b = (w[k >> 2] >> (8 * (k & 3))) & 0xffu;
            if (b & 2u) ids[(b & 4u) ? og++ : os++] = (uint32_t)(base + k);
        }
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < tg; k += CP_BLOCK) march_out[bg + k] = ids[k];
        for (uint32_t k = threadIdx.x; k < ts; k += CP_BLOCK) march_out[bs + k] = ids[tg + k];
    }
}

// Marches of iteration `it`.  Each workgroup owns a contiguous slice of the
// (id-sorted) march queue and hands jobs to its lanes through an LDS counter;
// the marched shapes' select data (padded box, inverse transform, step,
// passes) is staged in LDS once per workgroup.  A job is trace_pixel's
// SELECT/MARCH loop over the marched shapes for one path; (best, who) go back
// to the path, which the next bounce kernel reads from the live list.
// Measured and dropped (profiles/r2/ab_round2_experiments.txt): a per-wave phase vote,
// batched job switches, several march units per trip, non-temporal result stores.
constexpr uint32_t WF_BOUNCE_CAP = 8192;  // bounce grid (blocks) after the first iteration; threads loop over the live list
// waves per SIMD the march kernel's registers must allow (C2: 5 waves spill 100 B/lane: 1187; 4: 128 VGPRs,
// 20 B: 1273; 3: 1261 M samples/s, round 1)
constexpr int WF_MARCH_WAVES = 4;
struct MarchJob {
    uint32_t id;
    Ray ray;
    double best;
    int who;
    uint32_t hi;  // the stack-count bits of the who word, written back unchanged
};
__device__ __forceinline__ void job_who(MarchJob *j, uint32_t w) {
    j->who = unpack_who(w);
    j->hi = w & ~WHO_MASK;
}
__device__ __forceinline__ uint32_t job_who_word(int who, uint32_t hi) {
    return (uint32_t)(who + 1) | hi;
}

__device__ __forceinline__ void load_job(const PathSoA &S, uint32_t p, MarchJob *j) {
    const double *a = S.d8(p);
    constexpr uint32_t B = PathSoA::BLK;
    j->id = p;
    j->ray.o = dev::v3(a[PathSoA::OX * B], a[PathSoA::OY * B], a[PathSoA::OZ * B]);
    j->ray.d = dev::v3(a[PathSoA::DX * B], a[PathSoA::DY * B], a[PathSoA::DZ * B]);
    j->best = S.t(p);
    job_who(j, S.who(p));
}

// DIAG: per trip, the set of phase kinds present among the wave's lanes (bit
// 0 cheap, 1 select, 2 advance, 3 proof), lanes per kind and the trip's
// s_memtime cycles, summed per wave into diag[0..35] (tuning only).
template <int FK = march::F_ANY>
__global__ __launch_bounds__(256, WF_MARCH_WAVES) void wf_march(const WfArgs *__restrict__ A, int it,
                                                                   unsigned long long *diag, uint32_t slice_max) {
    __shared__ uint32_t head;
    const bool DIAG = PT_WAVE_DIAG && diag;  // (a diagnostics build with pt_wave_diag enabled)
    const WfArgs &a0 = kargs(A);
    const int nm = a0.sc.nmarch;
    const uint32_t count = a0.v.cnt[it * 4 + 1];
    if (a0.P.stop && blockIdx.x == 0 && threadIdx.x == 0 && a0.v.cnt[3]) dev::note_stop(a0.sc.guard, count > 0);
    // The block's jobs: local index q = 0, 1, ... maps to the queue position
    // pos(q).  slice == 0: one contiguous slice of the queue per block.
    // slice > 0: runs of `slice` consecutive jobs dealt round-robin to the
    // blocks, so a heavy region of the (pixel-sorted) queue is shared by many
    // blocks while each run stays pixel-coherent.  A queue shorter than
    // slice_max runs per block is dealt in shorter runs (count / blocks), so
    // the few jobs of a late iteration spread over the CUs instead of sharing
    // one block's waves: each wave's trips then cost only its own jobs' code
    // (a persistent launch lasts as long as its slowest wave; round 5).
    const uint32_t slice = slice_max == 0 ? 0u
                           : (count / gridDim.x < slice_max ? max(1u, count / gridDim.x) : slice_max);
    uint32_t per, lo;
    if (slice == 0) {
        per = (count + gridDim.x - 1) / gridDim.x;
        lo = blockIdx.x * per;
    } else {
        const uint32_t runs = (count + slice - 1) / slice;
        const uint32_t mine = runs > blockIdx.x ? (runs - blockIdx.x + gridDim.x - 1) / gridDim.x : 0u;
        per = mine * slice;
        lo = 0;
    }
    const uint32_t G = gridDim.x;
    auto pos = [&](uint32_t q) -> uint32_t {
        return slice == 0 ? lo + q : (q / slice * G + blockIdx.x) * slice + q % slice;
    };
    const uint32_t hi = slice == 0 ? min(count, lo + per) : per;
    if (slice == 0) per = hi > lo ? hi - lo : 0u;
    if (threadIdx.x == 0) head = blockDim.x;
    __syncthreads();
    // A queue of fewer jobs than the grid has lanes (the late iterations) is
    // dealt in runs of kw = ceil(count / waves) consecutive jobs, one run per
    // wave (wave w of block b: run w * blocks + b), one job per lane and no
    // refill: every wave of the grid takes part, each with the fewest jobs.  A
    // trip of a wave costs the union of its lanes' march phases, and the launch
    // lasts as long as its slowest wave: dealt per block, a late queue of ~10
    // jobs per block put them all in the block's first wave (round 5).
    const uint32_t nwv = blockDim.x >> 6;
    const bool runs_w = slice_max != 0 && count < G * blockDim.x;
    const uint32_t kw = runs_w ? (count + G * nwv - 1) / (G * nwv) : 0u;
    const uint32_t pw = ((threadIdx.x >> 6) * G + blockIdx.x) * kw + (threadIdx.x & 63);
    uint32_t q = threadIdx.x;
    bool have = runs_w ? (threadIdx.x & 63) < kw && pw < count : q < per && pos(q) < count;
    // one marched shape and jobs pre-selected by the bounce kernel: a job is
    // its march alone (no select, no ray transform, no bound quadratic here)
    const bool pre = a0.v.jo != nullptr;
    int s0 = 0, passes0 = 0;
    double step0 = 0.0;
    march::FParams F0{};
    if (pre) {
        s0 = dev::uniform_load(&a0.sc.march[0]);
        const DShape S = dev::uniform_shape(&a0.sc.shapes[s0]);
        F0 = dev::shape_params(S);
        step0 = S.p[0];
        passes0 = S.depth;
    }
    MarchJob cur;
    march::MarchState ms;
    bool marching = false;
    int km = 0, mshape = -1;
    auto start_job = [&](const WfView &v, uint32_t k) {  // k: queue position
        const uint32_t id = v.mq[k];  // position in the bounce's output
        if (pre) {
            cur.id = id;
            cur.best = v.out.t(id);
            job_who(&cur, v.out.who(id));
            const double2 *j = v.jo + (size_t)id * 4;
            const double2 a = j[0], b = j[1], c = j[2], e = j[3];
            march::march_start<FK>(F0, step0, passes0, a.x, a.y, b.x, b.y, c.x, c.y, e.x, e.y, &ms);
            marching = true;
            mshape = s0;
        } else {
            load_job(v.out, id, &cur);
        }
    };
    PT_MREG_KERNEL_BEGIN();
    if (have) start_job(a0.v, runs_w ? pw : pos(q));
    V3 inv = pre ? dev::v3(0.0, 0.0, 0.0) : dev::v3(1.0 / cur.ray.d.x, 1.0 / cur.ray.d.y, 1.0 / cur.ray.d.z);
    march::MarchStats mst{0, 0, 0, 0};
    unsigned long long dtrips[16], dcyc[16], dlanes[4];
    if (DIAG) {
        for (int k = 0; k < 16; k++) dtrips[k] = dcyc[k] = 0;
        for (int k = 0; k < 4; k++) dlanes[k] = 0;
    }
    unsigned long long t_prev = DIAG ? __builtin_amdgcn_s_memtime() : 0;
    int mask_prev = -1;
    while (DIAG ? __ballot(have) != 0 : have) {
        if (DIAG) {
            const unsigned long long now = __builtin_amdgcn_s_memtime();
            if (mask_prev >= 0) {
                dtrips[mask_prev]++;
                dcyc[mask_prev] += now - t_prev;
            }
            t_prev = now;
            const int phd = !have ? -1 : (marching ? march::march_phase(ms) : 3);
            const int kind = phd < 0 ? -1 : (phd == 3 ? 1 : (phd == march::MP_CHEAP ? 0 : (phd == march::MP_ADV ? 2 : 3)));
            int mk = 0;
            for (int k = 0; k < 4; k++) {
                const uint64_t b = __ballot(kind == k);
                if (b) mk |= 1 << k;
                dlanes[k] += __popcll(b);
            }
            mask_prev = mk;
        }
        if (!have) continue;
        // one unit of work per trip: a march iteration, a select step or a job switch
        {
            bool done = false;
            if (marching) {
                PT_MREG_STEP_BEGIN();
                const int st = march::march_step<false, true, FK>(ms, &mst);
                PT_MREG_STEP_END();
                if (st != march::M_RUNNING) {
                    if (st == march::M_GUARD) dev::note_guard(kargs(A).sc.guard);
                    // final test of ray_marching.rs:55-57 against [T_MIN, best], then the tie rule
                    if (st == march::M_DONE && !(ms.t < T_MIN || ms.t > cur.best) &&
                        (ms.t < cur.best || mshape > cur.who)) {
                        cur.best = ms.t;
                        cur.who = mshape;
                    }
                    marching = false;
                    done = pre;  // the job's only shape
                }
            } else {
                // select: next marched shape whose bound is entered before `best`
                const dev::Scene &sc = kargs(A).sc;
                while (km < nm) {
                    const int s = sc.march[km++];
                    const DBox &b = sc.boxes[s];
                    if (!dev::slab(b.lo, b.hi, cur.ray, inv, T_MIN, cur.best)) continue;
                    const DShape &S = sc.shapes[s];
                    const V3 o = dev::xf_point(S.inv, cur.ray.o), d = dev::xf_vector(S.inv, cur.ray.d);
                    if (march::march_begin<FK>(dev::shape_params(S), S.p[0], S.depth, o.x, o.y, o.z, d.x, d.y,
                                               d.z, &ms)) {
                        mshape = s;
                        marching = true;
                        break;
                    }
                }
                done = !marching;
            }
            if (done) {
                PT_MREG_REFILL_BEGIN();
                // vmcnt counts loads and stores in issue order: a store issued
                // before the next job's loads makes the wait for those loads a
                // wait for the store's completion too, so the finished job's
                // results are stored after the next job's loads are issued
                const uint32_t fid = cur.id;
                const double fbest = cur.best;
                const uint32_t fwho = job_who_word(cur.who, cur.hi);
                const WfView &v = kargs(A).v;
                if (runs_w) {
                    have = false;
                } else {
                    q = atomicAdd(&head, 1u);
                    have = q < per && pos(q) < count;
                    if (have) start_job(v, pos(q));
                }
                v.out.t(fid) = fbest;
                v.out.who(fid) = fwho;
                if (have && !pre) {
                    inv = dev::v3(1.0 / cur.ray.d.x, 1.0 / cur.ray.d.y, 1.0 / cur.ray.d.z);
                    km = 0;
                }
                PT_MREG_REFILL_END();
            }
        }
    }
    PT_MREG_KERNEL_END();
    if (DIAG && (threadIdx.x & 63) == 0) {
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        if (mask_prev >= 0) {
            dtrips[mask_prev]++;
            dcyc[mask_prev] += now - t_prev;
        }
        for (int k = 0; k < 16; k++) {
            atomicAdd(&diag[k], dtrips[k]);
            atomicAdd(&diag[16 + k], dcyc[k]);
        }
        for (int k = 0; k < 4; k++) atomicAdd(&diag[32 + k], dlanes[k]);
    }
}

// The BVH walk of the large-tree scenes without marched shapes (C5) as its own
// kernel (Tuning::wf_walk, round 5): the walk is latency-bound (a chain of
// dependent node loads per lane, ~70 % of the bounce's wave cycles waiting on
// memory), and inside the bounce kernel its lanes run at the bounce's register
// budget (118 VGPRs: 4 waves per SIMD).  Alone it needs far fewer registers,
// so more waves -- more independent node chains -- are in flight per SIMD.
// It runs after the compaction of iteration it, over the live list of it + 1:
// the ray each bounce stored, traced through the uniform list and the BVH
// (closest_nomarch, the same code and tie rule as the bounce's trace), and
// (best, who) written back in place; the next bounce shades them.
// QN: the walk reads the quantized 16-byte nodes (DNodeQ; a tree without them takes the 32-byte DNodeC).
template <int WAVES, bool QN>
__global__ __launch_bounds__(256, WAVES) void wf_walk(const WfArgs *__restrict__ A, int it) {
    __shared__ uint32_t pos[256];      // the block's list positions, grouped by octant
    constexpr uint32_t NB = 9u;  // groups: the 8 octants, and the last for no ray
    __shared__ uint32_t wcount[4][NB];  // rays per (wave, group)
    const uint32_t count = kargs(A).v.cnt[(it + 1) * 4 + 0];
    const uint32_t stride = gridDim.x * blockDim.x;
    // the trace after bounce it is shaded at depth P.depth - it: at 0 only hit or miss matters
    const bool any = kargs(A).P.depth == (uint32_t)it;
    // (an XCD-aware block order, each XCD walking a contiguous eighth of every grid-wide round, measured slower:
    // round 5)
    for (uint32_t base = blockIdx.x * blockDim.x; base < count; base += stride) {  // (block-uniform)
        const WfArgs &a = kargs(A);
        const WfView &v = a.v;
        const uint32_t i = base + threadIdx.x;
        constexpr uint32_t B = PathSoA::BLK;
        uint32_t p;
        {
            // Counting sort of the block's rays by the octant of their direction (the BVH layout they walk),
            // stable, so each group keeps the list's pixel order: a wave then walks one or two layouts with
            // neighbouring origins instead of up to eight (the rays after a diffuse bounce spread over the
            // hemisphere's octants; octant and major axis, 24 groups, scattered the pixel order: slower, r5s).
            const uint32_t q = i < count ? v.list[i] : 0u;
            const double *d = v.out.d8(q);
            const double dx = d[PathSoA::DX * B], dy = d[PathSoA::DY * B], dz = d[PathSoA::DZ * B];
            uint32_t oct = (__builtin_signbit(dx) ? 1u : 0u) | (__builtin_signbit(dy) ? 2u : 0u) |
                           (__builtin_signbit(dz) ? 4u : 0u);
            if (i >= count) oct = NB - 1u;
            const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
            uint32_t rank = 0;
            for (uint32_t o = 0; o < NB; o++) {
                const uint64_t m = __ballot(oct == o);
                if (oct == o) rank = (uint32_t)__popcll(m & ((1ull << ln) - 1ull));
                if (ln == 0) wcount[wv][o] = (uint32_t)__popcll(m);
            }
            __syncthreads();
            uint32_t at = 0;  // rays of lower groups in the block, then of this group in earlier waves
            for (uint32_t o = 0; o < NB; o++)
                for (uint32_t w2 = 0; w2 < 4; w2++) at += (o < oct || (o == oct && w2 < wv)) ? wcount[w2][o] : 0u;
            pos[at + rank] = q;
            __syncthreads();
            p = pos[threadIdx.x];
            __syncthreads();  // (pos and wcount are rewritten by the next trip)
        }
        if (i < count) {  // (the block's first count - base positions hold its rays)
            const double *d = v.out.d8(p);
            Ray ray;
            ray.o = dev::v3(d[PathSoA::OX * B], d[PathSoA::OY * B], d[PathSoA::OZ * B]);
            ray.d = dev::v3(d[PathSoA::DX * B], d[PathSoA::DY * B], d[PathSoA::DZ * B]);
            const V3 inv = dev::v3(1.0 / ray.d.x, 1.0 / ray.d.y, 1.0 / ray.d.z);
            double best = __builtin_inf();
            int who = -1;
            dev::closest_nomarch<false, false, true, QN>(a.sc, ray, inv, T_MIN, &best, &who, nullptr, any);
            v.out.t(p) = best;
            uint32_t &w = v.out.who(p);
            w = (w & ~WHO_MASK) | (uint32_t)(who + 1);
        }
    }
}

// In-order per-pixel sum of the chunk's samples; mean after the last chunk (a
// sample window's running sums instead when it ends short of spp).
// Each sample's radiance is first unwound from its path's end: the leaf
// radiance times the attenuations its stack holds, in the recursion's order
// (dev::unwind; end_path left the leaf and the stack depth).  Sample by
// sample: a version unwinding 8 samples level by level together needs more
// registers and measured slower (the kernel is latency-bound: occupancy wins).
constexpr uint32_t UNWIND_PIXELS = 1u << 18;  // chunks of fewer pixels unwind in their own pass (wf_unwind)
// The unwind of every slot of the chunk, one thread per slot, in place (the leaf record's radiance becomes the
// sample's): a thread per pixel unwinding its samples one after another waits for two dependent loads per sample.
template <bool EXT>
__global__ __launch_bounds__(256) void wf_unwind(const WfArgs *__restrict__ A) {
    const WfArgs &args = kargs(A);
    const WfView &v = args.v;
    if (v.cnt[3]) return;  // a stopped frame's chunk
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= v.ns * v.npix) return;
    const uint32_t pl = id % v.npix;
    uint32_t x, y, sl, pl2;
    slot_pixel(args.P, v, pl, &x, &y, &sl, &pl2);
    if (x >= args.P.width || y >= args.P.height) return;
    double *rec = v.leaf + (size_t)id * 4;
    const uint32_t fin = (uint32_t)__builtin_bit_cast(uint64_t, rec[3]);
    if (fin == 0) return;
    MemStack stk{v.ids + id, (size_t)v.cap, (int)fin, EXT ? v.att + id : nullptr};
    const V3 c = unwind_mem<EXT>(args.sc, stk, dev::v3(rec[0], rec[1], rec[2]));
    rec[0] = c.x;
    rec[1] = c.y;
    rec[2] = c.z;
}

template <bool EXT, bool UNWOUND = false>
__global__ __launch_bounds__(256) void wf_reduce(const WfArgs *__restrict__ A, int first, int last,
                                                 double *__restrict__ out) {
    const WfArgs &args = kargs(A);
    const dev::Scene &sc = args.sc;
    const FrameParams &P = args.P;
    const WfView &v = args.v;
    const uint32_t pl = blockIdx.x * blockDim.x + threadIdx.x;
    if (v.cnt[3]) {  // a stopped frame's chunk: nothing to sum
        if (P.stop && pl == 0) dev::note_stop(sc.guard, false);
        return;
    }
    if (pl >= v.npix) return;
    uint32_t x, y, sl, pl2;
    slot_pixel(P, v, pl, &x, &y, &sl, &pl2);
    const uint32_t ti = v.tile0 + pl / (TILE * TILE), th = pl % (TILE * TILE);
    const uint32_t w = th >> 6, l = th & 63;
    const uint32_t lx = ((w & 1u) << 3) | (l & 7u), ly = ((w >> 1) << 3) | (l >> 3);
    double *dst = P.compact ? out + ((size_t)ti * (TILE * TILE) + ly * TILE + lx) * 3
                            : out + ((size_t)y * P.width + x) * 3;
    if (x >= P.width || y >= P.height) {
        if (P.compact && last) dst[0] = dst[1] = dst[2] = 0.0;
        return;
    }
    V3 a = first == 1   ? dev::v3(0.0, 0.0, 0.0)
           : first == 2 ? dev::v3(dst[0], dst[1], dst[2])
                        : dev::v3(v.acc[pl * 3 + 0], v.acc[pl * 3 + 1], v.acc[pl * 3 + 2]);
    if (UNWOUND) {
#pragma unroll 4
        for (uint32_t s = 0; s < v.ns; s++) {
            const double *rec = v.leaf + ((size_t)s * v.npix + pl) * 4;
            a = dev::add(a, dev::v3(rec[0], rec[1], rec[2]));
        }
    } else
    for (uint32_t s = 0; s < v.ns; s++) {
        const size_t id = (size_t)s * v.npix + pl;
        const double *rec = v.leaf + id * 4;
        const uint32_t fin = (uint32_t)__builtin_bit_cast(uint64_t, rec[3]);
        MemStack stk{v.ids + id, (size_t)v.cap, (int)fin, EXT ? v.att + id : nullptr};
        a = dev::add(a, unwind_mem<EXT>(sc, stk, dev::v3(rec[0], rec[1], rec[2])));
    }
    if (last) {
        const V3 c = last == 2 ? a : dev::divs(a, (double)P.spp);
        dst[0] = c.x;
        dst[1] = c.y;
        dst[2] = c.z;
    } else {
        v.acc[pl * 3 + 0] = a.x;
        v.acc[pl * 3 + 1] = a.y;
        v.acc[pl * 3 + 2] = a.z;
    }
}

// ------------------------------------------------------------- kernel timer
struct KernelTimer {
    struct Rec {
        int kind;
        hipEvent_t a, b;
    };
    std::vector<Rec> recs;
    std::vector<hipEvent_t> pool;
    size_t used = 0;
    hipEvent_t get() {
        if (used == pool.size()) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
            pool.push_back(e);
        }
        return pool[used++];
    }
};
KernelTimer *timer_new() { return new KernelTimer; }
void timer_free(KernelTimer *t) {
    if (!t) return;
    for (auto e : t->pool) (void)hipEventDestroy(e);
    delete t;
}
hipError_t timer_begin(KernelTimer *t, hipStream_t st, int kind) {
    if (!t) return hipSuccess;
    KernelTimer::Rec r{kind, t->get(), t->get()};
    if (!r.a || !r.b) return hipErrorOutOfMemory;
    t->recs.push_back(r);
    return hipEventRecord(r.a, st);
}
hipError_t timer_end(KernelTimer *t, hipStream_t st) {
    if (!t || t->recs.empty()) return hipSuccess;
    return hipEventRecord(t->recs.back().b, st);
}
hipError_t timer_collect(KernelTimer *t, double *ms, uint32_t *launches) {
    for (int k = 0; k < K_KINDS; k++) ms[k] = 0.0, launches[k] = 0;
    if (!t) return hipSuccess;
    for (auto &r : t->recs) {
        hipError_t e = hipEventSynchronize(r.b);
        if (e != hipSuccess) return e;
        float x = 0.f;
        e = hipEventElapsedTime(&x, r.a, r.b);
        if (e != hipSuccess) return e;
        ms[r.kind] += x;
        launches[r.kind]++;
    }
    t->recs.clear();
    t->used = 0;
    return hipSuccess;
}

// ------------------------------------------------------------- host driver
static void free_args(WaveWorkspace *ws);
void wave_workspace_free(WaveWorkspace *ws) {
    for (int k = 0; k < WaveWorkspace::MAX_SLOTS - 1; k++) {
        if (ws->side[k]) (void)hipStreamDestroy(ws->side[k]);
        if (ws->join[k]) (void)hipEventDestroy(ws->join[k]);
        ws->side[k] = nullptr;
        ws->join[k] = nullptr;
    }
    free_args(ws);
    if (ws->fork) (void)hipEventDestroy(ws->fork);
    if (ws->reduced) (void)hipEventDestroy(ws->reduced);
    if (ws->done) (void)hipEventDestroy(ws->done);
    if (ws->args_ev) (void)hipEventDestroy(ws->args_ev);
    ws->fork = ws->reduced = ws->done = ws->args_ev = nullptr;
    ws->used = false;
    timer_free(ws->timer);
    ws->timer = nullptr;
    if (ws->diag) (void)hipFree(ws->diag);
    ws->diag = nullptr;
    if (ws->base) (void)hipFree(ws->base);
    ws->base = nullptr;
    ws->bytes = 0;
}

// The launches' argument blocks: a pinned host staging buffer and its device copy (render_wave).
static void free_args(WaveWorkspace *ws) {
    if (ws->args_pending && ws->args_ev) (void)hipEventSynchronize(ws->args_ev);
    if (ws->args_host) (void)hipHostFree(ws->args_host);
    if (ws->args_dev) (void)hipFree(ws->args_dev);
    ws->args_host = ws->args_dev = nullptr;
    ws->args_bytes = 0;
    ws->args_pending = false;
}

static hipError_t reserve_args(WaveWorkspace *ws, size_t bytes) {
    hipError_t e;
    // the staging buffer is free again once the previous frame's copy has run
    if (ws->args_pending) {
        if ((e = hipEventSynchronize(ws->args_ev)) != hipSuccess) return e;
        ws->args_pending = false;
    }
    if (bytes <= ws->args_bytes) return hipSuccess;
    // growing: the previous frame's kernels must be done with the device blocks
    if (ws->used && (e = hipEventSynchronize(ws->done)) != hipSuccess) return e;
    free_args(ws);
    if (bytes < ((size_t)64 << 10)) bytes = (size_t)64 << 10;
    if ((e = hipHostMalloc(&ws->args_host, bytes, hipHostMallocDefault)) != hipSuccess) {
        ws->args_host = nullptr;
        return e;
    }
    if ((e = hipMalloc(&ws->args_dev, bytes)) != hipSuccess) {
        ws->args_dev = nullptr;
        free_args(ws);
        return e;
    }
    ws->args_bytes = bytes;
    return hipSuccess;
}

static hipError_t reserve(WaveWorkspace *ws, size_t bytes) {
    if (bytes <= ws->bytes) return hipSuccess;
    // grow the path storage only; an enabled timer or diag buffer stays.  The
    // previous frame (possibly on another stream) must be done with it first.
    if (ws->used) {
        hipError_t e = hipEventSynchronize(ws->done);
        if (e != hipSuccess) return e;
    }
    if (ws->base) (void)hipFree(ws->base);
    ws->base = nullptr;
    ws->bytes = 0;
    hipError_t e = hipMalloc(&ws->base, bytes);
    if (e != hipSuccess) {
        ws->base = nullptr;
        return e;
    }
    ws->bytes = bytes;
    return hipSuccess;
}

// BVH nodes per octant layout from which the bounce runs its FMA_SLAB build
// (dev::closest_nomarch): C5's 100k-sphere tree has ~200k, cornell's ~960.
// The scenes whose BVH walk runs in wf_walk (Tuning::wf_walk): a large tree and no marched shape (C5).
static bool walk_split(const dev::Scene &sc, const Tuning &tu) {
    return tu.wf_walk && !sc.ext && sc.nnodes >= BIG_BVH_NODES && sc.nmarch == 0;
}

template <bool FIRST>
static void launch_bounce(uint32_t blocks, hipStream_t st, const dev::Scene &sc, const WfArgs *A, int it,
                          unsigned long long *diag, int fkind, int waves, bool split) {
    if (split) {  // shade and store the new ray only: wf_walk traces it
        switch (waves) {
        case 4: wf_bounce<FIRST, 4, march::F_NONE, false, true, true><<<blocks, 256, 0, st>>>(A, it); break;
        case 5: wf_bounce<FIRST, 5, march::F_NONE, false, true, true><<<blocks, 256, 0, st>>>(A, it); break;
        default: wf_bounce<FIRST, 3, march::F_NONE, false, true, true><<<blocks, 256, 0, st>>>(A, it); break;
        }
        return;
    }
    if (sc.ext) {  // non-solid textures or a Torus: the generic extended build
        wf_bounce<FIRST, 2, march::F_ANY, true><<<blocks, 256, 0, st>>>(A, it);
        return;
    }
    if (fkind != march::F_HEART) {  // another ray-marched function: the generic build
        wf_bounce<FIRST, 2, march::F_ANY><<<blocks, 256, 0, st>>>(A, it);
        return;
    }
    if (PT_WAVE_DIAG && diag) {  // (diagnostics builds)
        wf_bounce<FIRST, 2, march::F_HEART><<<blocks, 256, 0, st>>>(A, it, diag);
        return;
    }
    if (sc.nnodes >= BIG_BVH_NODES && sc.nmarch == 0) {  // a large BVH and no marched shape (C5): the FMA slab
        switch (waves) {                                   // build without march pre-check or Heart code
        case 4: wf_bounce<FIRST, 4, march::F_NONE, false, true><<<blocks, 256, 0, st>>>(A, it); break;
        case 5: wf_bounce<FIRST, 5, march::F_NONE, false, true><<<blocks, 256, 0, st>>>(A, it); break;
        default: wf_bounce<FIRST, 3, march::F_NONE, false, true><<<blocks, 256, 0, st>>>(A, it); break;
        }
        return;
    }
    if (waves == 3 && sc.nnodes >= BIG_BVH_NODES) {  // the default budget, a large BVH with a marched shape
        wf_bounce<FIRST, 3, march::F_HEART, false, true><<<blocks, 256, 0, st>>>(A, it);
        return;
    }
    switch (waves) {  // Tuning::wf_bounce_waves
    case 2: wf_bounce<FIRST, 2, march::F_HEART><<<blocks, 256, 0, st>>>(A, it); break;
    case 4: wf_bounce<FIRST, 4, march::F_HEART><<<blocks, 256, 0, st>>>(A, it); break;
    case 5: wf_bounce<FIRST, 5, march::F_HEART><<<blocks, 256, 0, st>>>(A, it); break;
    case 6: wf_bounce<FIRST, 6, march::F_HEART><<<blocks, 256, 0, st>>>(A, it); break;
    case 8: wf_bounce<FIRST, 8, march::F_HEART><<<blocks, 256, 0, st>>>(A, it); break;
    default: wf_bounce<FIRST, 3, march::F_HEART><<<blocks, 256, 0, st>>>(A, it); break;
    }
}

// Exactly the resident blocks of one kernel build (persistent grids).
template <class K>
static uint32_t resident_blocks(K kern) {
    int dev = 0, cus = 256, occ = 0;
    if (hipGetDevice(&dev) == hipSuccess) {
        hipDeviceProp_t pr;
        if (hipGetDeviceProperties(&pr, dev) == hipSuccess) cus = pr.multiProcessorCount;
    }
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, 256, 0) != hipSuccess || occ < 1) occ = 1;
    return (uint32_t)(cus * occ);
}

// Chunks in flight (Tuning::wf_slots): each has its own path state (slot) and
// runs on its own stream, so one chunk's bounce/compaction kernels fill the
// tails of the other's march kernels (and its memory-bound bounces overlap the
// other's VALU-bound marches).  Only the reduces are chained, in chunk order.
static hipError_t ensure_streams(WaveWorkspace *ws, int slots) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (ws->device != dev) {  // streams and events belong to one device
        // the previous frame must be done with the streams and the workspace
        if (ws->used && ws->done && (e = hipEventSynchronize(ws->done)) != hipSuccess) return e;
        free_args(ws);  // (the device blocks live on the old device)
        if (ws->args_ev) (void)hipEventDestroy(ws->args_ev);
        ws->args_ev = nullptr;
        for (int k = 0; k < WaveWorkspace::MAX_SLOTS - 1; k++) {
            if (ws->side[k]) (void)hipStreamDestroy(ws->side[k]);
            if (ws->join[k]) (void)hipEventDestroy(ws->join[k]);
            ws->side[k] = nullptr;
            ws->join[k] = nullptr;
        }
        if (ws->fork) (void)hipEventDestroy(ws->fork);
        if (ws->reduced) (void)hipEventDestroy(ws->reduced);
        if (ws->done) (void)hipEventDestroy(ws->done);
        ws->fork = ws->reduced = ws->done = nullptr;
        ws->used = false;
        ws->device = dev;
    }
    if (!ws->fork && (e = hipEventCreateWithFlags(&ws->fork, hipEventDisableTiming)) != hipSuccess) return e;
    if (!ws->done && (e = hipEventCreateWithFlags(&ws->done, hipEventDisableTiming)) != hipSuccess) return e;
    if (!ws->reduced && (e = hipEventCreateWithFlags(&ws->reduced, hipEventDisableTiming)) != hipSuccess) return e;
    if (!ws->args_ev && (e = hipEventCreateWithFlags(&ws->args_ev, hipEventDisableTiming)) != hipSuccess) return e;
    for (int k = 0; k < slots - 1; k++) {
        if (!ws->side[k] && (e = hipStreamCreateWithFlags(&ws->side[k], hipStreamNonBlocking)) != hipSuccess) return e;
        if (!ws->join[k] && (e = hipEventCreateWithFlags(&ws->join[k], hipEventDisableTiming)) != hipSuccess) return e;
    }
    return hipSuccess;
}

// Chunks keep at least MIN_CHUNK_PATHS paths to fill the device (Tuning::wf_min_chunks).
constexpr uint32_t MIN_CHUNK_PATHS = 1u << 21;

struct Slot {
    WfView v;
    uint32_t *cp_blk;
    PathSoA set[2];  // iteration it reads set[it & 1] and writes set[(it + 1) & 1]
};

static hipError_t render_wave(const dev::Scene &sc, const FrameParams &P0, double *out, hipStream_t st,
                                 WaveWorkspace *ws, int fkind) {
    const Tuning &tu = ws->tune;
    // the launch's samples: the frame's, or a resumable frame's window [s_begin, s_end) of them
    const uint32_t s_begin = P0.s_begin, s_end = P0.s_end ? P0.s_end : P0.spp, nsw = s_end - s_begin;
    const uint32_t ntiles = P0.tile_count;
    const int iters = (int)P0.depth + 2;  // traces per path <= depth + 1, then one last shade
    const size_t cnt_words = (size_t)(iters + 2) * 4;
    auto al = [](size_t n) { return (n + 255) & ~(size_t)255; };
    // pre-selected march jobs (one marched shape): the bounce kernel hands the march its object-space ray
    // and bound (C2 +9 %: iso march 340 -> 275 ms, bounce 248 -> 256, round 1)
    const bool presel = sc.nmarch == 1 && !ws->diag;
    // The chunk plan for cap_want path slots per chunk: tile groups (only for frames beyond cap_want pixels),
    // then sample chunks, the streams, and the workspace bytes.
    struct Plan {
        uint32_t group_tiles, npix_max, ns, cap, cap_tiles;
        int slots;
        size_t att_bytes, slot_bytes, bytes;
    };
    auto plan_for = [&](uint32_t cap_want) {
        Plan pl;
        const uint32_t tiles_per_group = cap_want / (TILE * TILE) ? cap_want / (TILE * TILE) : 1;
        pl.group_tiles = ntiles < tiles_per_group ? ntiles : tiles_per_group;
        pl.npix_max = pl.group_tiles * TILE * TILE;
        uint32_t ns = cap_want / pl.npix_max;
        if (ns < 1) ns = 1;
        if (ns > nsw) ns = nsw;
        // A small frame (one rank's share of a multi-GPU frame) still gets at least wf_min_chunks sample
        // chunks, so the pipelined slots overlap one chunk's short tail iterations with the next chunk's work;
        // chunks keep at least MIN_CHUNK_PATHS paths to fill the device.  (A progressive frame's band, P0.stop
        // set, gets at least two: one per chunk stream; and any frame at least one per chunk stream while its
        // chunks keep MIN_CHUNK_PATHS paths, whatever wf_paths allows.)
        uint32_t mc = P0.stop && tu.wf_min_chunks < 2 ? 2u : (uint32_t)tu.wf_min_chunks;
        if (mc < (uint32_t)tu.wf_slots) mc = (uint32_t)tu.wf_slots;
        if (mc > 1 && ntiles <= pl.group_tiles) {
            uint32_t want = (nsw + mc - 1) / mc;
            const uint32_t floor_ns = (MIN_CHUNK_PATHS + pl.npix_max - 1) / pl.npix_max;
            if (want < floor_ns) want = floor_ns;
            if (want < ns) ns = want;
        }
        pl.ns = ns;
        pl.cap = ns * pl.npix_max;
        pl.cap_tiles = (pl.cap + CP_TILE - 1) / CP_TILE;  // compaction tiles (status padded to them)
        // no more slots than chunks
        const uint64_t chunks = (uint64_t)((ntiles + pl.group_tiles - 1) / pl.group_tiles) * ((nsw + ns - 1) / ns);
        pl.slots = tu.wf_slots;
        if ((uint64_t)pl.slots > chunks) pl.slots = (int)chunks;
        const size_t cap = pl.cap;
        pl.att_bytes = sc.tex ? cap * 24 * (P0.depth + 1) : 0;  // textured attenuation values
        // two path-state sets, leaf records, lists, id stacks, statuses, compaction tiles, counters
        pl.slot_bytes = al(cap * PathSoA::BYTES) * 2 + al(cap * 32) + (presel ? al(cap * 64) : 0) + al(cap * 4) * 2 +
                        al(cap * 4 * (P0.depth + 1)) + al((size_t)pl.cap_tiles * CP_TILE) +
                        al(((size_t)pl.cap_tiles + CP_BLOCK) * 12) + al(cnt_words * 4) + al(pl.att_bytes);
        pl.bytes = pl.slot_bytes * (size_t)pl.slots + al((size_t)pl.npix_max * 24) + 8192;
        return pl;
    };
    // Path slots per chunk: Tuning::wf_paths, or by depth (deep frames: bigger chunks, fewer tails), halved
    // until the plan fits the device memory the workspace may take (what is free plus what it holds now, less
    // 2 GiB): a deep textured frame's per-slot attenuation values ((depth + 1) * 24 B per path) would otherwise
    // ask for more than the device has (1080p, 256 spp, depth 50 at 128M paths needed ~430 GB).
    // (deep frames: 256M paths, two chunks of a 1080p x 256-spp frame in one step, ~120 GB per chunk stream at depth
    // 50: one tail of late iterations instead of two, C2 depth 50 1237 -> 1251, profiles/r6/ab/r6aa_*; 128M until round 6)
    uint32_t cap_want = tu.wf_paths ? (uint32_t)tu.wf_paths : (P0.depth > 16 ? 1u << 28 : 3u << 24);
    Plan pl = plan_for(cap_want);
    {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
            const size_t reserve_b = (size_t)2 << 30;
            const size_t avail = free_b + ws->bytes > reserve_b ? free_b + ws->bytes - reserve_b : 0;
            while (pl.bytes > avail && cap_want > MIN_CHUNK_PATHS) {
                cap_want = cap_want / 2 > MIN_CHUNK_PATHS ? cap_want / 2 : MIN_CHUNK_PATHS;
                pl = plan_for(cap_want);
            }
        }
    }
    const uint32_t group_tiles = pl.group_tiles, npix_max = pl.npix_max, ns = pl.ns, cap = pl.cap,
                   cap_tiles = pl.cap_tiles;
    const int slots = pl.slots;
    const size_t att_bytes = pl.att_bytes, bytes = pl.bytes;
    hipError_t e = ensure_streams(ws, slots);
    if (e != hipSuccess) return e;
    // One workspace serves every frame of the renderer, whichever stream it is
    // queued on (render_start's own stream, a caller's stream in
    // render_device): this frame's kernels wait for the previous frame's.
    if (ws->used && (e = hipStreamWaitEvent(st, ws->done, 0)) != hipSuccess) return e;
    e = reserve(ws, bytes);
    if (e != hipSuccess) return e;
    // carve the workspace: the slots' path state, then the shared running sums
    char *p = (char *)ws->base;
    auto take = [&](size_t n) {
        char *r = p;
        p += al(n);
        return (void *)r;
    };
    Slot sl[WaveWorkspace::MAX_SLOTS];
    for (int k = 0; k < slots; k++) {
        WfView &v = sl[k].v;
        for (int h = 0; h < 2; h++) {
            PathSoA &S = sl[k].set[h];
            S.base = (char *)take((size_t)cap * PathSoA::BYTES);
            S.cap = cap;
        }
        v.ids = (uint32_t *)take((size_t)cap * 4 * (P0.depth + 1));
        v.leaf = (double *)take((size_t)cap * 32);  // 32-byte leaf records (end_path)
        v.list = (uint32_t *)take((size_t)cap * 4);
        v.mq = (uint32_t *)take((size_t)cap * 4);
        v.status = (uint8_t *)take((size_t)cap_tiles * CP_TILE);
        sl[k].cp_blk = (uint32_t *)take(((size_t)cap_tiles + CP_BLOCK) * 12);  // CpLayout: 3 x per * 256 words
        v.cnt = (uint32_t *)take(cnt_words * 4);
        v.att = att_bytes ? (double *)take(att_bytes) : nullptr;
        v.jo = presel ? (double2 *)take((size_t)cap * 64) : nullptr;
        v.cap = cap;
    }
    double *acc = (double *)take((size_t)npix_max * 24);
    for (int k = 0; k < slots; k++) sl[k].v.acc = acc;
    if ((size_t)(p - (char *)ws->base) > ws->bytes) return hipErrorOutOfMemory;

    // persistent march grid: exactly the resident blocks of the device (a half-machine grid measured slower)
    static const uint32_t march_blocks = resident_blocks(wf_march<march::F_HEART>);
    const uint32_t march_slice = (uint32_t)tu.wf_march_slice;
    const bool split = walk_split(sc, tu);
    // Chunk j of step k runs on stream j (its path-state slot); a step's chunks
    // are enqueued iteration by iteration across the step.  (Measured slower and
    // removed in round 6, DESIGN.md §5: bounce or march launches chained across
    // the streams, side streams at another priority, streams staggered by part
    // of a chunk, a tail kernel running a chunk's last paths to their ends.)
    struct Chunk {
        uint32_t g0, gt, s0, ns;
        int slot;
        uint32_t step;
    };
    // Sample chunks of a tile group: as few as fit ns samples each, rounded up
    // to whole rounds of `slots` (no round with an idle stream), with the
    // samples spread evenly over them (no short last chunk).  The per-pixel
    // sums take the chunks in sample order either way.
    uint32_t nchunks = (nsw + ns - 1) / ns;
    if (slots > 1 && nchunks > 1 && nchunks % (uint32_t)slots) nchunks += (uint32_t)slots - nchunks % (uint32_t)slots;
    if (nchunks > nsw) nchunks = nsw;
    const uint32_t S = (uint32_t)slots;
    std::vector<Chunk> chunk_list;
    uint32_t step0 = 0;
    for (uint32_t g0 = 0; g0 < ntiles; g0 += group_tiles) {
        const uint32_t gt = ntiles - g0 < group_tiles ? ntiles - g0 : group_tiles;
        uint32_t s0 = s_begin;
        for (uint32_t c = 0; c < nchunks; c++) {
            const uint32_t s1 = s_begin + (uint32_t)((uint64_t)nsw * (c + 1) / nchunks);  // <= ceil(nsw / nchunks) <= ns
            chunk_list.push_back(Chunk{g0, gt, s0, s1 - s0, (int)(c % S), step0 + c / S});
            s0 = s1;
        }
        step0 += (nchunks + S - 1) / S;
    }
    // The launches' argument blocks (WfArgs): chunk ci at iteration parity h is block 2 ci + h.  They are
    // written to the pinned staging buffer, which the previous frame's copy must have read, and copied to the
    // device on st after the previous frame's kernels (the wait on ws->done above), before the side streams fork.
    const size_t nargs = chunk_list.size() * 2;
    if ((e = reserve_args(ws, nargs * sizeof(WfArgs))) != hipSuccess) return e;
    WfArgs *ah = (WfArgs *)ws->args_host, *ad = (WfArgs *)ws->args_dev;
    for (size_t ci = 0; ci < chunk_list.size(); ci++) {
        const Chunk &ch = chunk_list[ci];
        const int j = ch.slot;
        WfView v = sl[j].v;
        v.tile0 = P0.tile_begin + ch.g0;
        v.npix = ch.gt * TILE * TILE;
        v.s0 = ch.s0;
        v.ns = ch.ns;
        for (int h = 0; h < 2; h++) {
            v.in = sl[j].set[h];
            v.out = sl[j].set[h ^ 1];
            ah[2 * ci + h] = WfArgs{sc, P0, v};
        }
    }
    if ((e = hipMemcpyAsync(ad, ah, nargs * sizeof(WfArgs), hipMemcpyHostToDevice, st)) != hipSuccess) return e;
    if ((e = hipEventRecord(ws->args_ev, st)) != hipSuccess) return e;
    ws->args_pending = true;
    // the side streams start after everything the caller queued on st
    if (slots > 1) {
        if ((e = hipEventRecord(ws->fork, st)) != hipSuccess) return e;
        for (int k = 0; k < slots - 1; k++)
            if ((e = hipStreamWaitEvent(ws->side[k], ws->fork, 0)) != hipSuccess) return e;
    }
    for (size_t r0 = 0; r0 < chunk_list.size();) {
        size_t r1 = r0;  // the step's chunks [r0, r1), in sample order, at most one per stream
        while (r1 < chunk_list.size() && chunk_list[r1].step == chunk_list[r0].step) r1++;
        for (size_t c = r0; c < r1; c++) {  // the step's chunks: cleared counters
            const int j = chunk_list[c].slot;
            const hipStream_t cs = j == 0 ? st : ws->side[j - 1];
            if ((e = hipMemsetAsync(sl[j].v.cnt, 0, cnt_words * 4, cs)) != hipSuccess) return e;
            if (P0.stop) {
                stop_gate<<<1, 64, 0, cs>>>(P0.stop, sl[j].v.cnt, -1);
                if ((e = hipGetLastError()) != hipSuccess) return e;
            }
        }
        for (int it = 0; it < iters; it++) {
            for (size_t c = r0; c < r1; c++) {
                const Chunk &ch = chunk_list[c];
                const int j = ch.slot;
                const hipStream_t cs = j == 0 ? st : ws->side[j - 1];
                const WfArgs *A = ad + 2 * c + (it & 1);
                const WfView &v = sl[j].v;
                uint32_t *cp_blk = sl[j].cp_blk;
                const uint32_t paths = ch.ns * ch.gt * TILE * TILE;
                uint32_t bb = (paths + 255) / 256;
                if (bb > WF_BOUNCE_CAP) bb = WF_BOUNCE_CAP;
                // iteration 0: slots [0, paths) are the chunk's camera rays
                if ((e = timer_begin(ws->timer, cs, K_BOUNCE)) != hipSuccess) return e;
                if (it == 0)
                    launch_bounce<true>((paths + 255) / 256, cs, sc, A, 0, ws->diag, fkind, tu.wf_bounce_waves,
                                            split);
                else
                    launch_bounce<false>(bb, cs, sc, A, it, ws->diag, fkind, tu.wf_bounce_waves, split);
                if ((e = hipGetLastError()) != hipSuccess) return e;
                if ((e = timer_end(ws->timer, cs)) != hipSuccess) return e;
                if (it == iters - 1) continue;  // the last bounce only shades
                // live list for it + 1 and march queue for it, both id-sorted
                if ((e = timer_begin(ws->timer, cs, K_SELECT)) != hipSuccess) return e;
                const uint32_t ptiles = (paths + CP_TILE - 1) / CP_TILE;
                const uint32_t *n_in = it == 0 ? nullptr : &v.cnt[it * 4 + 0];  // the bounce's input count
                const CpLayout L = CpLayout::of(ptiles);
                const uint32_t cgrid = CP_GRID && ptiles > CP_GRID ? CP_GRID : ptiles;
                cp_count<<<cgrid, CP_BLOCK, 0, cs>>>(v.status, cp_blk, L, n_in, paths);
                cp_scan<<<1, CP_BLOCK, 0, cs>>>(cp_blk, ptiles, L, n_in, paths, &v.cnt[(it + 1) * 4 + 0],
                                                &v.cnt[it * 4 + 1], &v.cnt[it * 4 + 2]);
                cp_scatter<<<cgrid, CP_BLOCK, 0, cs>>>(v.status, cp_blk, L, &v.cnt[it * 4 + 2], v.list, v.mq, n_in,
                                                       paths);
                if (P0.stop) stop_gate<<<1, 64, 0, cs>>>(P0.stop, v.cnt, it);
                if ((e = hipGetLastError()) != hipSuccess) return e;
                if ((e = timer_end(ws->timer, cs)) != hipSuccess) return e;
                if (split) {  // the new rays' BVH walk, over the live list of it + 1
                    if ((e = timer_begin(ws->timer, cs, K_WALK)) != hipSuccess) return e;
                    if (!sc.qnodes) {  // (a tree without the quantized form)
                        wf_walk<5, false><<<bb, 256, 0, cs>>>(A, it);
                    } else {
                        switch (tu.wf_walk) {  // the walk's register budget, waves per SIMD
                        case 4: wf_walk<4, true><<<bb, 256, 0, cs>>>(A, it); break;
                        case 6: wf_walk<6, true><<<bb, 256, 0, cs>>>(A, it); break;
                        case 8: wf_walk<8, true><<<bb, 256, 0, cs>>>(A, it); break;
                        default: wf_walk<5, true><<<bb, 256, 0, cs>>>(A, it); break;
                        }
                    }
                    if ((e = hipGetLastError()) != hipSuccess) return e;
                    if ((e = timer_end(ws->timer, cs)) != hipSuccess) return e;
                }
                if (sc.nmarch == 0) continue;  // no ray-marched shape: the march queue is always empty
                if ((e = timer_begin(ws->timer, cs, K_MARCH)) != hipSuccess) return e;
                if (fkind != march::F_HEART)
                    wf_march<march::F_ANY><<<march_blocks, 256, 0, cs>>>(A, it, nullptr, march_slice);
                else if (ws->diag)
                    wf_march<march::F_HEART><<<march_blocks, 256, 0, cs>>>(A, it, ws->diag, march_slice);
                else
                    wf_march<march::F_HEART><<<march_blocks, 256, 0, cs>>>(A, it, nullptr, march_slice);
                if ((e = hipGetLastError()) != hipSuccess) return e;
                if ((e = timer_end(ws->timer, cs)) != hipSuccess) return e;
            }
        }
        // the per-pixel sums take the chunks in sample order (chunk_list order)
        for (size_t c = r0; c < r1; c++) {
            const Chunk &ch = chunk_list[c];
            const int j = ch.slot;
            const hipStream_t cs = j == 0 ? st : ws->side[j - 1];
            const WfArgs *A = ad + 2 * c;
            const uint32_t npix = ch.gt * TILE * TILE;
            // a chunk of few pixels unwinds its slots first, one thread each (a thread per pixel would be one wave
            // per SIMD walking its samples' dependent loads one after another), before it waits for the previous
            // chunk's sums.  Larger chunks fill the machine with pixels, and the extra pass over the slots costs
            // more than it saves: C1 +1.5 %, but C2 -2.2 to -3.5 %, C5 -2.7 %, even C2 depth 50 -1.4 %
            // (profiles/r6/ab/r6m_reduce_split_summary.txt, r6q_unwind_all_summary.txt)
            const bool unwound = npix < UNWIND_PIXELS;
            if (unwound) {
                const uint32_t slots_c = ch.ns * npix;
                if ((e = timer_begin(ws->timer, cs, K_UNWIND)) != hipSuccess) return e;
                if (sc.ext)
                    wf_unwind<true><<<(slots_c + 255) / 256, 256, 0, cs>>>(A);
                else
                    wf_unwind<false><<<(slots_c + 255) / 256, 256, 0, cs>>>(A);
                if ((e = hipGetLastError()) != hipSuccess) return e;
                if ((e = timer_end(ws->timer, cs)) != hipSuccess) return e;
            }
            if (slots > 1 && c > 0 && (e = hipStreamWaitEvent(cs, ws->reduced, 0)) != hipSuccess) return e;
            if ((e = timer_begin(ws->timer, cs, K_REDUCE)) != hipSuccess) return e;
            // first: 1 = sums from zero, 2 = from out's running sums; last: 1 = means, 2 = running sums to out
            const int first = ch.s0 == s_begin ? (s_begin == 0 ? 1 : 2) : 0;
            const int last = ch.s0 + ch.ns >= s_end ? (s_end == P0.spp ? 1 : 2) : 0;
            const uint32_t rb = (npix + 255) / 256;
            if (sc.ext && unwound)
                wf_reduce<true, true><<<rb, 256, 0, cs>>>(A, first, last, out);
            else if (sc.ext)
                wf_reduce<true, false><<<rb, 256, 0, cs>>>(A, first, last, out);
            else if (unwound)
                wf_reduce<false, true><<<rb, 256, 0, cs>>>(A, first, last, out);
            else
                wf_reduce<false, false><<<rb, 256, 0, cs>>>(A, first, last, out);
            if ((e = hipGetLastError()) != hipSuccess) return e;
            if ((e = timer_end(ws->timer, cs)) != hipSuccess) return e;
            if (slots > 1 && (e = hipEventRecord(ws->reduced, cs)) != hipSuccess) return e;
        }
        r0 = r1;
    }
    // the caller's stream resumes after every side stream's last chunk
    for (int k = 0; k < slots - 1; k++) {
        if ((e = hipEventRecord(ws->join[k], ws->side[k])) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(st, ws->join[k], 0)) != hipSuccess) return e;
    }
    if ((e = hipEventRecord(ws->done, st)) != hipSuccess) return e;
    ws->used = true;
    return hipSuccess;
}

#ifdef PT_LANE_PROF
// Lane profile of the bounce kernel (pt_lprof.hpp): out[k] wave passes and out[N + k] active lanes summed at
// profiling point k, N = the return value; clear: zero the counters afterwards.
extern "C" int pt_lane_prof(unsigned long long *out, int clear) {
    if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(lprof::g_counts), sizeof(lprof::g_counts)) != hipSuccess)
        return -1;
    if (clear) {
        static const unsigned long long z[2 * lprof::N_POINTS] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(lprof::g_counts), z, sizeof(z)) != hipSuccess) return -1;
    }
    return lprof::N_POINTS;
}
#endif

#ifdef PT_MARCH_REGIONS
// Region wave-cycles of the march kernel since the last clear (tuning builds).
extern "C" int pt_march_regions(unsigned long long *out, int clear) {
    if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(mreg::g_acc), sizeof(mreg::g_acc)) != hipSuccess) return -1;
    if (clear) {
        static const unsigned long long z[mreg::G_N] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(mreg::g_acc), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

hipError_t launch_render_wave(const dev::Scene &sc, const FrameParams &P, double *out, hipStream_t st,
                              WaveWorkspace *ws, int fkind) {
    if (P.tile_count == 0 || P.spp == 0) return hipSuccess;
    // (the wavefront keeps attenuation ids in HBM, so one build serves every depth)
    return render_wave(sc, P, out, st, ws, fkind);
}

}  // namespace pt
