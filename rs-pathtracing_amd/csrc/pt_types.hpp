// pt_types.hpp — device-visible layouts shared by the host library and the
// HIP kernels.  One DShape per leaf of the realized shape list (JSON shapes in
// file order, then the add_random_spheres spheres), 320 B each (five 64-B
// lines); matrices keep only the three rows the kernels apply.
#pragma once
#include <cstdint>

namespace pt {

enum ShapeKind : int32_t { SPHERE = 0, RECTANGLE = 1, CUBE = 2, MARCH = 3, TORUS = 4 };
enum MaterialKind : int32_t { LAMBERTIAN = 0, METAL = 1, DIELECTRIC = 2, DIFFUSE_LIGHT = 3, EMPTY = 4 };

struct alignas(64) DShape {
    // a miss test of a sphere or cube reads only the first two cache lines
    // (type + inv); rectangles add the third (p)
    int32_t type, material, inverse_normal, depth;
    double inv[12];  // InversableTransform::inverse, rows 0..2 (3x4)
    int32_t func;
    // 1: a sphere whose inverse transform is a diagonal scale plus a translation with every translation entry
    // nonzero (rotation 0, as add_random_spheres makes them): its object-space ray takes 2 FLOP per component
    // with the same bits as the full transform (dev::sphere_axis_t)
    int32_t axis;
    int32_t pad[2];
    double p[4];     // Rectangle x0,y0,x1,y1 | RayMarchingShape: step | Torus radius, tube_radius
    double dir[12];  // InversableTransform::direct, rows 0..2
    double fk[4];    // RayMarchingShape function constants (pt_funcs.hpp FParams::k)
    double fradius;  // its bound's sphere_radius
    double pad2[3];
};
static_assert(sizeof(DShape) == 320, "DShape is five cache lines");

// tex: -1 when the albedo (Lambertian, Metal) or emit (DiffuseLight) texture
// is a SolidColor, whose colour is stored here; otherwise the root DTexture.
struct alignas(8) DMaterial {
    int32_t type, tex;
    double albedo[3];
    double fuzz, ior;
    double emit[3];
};

// Texture tree node (src/world/texture.rs).  Checker nodes choose their odd or
// even child node; SolidColor, NoiseTexture and ImageTexture are leaves.
enum TextureKind : int32_t { TEX_SOLID = 0, TEX_CHECKER = 1, TEX_UVCHECKER = 2, TEX_NOISE = 3, TEX_IMAGE = 4 };
struct alignas(8) DTexture {
    int32_t type, odd, even, aux;  // aux: Perlin table (noise) or image index
    double c[3];  // SolidColor color | CheckerTexture multipliers | UVChecker multipliers (2) | noise scale
};
// Perlin (src/algebra/noise.rs:6-42): the three permutations and ranvec
// (ranfloat is drawn but never read by the texture).
struct DPerlin {
    int32_t perm[3][256];
    double ranvec[256][3];
};
// ImageTexture pixels (RGBA8, row-major) in the scene's pixel pool.
struct DImage {
    uint64_t offset;
    uint32_t width, height;
};

// Threaded (skip-pointer) BVH node over shapes, DFS order: on an AABB hit go
// to i+1 (first child, or the next node after a leaf's shapes are tested), on
// a miss jump to `skip`.  Leaf nodes list `count` shape ids from leaf[first].
struct alignas(64) DNode {
    double lo[3], hi[3];
    int32_t skip, first, count, pad;
};
static_assert(sizeof(DNode) == 64, "DNode is one cache line");

// The device form of a DNode, half a cache line: the f64 box rounded outward
// to f32 (so its f64 slab test accepts a superset of the exact box's rays:
// rounding is monotone, and the exact leaf tests still decide every hit, in
// the order-independent tie rule of closest_nomarch), skip as in DNode, and
// first | count << 24 (leaves hold at most 16 shapes; first < 2^24 is checked
// when the BVH is built); bit 31 marks a one-shape leaf whose `first` is the
// shape id itself rather than an index into the leaf list.
// In octant o's layout (pt_accel.hpp) the box is stored as near and far
// planes: for an axis where o's ray direction is negative (sign bit set) the
// two are the box's hi and lo, so the walk needs no min/max per axis.
struct alignas(32) DNodeC {
    float nr[3], fr[3];
    int32_t skip;
    uint32_t first_count;
};
static_assert(sizeof(DNodeC) == 32, "DNodeC is half a cache line");

// The large-tree walk's node form (wf_walk, round 5), a quarter cache line: the six planes of a DNodeC as
// 16-bit steps of a per-axis grid (plane = g0[k] + q * gs[k], gs a power of two covering the root box in 65535
// steps), lo planes rounded down and hi planes up (the box only grows: the slab test stays conservative), and one
// link word: an interior node's skip, or a leaf (bit 31; a leaf's skip is always the next node) with bit 30 set
// for a one-shape leaf whose `first` is the shape id, count in bits 24-29 and first in bits 0-23.
struct alignas(16) DNodeQ {
    uint16_t q[6];  // near planes (x, y, z), then far planes, in the octant's order
    uint32_t link;
};
static_assert(sizeof(DNodeQ) == 16, "DNodeQ is a quarter cache line");
// byte offset of the leaf records in the quantized nodes' buffer (grid, layouts, one node of padding, records)
__host__ __device__ inline size_t qleaf_offset(int nnodes_per_octant) {
    return 64 + ((size_t)(8 * (size_t)nnodes_per_octant + 1) * 16 + 63) / 64 * 64;
}
// The quantized nodes' device buffer starts with their grid; the octant layouts follow it.
struct alignas(64) DQGrid {
    double g0[3], gs[3];
    float bound;  // >= |every quantized plane| and >= |g0|
    float pad[3];
};
static_assert(sizeof(DQGrid) == 64, "DQGrid is one cache line");

constexpr int BIG_BVH_NODES = 1 << 15;  // binary nodes from which the bounce runs its large-tree builds (C5)

// A one-shape leaf of the large-tree walk's quantized nodes (round 6): the shape id, and for a sphere whose inverse
// transform is a diagonal scale plus a translation (DShape::axis) the six entries sphere_axis_t reads (m0, m5,
// m10, m3, m7, m11), so its exact test reads this 64-byte record (one line, siblings' records adjacent) and not
// two lines of the 320-byte shape; any other shape is tested from sc.shapes.  C5 walk 179.5 -> 172.0 ms per
// one-stream frame, 2118 -> 2180 M samples/s (profiles/r6/ab/r6c_wide_dp_qrec_c5.log).
struct alignas(64) DLeafRec {
    double m[6];
    int32_t shape, axis;
    int32_t pad[2];
};
static_assert(sizeof(DLeafRec) == 64, "DLeafRec is one 64-byte record");

struct DBox {
    double lo[3], hi[3];
};

// Per-frame constants: MultisamplerRayCaster (src/camera/ray_caster.rs:30-48)
// plus the tile shard this launch renders.
struct FrameParams {
    double pos[3], right[3], up[3], left_top[3];
    double pixel_resolution;
    double s11;  // UniformFloat::new_inclusive(-1, 1).scale (rand 0.8)
    uint64_t seed;
    uint32_t width, height, spp, depth;
    uint32_t rank, world, tiles_x, tile_begin;
    uint32_t tile_count, compact;
    // sample window [s_begin, s_end) of a resumable frame (pt_render_device_samples; s_end 0 = spp): the launch
    // adds those samples to the per-pixel running sums in `out` (read when s_begin > 0) and stores the sums,
    // or the means when s_end = spp; samples keep their frame-wide indices, so the windows' results are the
    // whole frame's bit for bit
    uint32_t s_begin, s_end;
    // progressive frames: the renderer's stop flag in host-mapped memory
    // (pt_render_stop sets it while it drains the queued launches); null: none
    const int *stop;
};

// Work counters of the diagnostic (STATS) kernel build: the kernel's own event
// counts, turned into algorithmic FLOPs per sample by bench.py.
enum Counter : int {
    C_SAMPLES, C_BOUNCES, C_TEST_SPHERE, C_TEST_RECT, C_TEST_CUBE, C_TEST_MARCH, C_NODE_SLABS, C_MARCH_SLABS,
    C_MARCH_STEPS, C_MARCH_TRIES, C_MARCH_BLOCKS, C_HITS, C_LAMBERT, C_METAL, C_DIELECTRIC, C_REJECT_TRIES,
    C_UNWIND, C_TEST_TORUS, C_MARCH_GUARD, C_COUNT
};
struct Ctr {
    uint64_t c[C_COUNT];
};

constexpr uint32_t TILE = 16;  // 16x16 pixels = one 256-thread workgroup
constexpr double T_MIN = 0.001;  // ray_color: closest_hit(ray, 0.001, INF), src/renderer/mod.rs:24

}  // namespace pt
