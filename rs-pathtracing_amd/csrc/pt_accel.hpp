// pt_accel.hpp — closest-hit acceleration for the GPU path (host build).
//
// The reference wraps the shape list in a randomly split BvhNode tree
// (src/world/shapes/mod.rs:620-729); its result is the ShapeCollection linear
// minimum (mod.rs:587-596) up to exact ties.  Here the realized list is split
// into three groups, all tested with one acceptance rule — accept t if
// t < best or (t == best and shape index > best index) — which reproduces the
// linear scan's "later shape wins a tie" in any visiting order:
//   * `lin`   — the JSON shapes when there are few, and every Torus: a
//               wave-uniform loop;
//   * BVH     — everything else that is not ray-marched (random spheres,
//               large scenes), median-split, threaded, padded f64 boxes;
//   * `march` — ray-marched shapes, tested last behind their padded box
//               against the best distance so far.
#pragma once
#include <cstdint>
#include <vector>

#include "pt_scene.hpp"
#include "pt_types.hpp"

namespace pt {

// The BVH is stored as 8 threaded (stackless, skip-pointer) layouts of the same
// tree, one per ray-direction octant: layout o = (d.x < 0) | (d.y < 0) << 1 |
// (d.z < 0) << 2 visits, at every interior node, the child on the ray's near
// side of the split first, so the best hit shrinks early and far subtrees are
// skipped by their boxes.  Skip indices are relative to the layout; the leaf
// id ranges are shared.  8x the node memory (C5: ~50 MB of the 288 GB HBM)
// buys front-to-back order without a per-lane stack.
constexpr int BVH_OCTANTS = 8;
struct Accel {
    std::vector<DNode> nodes;    // BVH_OCTANTS layouts of nodes_per_octant() nodes each
    std::vector<DNodeC> cnodes;  // the same nodes in the device form (f32 boxes rounded outward)
    int nodes_per_octant() const { return (int)(nodes.size() / BVH_OCTANTS); }
    std::vector<int32_t> leaf;   // shape ids referenced by leaf nodes
    std::vector<int32_t> lin;    // wave-uniform list
    std::vector<int32_t> march;  // ray-marched shapes
    std::vector<DBox> boxes;     // padded world AABB per shape
    float bvh_bound = 0.f;  // >= |every plane of cnodes| (dev::Scene::bvh_bound)
    // the quantized nodes (trees of at least BIG_BVH_NODES nodes per layout; empty otherwise) and their grid
    std::vector<DNodeQ> qnodes;
    // the one-shape leaves' records (DLeafRec, octant 0's order), which their quantized links name
    std::vector<DLeafRec> qleaves;
    double qg0[3] = {0, 0, 0}, qgs[3] = {0, 0, 0};
    float qbound = 0.f;  // >= |every quantized plane| and >= |qg0|
};

constexpr int LIN_MAX = 32;  // JSON shape count up to which the JSON shapes form `lin`

// leaf_max: shapes per BVH leaf (the renderer option "bvh_leaf")
Accel build_accel(const Scene &sc, int json_shapes, int leaf_max = 1);
// the quantized nodes of a's layouts (build_accel does this for trees of at least BIG_BVH_NODES nodes per layout;
// tests call it for smaller ones)
void build_qnodes(Accel &a, const Scene &sc);

// conservative world AABB of one shape (reference get_bounding_box + padding)
DBox shape_box(const HostShape &s);

}  // namespace pt
