// pt_accel.cpp — see pt_accel.hpp.
#include "pt_accel.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <stdexcept>

namespace pt {

// Object-space bounds of each kind (get_bounding_box: Rectangle mod.rs:214-220,
// Cube :295-301, Sphere :384-398, RayMarchingShape ray_marching.rs:84-91 with
// Heart::get_bounds :174-187), transformed by the 8 corners (AABB::transform,
// mod.rs:93-108), then padded so that every point a leaf test can return lies
// strictly inside: 1e-7 relative + 1e-9 absolute, and for a ray-marched shape
// two march steps more (a forward pass may overshoot `end` by one step).
DBox shape_box(const HostShape &s) {
    double lo[3], hi[3];
    switch (s.type) {
    case RECTANGLE:
        lo[0] = s.x0; lo[1] = s.y0; lo[2] = -0.0001;
        hi[0] = s.x1; hi[1] = s.y1; hi[2] = 0.0001;
        break;
    case MARCH:
        if (s.func == 0) {  // Heart: the fixed ellipsoid bound (ray_marching.rs:126-145)
            lo[0] = -1.45; lo[1] = -(1.45 / 2.05); lo[2] = -1.45;
            hi[0] = 1.45; hi[1] = 1.45 / 2.05; hi[2] = 1.45;
        } else {  // the other functions: the sphere_radius ball
            const double r = std::fabs(s.fr);
            lo[0] = lo[1] = lo[2] = -r;
            hi[0] = hi[1] = hi[2] = r;
        }
        break;
    case TORUS: {  // get_bounding_box (mod.rs:478-485)
        const double a = s.radius + s.tube_radius;
        lo[0] = -a; lo[1] = -a; lo[2] = -s.tube_radius;
        hi[0] = a; hi[1] = a; hi[2] = s.tube_radius;
        break;
    }
    default:
        lo[0] = lo[1] = lo[2] = -1.0;
        hi[0] = hi[1] = hi[2] = 1.0;
    }
    DBox b;
    for (int k = 0; k < 3; k++) {
        b.lo[k] = INFINITY;
        b.hi[k] = -INFINITY;
    }
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++)
            for (int k = 0; k < 2; k++) {
                double p[3] = {i ? hi[0] : lo[0], j ? hi[1] : lo[1], k ? hi[2] : lo[2]};
                for (int r = 0; r < 3; r++) {
                    double v = p[0] * s.direct[r][0] + p[1] * s.direct[r][1] + p[2] * s.direct[r][2] + s.direct[r][3];
                    b.lo[r] = std::min(b.lo[r], v);
                    b.hi[r] = std::max(b.hi[r], v);
                }
            }
    double extent = 0;
    for (int r = 0; r < 3; r++)
        extent = std::max({extent, std::fabs(b.lo[r]), std::fabs(b.hi[r]), b.hi[r] - b.lo[r]});
    double pad = 1e-7 * extent + 1e-9;
    if (s.type == MARCH) pad += 2.0 * std::fabs(s.step);
    for (int r = 0; r < 3; r++) {
        b.lo[r] -= pad;
        b.hi[r] += pad;
    }
    return b;
}

namespace {

struct Builder {
    const std::vector<DBox> &boxes;
    Accel &out;
    int leaf_max = 1;  // shapes per leaf (Tuning::bvh_leaf; C5 measured 677 / 609 / 534 M samples/s at 1 / 2 / 4)
    // the tree in build order: node box (DNode with first/count for leaves),
    // split axis and children (-1 for a leaf)
    struct TNode {
        DNode n;
        int axis, left, right;
    };
    std::vector<TNode> tree;

    // one threaded layout: DFS with the near child first for the octant's
    // direction signs; skip = index after the subtree, relative to `base`
    void thread(int t, int oct, size_t base) {
        const size_t me = out.nodes.size();
        out.nodes.push_back(tree[t].n);
        if (tree[t].left >= 0) {
            const bool neg = (oct >> tree[t].axis) & 1;  // moving toward -axis: the high half is nearer
            thread(neg ? tree[t].right : tree[t].left, oct, base);
            thread(neg ? tree[t].left : tree[t].right, oct, base);
        }
        out.nodes[me].skip = (int32_t)(out.nodes.size() - base);
    }

    int emit(std::vector<int32_t> &ids, size_t a, size_t b) {
        const int me = (int)tree.size();
        tree.push_back(TNode{DNode{}, 0, -1, -1});
        DNode n{};
        for (int k = 0; k < 3; k++) {
            n.lo[k] = INFINITY;
            n.hi[k] = -INFINITY;
        }
        double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (size_t i = a; i < b; i++) {
            const DBox &x = boxes[ids[i]];
            for (int k = 0; k < 3; k++) {
                n.lo[k] = std::min(n.lo[k], x.lo[k]);
                n.hi[k] = std::max(n.hi[k], x.hi[k]);
                double c = 0.5 * (x.lo[k] + x.hi[k]);
                clo[k] = std::min(clo[k], c);
                chi[k] = std::max(chi[k], c);
            }
        }
        if (b - a <= (size_t)leaf_max) {
            n.first = (int32_t)out.leaf.size();
            n.count = (int32_t)(b - a);
            for (size_t i = a; i < b; i++) out.leaf.push_back(ids[i]);
            tree[me].n = n;
            return me;
        }
        int axis = 0;
        for (int k = 1; k < 3; k++)
            if (chi[k] - clo[k] > chi[axis] - clo[axis]) axis = k;
        // Binned surface-area split: 32 bins per axis over the centroid bounds, the cut that minimises
        // n_left * area(left) + n_right * area(right) (C5 node tests per sample 127.6 -> 120.6, 1568 -> 1635 M
        // samples/s; 8 / 64 / 128 bins: 121.7 / 120.0 / 120.6 on the host count); the median split on the widest
        // centroid axis when no cut separates the boxes.  Any tree gives the same hits: the acceptance rule is
        // order-independent.
        if (b - a > 2) {
            constexpr int NB = 32;
            auto area = [](const double *lo, const double *hi) {
                const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
                return x * y + y * z + z * x;
            };
            double best = INFINITY;
            int bk = -1, bi = -1;
            for (int k = 0; k < 3; k++) {
                const double ext = chi[k] - clo[k];
                if (!(ext > 0.0)) continue;
                int cnt[NB] = {};
                double blo[NB][3], bhi[NB][3];
                for (int j = 0; j < NB; j++)
                    for (int r = 0; r < 3; r++) blo[j][r] = INFINITY, bhi[j][r] = -INFINITY;
                for (size_t i = a; i < b; i++) {
                    const DBox &x = boxes[ids[i]];
                    int j = (int)((0.5 * (x.lo[k] + x.hi[k]) - clo[k]) / ext * NB);
                    j = j < 0 ? 0 : (j >= NB ? NB - 1 : j);
                    cnt[j]++;
                    for (int r = 0; r < 3; r++) blo[j][r] = std::min(blo[j][r], x.lo[r]), bhi[j][r] = std::max(bhi[j][r], x.hi[r]);
                }
                double rlo[NB][3], rhi[NB][3];
                int rc[NB];
                for (int j = NB - 1; j >= 0; j--) {
                    for (int r = 0; r < 3; r++) {
                        rlo[j][r] = j + 1 < NB ? std::min(rlo[j + 1][r], blo[j][r]) : blo[j][r];
                        rhi[j][r] = j + 1 < NB ? std::max(rhi[j + 1][r], bhi[j][r]) : bhi[j][r];
                    }
                    rc[j] = (j + 1 < NB ? rc[j + 1] : 0) + cnt[j];
                }
                double llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
                int lc = 0;
                for (int j = 0; j + 1 < NB; j++) {
                    lc += cnt[j];
                    for (int r = 0; r < 3; r++) llo[r] = std::min(llo[r], blo[j][r]), lhi[r] = std::max(lhi[r], bhi[j][r]);
                    if (lc == 0 || rc[j + 1] == 0) continue;
                    const double c = lc * area(llo, lhi) + rc[j + 1] * area(rlo[j + 1], rhi[j + 1]);
                    if (c < best) best = c, bk = k, bi = j;
                }
            }
            if (bk >= 0) {
                const double ext = chi[bk] - clo[bk];
                auto left = [&](int32_t id) {
                    const DBox &x = boxes[id];
                    int j = (int)((0.5 * (x.lo[bk] + x.hi[bk]) - clo[bk]) / ext * NB);
                    j = j < 0 ? 0 : (j >= NB ? NB - 1 : j);
                    return j <= bi;
                };
                const size_t m = (size_t)(std::stable_partition(ids.begin() + a, ids.begin() + b, left) - ids.begin());
                if (m > a && m < b) {
                    const int l = emit(ids, a, m);
                    const int r = emit(ids, m, b);
                    n.count = 0;
                    n.first = 0;
                    tree[me] = TNode{n, bk, l, r};
                    return me;
                }
            }
        }
        size_t mid = a + (b - a) / 2;
        std::nth_element(ids.begin() + a, ids.begin() + mid, ids.begin() + b, [&](int32_t x, int32_t y) {
            double cx = boxes[x].lo[axis] + boxes[x].hi[axis], cy = boxes[y].lo[axis] + boxes[y].hi[axis];
            return cx < cy || (cx == cy && x < y);
        });
        const int l = emit(ids, a, mid);
        const int r = emit(ids, mid, b);
        n.count = 0;
        n.first = 0;
        tree[me] = TNode{n, axis, l, r};
        return me;
    }
};

}  // namespace

// The grid of the quantized nodes: per axis the step is the smallest power of two with which 65535 steps from
// g0 = floor(lo / step) * step cover the root box.  False (grid unset) when the box is not finite or too wide for
// a finite step.
static bool make_grid(Accel &a) {
    double lo[3], hi[3];
    for (int k = 0; k < 3; k++) lo[k] = INFINITY, hi[k] = -INFINITY;
    for (const DNode &n : a.nodes)
        for (int k = 0; k < 3; k++) lo[k] = std::min(lo[k], n.lo[k]), hi[k] = std::max(hi[k], n.hi[k]);
    for (int k = 0; k < 3; k++) {
        if (!(std::isfinite(lo[k]) && std::isfinite(hi[k]) && std::isfinite(hi[k] - lo[k]))) return false;
        double step = std::ldexp(1.0, std::ilogb(std::max(hi[k] - lo[k], 1e-300) / 65535.0));
        for (int guard = 0;; guard++) {
            const double g0 = std::floor(lo[k] / step) * step;
            if (std::isfinite(g0) && std::ceil((hi[k] - g0) / step) <= 65535.0 && g0 <= lo[k]) {
                a.qg0[k] = g0;
                a.qgs[k] = step;
                break;
            }
            step *= 2.0;
            if (!std::isfinite(step) || guard > 64) return false;
        }
    }
    return true;
}
// a plane rounded down (lo) or up (hi) to the grid, as a step count in [0, 65535]
static double q_down(const Accel &a, double v, int k) {
    double q = std::floor((v - a.qg0[k]) / a.qgs[k]);
    while (q > 0 && a.qg0[k] + q * a.qgs[k] > v) q -= 1.0;
    return std::max(0.0, std::min(65535.0, q));
}
static double q_up(const Accel &a, double v, int k) {
    double q = std::ceil((v - a.qg0[k]) / a.qgs[k]);
    while (q < 65535.0 && a.qg0[k] + q * a.qgs[k] < v) q += 1.0;
    return std::max(0.0, std::min(65535.0, q));
}

// The quantized nodes of a large tree (DNodeQ) on the grid of make_grid: every lo plane is rounded down to the
// grid and every hi plane up, checked in f64 (g0 + q * step is exact there).  Left empty if the grid cannot be
// made, a leaf's skip is not the next node (the threaded layouts always make it so) or a link does not fit.
// A one-shape leaf's link names its 64-byte record (DLeafRec, qleaves), laid out in octant 0's order so that
// leaves of one subtree share lines.
void build_qnodes(Accel &a, const Scene &sc) {
    const size_t per_oct = a.nodes.size() / BVH_OCTANTS;
    if (!make_grid(a)) return;
    std::vector<DNodeQ> out;
    out.reserve(a.nodes.size());
    // the one-shape leaves' records in octant 0's order
    std::vector<int32_t> rec_of(a.leaf.size() + 1, -1);  // by leaf-list index
    std::vector<DLeafRec> recs;
    for (size_t ni = 0; ni < per_oct; ni++) {
        const DNode &n = a.nodes[ni];
        if (n.count != 1 || !(a.cnodes[ni].first_count >> 31)) continue;
        const int id = a.leaf[n.first];
        const DShape d = to_device(sc.shapes[id]);
        DLeafRec l{};
        l.m[0] = d.inv[0], l.m[1] = d.inv[5], l.m[2] = d.inv[10];
        l.m[3] = d.inv[3], l.m[4] = d.inv[7], l.m[5] = d.inv[11];
        l.shape = id;
        l.axis = d.axis;
        rec_of[n.first] = (int32_t)recs.size();
        recs.push_back(l);
    }
    double bound = 0.0;
    for (int k = 0; k < 3; k++) bound = std::max(bound, std::fabs(a.qg0[k]));
    for (size_t ni = 0; ni < a.nodes.size(); ni++) {
        const DNode &n = a.nodes[ni];
        const int oct = (int)(ni / per_oct);
        DNodeQ c{};
        for (int k = 0; k < 3; k++) {
            const double ql = q_down(a, n.lo[k], k), qh = q_up(a, n.hi[k], k);
            if (a.qg0[k] + ql * a.qgs[k] > n.lo[k] || a.qg0[k] + qh * a.qgs[k] < n.hi[k]) return;  // (cannot happen)
            bound = std::max({bound, std::fabs(a.qg0[k] + ql * a.qgs[k]), std::fabs(a.qg0[k] + qh * a.qgs[k])});
            const bool neg = (oct >> k) & 1;  // the octant's rays move toward -k: hi is the near plane
            c.q[k] = (uint16_t)(neg ? qh : ql);
            c.q[3 + k] = (uint16_t)(neg ? ql : qh);
        }
        if (n.count == 0) {
            if (n.skip < 0) return;
            c.link = (uint32_t)n.skip;
        } else {
            if ((size_t)n.skip != ni % per_oct + 1 || n.count > 63) return;
            const uint32_t fc = a.cnodes[ni].first_count;  // the compact form's leaf: direct id or list index
            const bool direct = fc >> 31;
            uint32_t first = fc & 0xffffffu;
            if (direct) {  // the record of the shape (octant 0 lists every leaf)
                if (rec_of[n.first] < 0) return;
                first = (uint32_t)rec_of[n.first];
            }
            c.link = 1u << 31 | (direct ? 1u << 30 : 0u) | (uint32_t)n.count << 24 | first;
        }
        out.push_back(c);
    }
    a.qnodes.swap(out);
    a.qleaves.swap(recs);
    a.qbound = (float)bound;
    if ((double)a.qbound < bound) a.qbound = std::nextafter(a.qbound, INFINITY);
}

Accel build_accel(const Scene &sc, int json_shapes, int leaf_max) {
    Accel a;
    a.boxes.reserve(sc.shapes.size());
    for (auto &s : sc.shapes) a.boxes.push_back(shape_box(s));
    std::vector<int32_t> rest;
    bool small = json_shapes <= LIN_MAX;
    for (int32_t i = 0; i < (int32_t)sc.shapes.size(); i++) {
        if (sc.shapes[i].type == MARCH) a.march.push_back(i);
        // a Torus root comes from a closed-form quartic whose error has no
        // useful bound: never behind a box (the acceptance rule keeps the
        // linear scan's result in any visiting order)
        else if ((small && i < json_shapes) || sc.shapes[i].type == TORUS) a.lin.push_back(i);
        else rest.push_back(i);
    }
    // A shape whose box dwarfs the typical one (a ground sphere under a field
    // of small ones) would inflate the box of every ancestor of its leaf, so
    // rays would enter those nodes everywhere: it joins the wave-uniform list
    // instead (while that list has room).
    if (rest.size() > 64) {
        auto ext = [&](int32_t i) {
            const DBox &b = a.boxes[i];
            return std::max({b.hi[0] - b.lo[0], b.hi[1] - b.lo[1], b.hi[2] - b.lo[2]});
        };
        std::vector<double> e;
        e.reserve(rest.size());
        for (int32_t i : rest) e.push_back(ext(i));
        std::nth_element(e.begin(), e.begin() + e.size() / 2, e.end());
        const double big = 64.0 * e[e.size() / 2];
        std::vector<int32_t> keep;
        keep.reserve(rest.size());
        for (int32_t i : rest) {
            if (ext(i) > big && a.lin.size() < (size_t)LIN_MAX) a.lin.push_back(i);
            else keep.push_back(i);
        }
        rest.swap(keep);
    }
    if (!rest.empty()) {
        Builder b{a.boxes, a};
        b.leaf_max = std::max(1, std::min(16, leaf_max));
        const int root = b.emit(rest, 0, rest.size());
        a.nodes.reserve(b.tree.size() * BVH_OCTANTS);
        for (int oct = 0; oct < BVH_OCTANTS; oct++) b.thread(root, oct, a.nodes.size());
    }
    a.cnodes.reserve(a.nodes.size());
    const size_t per_oct = a.nodes.size() / BVH_OCTANTS;
    for (size_t ni = 0; ni < a.nodes.size(); ni++) {
        const DNode &n = a.nodes[ni];
        const int oct = per_oct ? (int)(ni / per_oct) : 0;
        if (n.first < 0 || n.first >= (1 << 24) || n.count < 0 || n.count > 255)
            throw std::runtime_error("BVH too large for the compact node form (leaf index >= 2^24)");
        DNodeC c{};
        for (int k = 0; k < 3; k++) {
            float lo = (float)n.lo[k], hi = (float)n.hi[k];
            if ((double)lo > n.lo[k]) lo = std::nextafter(lo, -INFINITY);
            if ((double)hi < n.hi[k]) hi = std::nextafter(hi, INFINITY);
            const bool neg = (oct >> k) & 1;  // the octant's rays move toward -k: hi is the near plane
            c.nr[k] = neg ? hi : lo;
            c.fr[k] = neg ? lo : hi;
        }
        c.skip = n.skip;
        for (int k = 0; k < 3; k++) a.bvh_bound = std::max({a.bvh_bound, std::fabs(c.nr[k]), std::fabs(c.fr[k])});
        // a one-shape leaf holds the shape id itself (bit 31), saving the dependent leaf[] load
        if (n.count == 1 && a.leaf[n.first] >= 0 && a.leaf[n.first] < (1 << 24))
            c.first_count = (uint32_t)a.leaf[n.first] | 1u << 24 | 1u << 31;
        else
            c.first_count = (uint32_t)n.first | (uint32_t)n.count << 24;
        a.cnodes.push_back(c);
    }
    if (per_oct >= (size_t)BIG_BVH_NODES) {
        build_qnodes(a, sc);
    }
    return a;
}

}  // namespace pt
