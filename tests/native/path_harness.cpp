// Test-only host build of the product's sample path: the same pt_device.hpp
// functions the HIP kernels run, compiled for the CPU, on a scene realized by
// the product's own loader and BVH builder.  Lets the CPU suite compare the
// GPU algorithm (uniform list + threaded BVH + skipping march + flat sample
// loop) with the oracle bit for bit.  Never used by the product.
#include <cmath>
#include <cstring>
#include <vector>

#include "../../rs-pathtracing_amd/csrc/pt_accel.hpp"
#include "../../rs-pathtracing_amd/csrc/pt_device.hpp"
#include "../../rs-pathtracing_amd/csrc/pt_scene.hpp"

using namespace pt;

struct Bundle {
    Scene sc;
    Accel acc;
    std::vector<DQGrid> qbuf;  // the quantized layouts after their grid, as the device buffer (DQGrid-aligned)
    std::vector<DShape> shapes;
    std::vector<DMaterial> mats;
    dev::Scene view;
    double s11;
};

extern "C" void *h_scene_new(const char *json, size_t len, int random_spheres, uint64_t seed) {
    try {
        Bundle *b = new Bundle();  // value-initialised: every dev::Scene field not set below is 0 (cancel: none)
        b->sc = scene_from_json(json, len, random_spheres != 0, seed);
        b->acc = build_accel(b->sc, b->sc.json_shapes);
        for (auto &s : b->sc.shapes) b->shapes.push_back(to_device(s));
        for (auto &m : b->sc.materials) b->mats.push_back(to_device(m));
        b->view.shapes = b->shapes.data();
        b->view.mats = b->mats.data();
        b->view.nodes = b->acc.cnodes.data();
        b->view.leaf = b->acc.leaf.data();
        b->view.lin = b->acc.lin.data();
        b->view.march = b->acc.march.data();
        b->view.boxes = b->acc.boxes.data();
        const bool tex = !b->sc.textures.empty();
        b->view.tex = tex ? b->sc.textures.data() : nullptr;
        b->view.perlin = tex ? b->sc.perlins.data() : nullptr;
        b->view.images = tex ? b->sc.images.data() : nullptr;
        b->view.pixels = tex ? b->sc.pixels.data() : nullptr;
        if (b->acc.qnodes.empty() && !b->acc.nodes.empty()) build_qnodes(b->acc, b->sc);  // (small trees too)
        if (!b->acc.qnodes.empty()) {
            const size_t nb = b->acc.qnodes.size() * sizeof(DNodeQ);
            const size_t ro = qleaf_offset(b->acc.nodes_per_octant()), rb = b->acc.qleaves.size() * sizeof(DLeafRec);
            b->qbuf.resize((ro + rb + sizeof(DQGrid) - 1) / sizeof(DQGrid) + 1);  // (+ padding, the leaf records)
            if (rb) std::memcpy((char *)b->qbuf.data() + ro, b->acc.qleaves.data(), rb);
            DQGrid &g = b->qbuf[0];
            for (int k = 0; k < 3; k++) g.g0[k] = b->acc.qg0[k], g.gs[k] = b->acc.qgs[k];
            g.bound = b->acc.qbound;
            std::memcpy(&b->qbuf[1], b->acc.qnodes.data(), nb);
            b->view.qnodes = b->qbuf.data();
        }
        b->view.nnodes = b->acc.nodes_per_octant();
        b->view.bvh_bound = b->acc.bvh_bound;
        b->view.nlin = (int)b->acc.lin.size();
        b->view.nmarch = (int)b->acc.march.size();
        b->view.diag = 0;
        b->s11 = uniform_incl_scale(-1.0, 1.0);
        return b;
    } catch (...) {
        return nullptr;
    }
}
extern "C" void h_scene_free(void *p) { delete (Bundle *)p; }
extern "C" void h_accel_stats(void *p, int *out) {
    Bundle *b = (Bundle *)p;
    out[0] = b->acc.nodes_per_octant();
    out[1] = (int)b->acc.lin.size();
    out[2] = (int)b->acc.march.size();
    out[3] = (int)b->acc.leaf.size();
}

// Device node form against the host nodes: each f32 box must contain the f64
// box, skip must match, and first/count must decode to the same leaf shapes.
// Returns the number of nodes that fail (0 expected).
extern "C" int h_node_check(void *p) {
    Bundle *b = (Bundle *)p;
    const auto &N = b->acc.nodes;
    const auto &Cn = b->acc.cnodes;
    if (N.size() != Cn.size()) return -1;
    int bad = 0;
    for (size_t i = 0; i < N.size(); i++) {
        bool ok = Cn[i].skip == N[i].skip;
        const size_t per = N.size() / BVH_OCTANTS;
        const int oct = per ? (int)(i / per) : 0;  // layout oct stores (near, far) planes: (hi, lo) on its negative axes
        for (int k = 0; k < 3; k++) {
            const bool neg = (oct >> k) & 1;
            const double lo = neg ? Cn[i].fr[k] : Cn[i].nr[k], hi = neg ? Cn[i].nr[k] : Cn[i].fr[k];
            ok = ok && lo <= N[i].lo[k] && hi >= N[i].hi[k];
        }
        const uint32_t fc = Cn[i].first_count;
        const int count = (int)(fc >> 24 & 0x7fu), first = (int)(fc & 0xffffffu);
        ok = ok && count == N[i].count;
        if (fc >> 31) ok = ok && count == 1 && first == b->acc.leaf[N[i].first];
        else ok = ok && first == N[i].first;
        bad += !ok;
    }
    return bad;
}

// The quantized nodes against the host nodes: every quantized box (g0 + q gs, in f64) must contain the f64 box,
// an interior node's link must be its skip and a leaf's must decode to its shapes.  Returns the failures (0
// expected), or -1 without quantized nodes.
extern "C" int h_qnode_check(void *p) {
    Bundle *b = (Bundle *)p;
    const auto &N = b->acc.nodes;
    const auto &Q = b->acc.qnodes;
    const auto &Cn = b->acc.cnodes;
    if (Q.size() != N.size() || N.empty()) return -1;
    const size_t per = N.size() / BVH_OCTANTS;
    int bad = 0;
    for (size_t i = 0; i < N.size(); i++) {
        const int oct = (int)(i / per);
        bool ok = true;
        for (int k = 0; k < 3; k++) {
            const bool neg = (oct >> k) & 1;
            const double ql = neg ? Q[i].q[3 + k] : Q[i].q[k], qh = neg ? Q[i].q[k] : Q[i].q[3 + k];
            const double lo = b->acc.qg0[k] + ql * b->acc.qgs[k], hi = b->acc.qg0[k] + qh * b->acc.qgs[k];
            ok = ok && lo <= N[i].lo[k] && hi >= N[i].hi[k] && std::fabs(lo) <= b->acc.qbound &&
                 std::fabs(hi) <= b->acc.qbound;
        }
        const uint32_t l = Q[i].link;
        if (N[i].count == 0) {
            ok = ok && !(l >> 31) && (int32_t)l == N[i].skip;
        } else {
            const uint32_t fc = Cn[i].first_count;
            const bool rec = (l >> 30) & 1u;  // a one-shape leaf's record names the shape
            const uint32_t named = rec ? ((l & 0xffffffu) < b->acc.qleaves.size()
                                              ? (uint32_t)b->acc.qleaves[l & 0xffffffu].shape : ~0u)
                                       : (l & 0xffffffu);
            if (rec && named != ~0u) {  // the record's axis entries are its shape's
                const DLeafRec &L = b->acc.qleaves[l & 0xffffffu];
                const DShape &S = b->shapes[named];
                ok = ok && L.axis == S.axis && L.m[0] == S.inv[0] && L.m[1] == S.inv[5] && L.m[2] == S.inv[10] &&
                     L.m[3] == S.inv[3] && L.m[4] == S.inv[7] && L.m[5] == S.inv[11];
            }
            ok = ok && (l >> 31) && (int)(l >> 24 & 0x3fu) == N[i].count && named == (fc & 0xffffffu) &&
                 ((l >> 30) & 1u) == (fc >> 31) && (size_t)N[i].skip == i % per + 1;
        }
        bad += !ok;
    }
    return bad;
}

extern "C" int h_closest(void *p, const double *ray, double min_t, double max_t, double *t, double *point,
                         double *normal, int *front) {
    Bundle *b = (Bundle *)p;
    dev::Ray r;
    r.o = dev::v3(ray[0], ray[1], ray[2]);
    r.d = dev::v3(ray[3], ray[4], ray[5]);
    int who = dev::closest(b->view, r, min_t, max_t, t);
    if (who >= 0) {
        dev::Hit h = dev::finish(b->shapes[who], r, *t);
        point[0] = h.p.x, point[1] = h.p.y, point[2] = h.p.z;
        normal[0] = h.n.x, normal[1] = h.n.y, normal[2] = h.n.z;
        *front = h.front;
    }
    return who;
}

extern "C" void h_ray_color(void *p, const double *ray, uint64_t *state, uint32_t depth, double *out) {
    Bundle *b = (Bundle *)p;
    dev::Ray r;
    r.o = dev::v3(ray[0], ray[1], ray[2]);
    r.d = dev::v3(ray[3], ray[4], ray[5]);
    dev::Rng rng{*state};
    std::vector<double> vals((depth + 1) * 3);  // textured attenuation values of this one lane
    dev::V3 c = depth <= 8 ? dev::ray_color<4, true>(b->view, r, depth, rng, b->s11, vals.data(), 1)
                           : dev::ray_color<32, true>(b->view, r, depth, rng, b->s11, vals.data(), 1);
    *state = rng.s;
    out[0] = c.x, out[1] = c.y, out[2] = c.z;
}

extern "C" void h_trace_pixels(void *p, uint32_t w, uint32_t h, uint32_t spp, uint32_t depth, uint64_t seed,
                               const uint32_t *pixels, size_t n, double *out) {
    Bundle *b = (Bundle *)p;
    FrameParams P;
    std::memset(&P, 0, sizeof P);
    caster_params(b->sc.camera, w, h, &P);
    P.s11 = b->s11;
    P.seed = seed;
    P.width = w;
    P.height = h;
    P.spp = spp;
    P.depth = depth;
    std::vector<double> vals((depth + 1) * 3);
    for (size_t i = 0; i < n; i++) {
        dev::V3 c = depth <= 8 ? dev::trace_pixel<4, false, false, march::F_ANY, true>(
                                     b->view, P, pixels[i] % w, pixels[i] / w, nullptr, nullptr, vals.data(), 1)
                               : dev::trace_pixel<32, false, false, march::F_ANY, true>(
                                     b->view, P, pixels[i] % w, pixels[i] / w, nullptr, nullptr, vals.data(), 1);
        out[3 * i] = c.x, out[3 * i + 1] = c.y, out[3 * i + 2] = c.z;
    }
}

// trace_pixel's STATS build on the host: the event counters pt_count_work
// returns from the GPU, for an equality check.
extern "C" void h_count_work(void *p, uint32_t w, uint32_t h, uint32_t spp, uint32_t depth, uint64_t seed,
                             const uint32_t *pixels, size_t n, uint64_t *counters) {
    Bundle *b = (Bundle *)p;
    FrameParams P;
    std::memset(&P, 0, sizeof P);
    caster_params(b->sc.camera, w, h, &P);
    P.s11 = b->s11;
    P.seed = seed;
    P.width = w;
    P.height = h;
    P.spp = spp;
    P.depth = depth;
    Ctr c;
    std::memset(&c, 0, sizeof c);
    std::vector<double> vals((depth + 1) * 3);
    for (size_t i = 0; i < n; i++) {
        if (depth <= 8)
            dev::trace_pixel<4, true, false, march::F_ANY, true>(b->view, P, pixels[i] % w, pixels[i] / w, &c, nullptr,
                                                                 vals.data(), 1);
        else
            dev::trace_pixel<32, true, false, march::F_ANY, true>(b->view, P, pixels[i] % w, pixels[i] / w, &c,
                                                                  nullptr, vals.data(), 1);
    }
    for (int k = 0; k < C_COUNT; k++) counters[k] = c.c[k];
}

// The non-marched closest hit (uniform list + BVH) with the BVH slab in one of
// its two arithmetic forms: fma = 0 (b - o) * 1/d, 1 fma(b, 1/d, -o/d) (the
// FMA_SLAB bounce build for large BVHs).  Both must give the same (who, t).
extern "C" int h_closest_nomarch(void *p, const double *ray, int fma, double *t) {
    Bundle *b = (Bundle *)p;
    dev::Ray r;
    r.o = dev::v3(ray[0], ray[1], ray[2]);
    r.d = dev::v3(ray[3], ray[4], ray[5]);
    const dev::V3 inv = dev::v3(1.0 / r.d.x, 1.0 / r.d.y, 1.0 / r.d.z);
    double best = __builtin_inf();
    int who = -1;
    if (fma == 2) {  // the quantized nodes (wf_walk's build)
        if (!b->view.qnodes) return -2;
        dev::closest_nomarch<false, false, true, true>(b->view, r, inv, T_MIN, &best, &who);
    } else if (fma) {
        dev::closest_nomarch<false, false, true>(b->view, r, inv, T_MIN, &best, &who);
    } else {
        dev::closest_nomarch<false, false, false>(b->view, r, inv, T_MIN, &best, &who);
    }
    *t = best;
    return who;
}

// Per ray, the large-tree walk's node tests (the quantized binary layouts, wf_walk's build): counts[i] for ray i
// (6 doubles each), with the closest hit's shape and t (the SIMT-cost analysis of scripts/walk_lanes.py).
extern "C" int h_walk_counts(void *p, const double *rays, size_t n, uint32_t *counts, int *who, double *t) {
    Bundle *b = (Bundle *)p;
    if (!b->view.qnodes) return -1;
    for (size_t i = 0; i < n; i++) {
        dev::Ray r;
        r.o = dev::v3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]);
        r.d = dev::v3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
        const dev::V3 inv = dev::v3(1.0 / r.d.x, 1.0 / r.d.y, 1.0 / r.d.z);
        Ctr c;
        std::memset(&c, 0, sizeof c);
        double best = __builtin_inf();
        int w = -1;
        dev::closest_nomarch<true, false, true, true>(b->view, r, inv, T_MIN, &best, &w, &c);
        counts[i] = (uint32_t)c.c[C_NODE_SLABS];
        who[i] = w;
        t[i] = best;
    }
    return 0;
}
