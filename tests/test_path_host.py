"""The product's sample-path code (pt_device.hpp: uniform list + threaded BVH +
skipping march + flat per-lane sample loop), compiled for the host by
tests/native/Makefile, against the oracle — bit for bit, on the CPU.  The GPU
tests repeat the comparison with the same code compiled for gfx950."""
import ctypes as C
import json
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle as O
from conftest import native_lib

NATIVE = Path(__file__).resolve().parent / "native"


@pytest.fixture(scope="module")
def H():
    subprocess.run(["make", "-s", "-C", str(NATIVE)], check=True)
    L = C.CDLL(native_lib("libpath.so"))
    d = C.POINTER(C.c_double)
    L.h_scene_new.restype = C.c_void_p
    L.h_scene_new.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_uint64]
    L.h_scene_free.argtypes = [C.c_void_p]
    L.h_accel_stats.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
    L.h_node_check.argtypes = [C.c_void_p]
    L.h_closest.argtypes = [C.c_void_p, d, C.c_double, C.c_double, d, d, d, C.POINTER(C.c_int)]
    L.h_ray_color.argtypes = [C.c_void_p, d, C.POINTER(C.c_uint64), C.c_uint32, d]
    L.h_trace_pixels.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64,
                                 C.POINTER(C.c_uint32), C.c_size_t, d]
    return L


class Pair:
    def __init__(self, H, text, seed=1, random_spheres=True):
        raw = text.encode()
        self.H = H
        self.h = H.h_scene_new(raw, len(raw), 1 if random_spheres else 0, seed)
        assert self.h
        self.o = O.Scene(text, random_spheres=random_spheres, seed=seed)

    def __del__(self):
        self.H.h_scene_free(self.h)

    def closest(self, ray, min_t=0.001, max_t=float("inf")):
        t, p, n, f = C.c_double(), (C.c_double * 3)(), (C.c_double * 3)(), C.c_int()
        who = self.H.h_closest(self.h, (C.c_double * 6)(*ray), min_t, max_t, C.byref(t), p, n, C.byref(f))
        return who, t.value, list(p), list(n), f.value


@pytest.fixture(scope="module")
def cornell(H, cornell_text):
    return Pair(H, cornell_text)


def rays_cornell(rng, n):
    o = rng.uniform([-20, 0, -20], [555, 555, 555], size=(n, 3))
    o[: n // 3] = [278, 278, -800]
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    # aim a third at the Heart region and a sixth at the random-sphere corner
    k = n // 3
    tgt = rng.uniform([140, 130, 80], [285, 270, 215], size=(k, 3))
    d[:k] = tgt - o[:k]
    m = n // 6
    o[k:k + m] = rng.uniform([-30, 1, -30], [30, 5, 30], (m, 3))
    d[k:k + m] = rng.uniform([-11, 0, -11], [11, 0.5, 11], (m, 3)) - o[k:k + m]
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return np.concatenate([o, d], axis=1)


def test_accel_layout(H, cornell):
    st = (C.c_int * 4)()
    H.h_accel_stats(cornell.h, st)
    nodes, nlin, nmarch, nleaf = list(st)
    assert nlin == 8 and nmarch == 1  # 6 rectangles + 2 cubes uniform; the Heart marched last
    assert nleaf == cornell.o.num_shapes - 9  # every random sphere sits in the BVH once


def test_compact_nodes_contain_host_boxes(H, cornell):
    # DNodeC (pt_types.hpp): f32 boxes rounded outward must contain the f64 boxes, and the packed
    # first/count (or the direct shape id of a one-shape leaf) must decode to the host node's leaf
    assert H.h_node_check(cornell.h) == 0


def test_closest_hit_matches_oracle(cornell):
    rng = np.random.default_rng(21)
    for ray in rays_cornell(rng, 3000):
        who, t, p, n, f = cornell.closest(ray)
        h = cornell.o.closest_hit(ray[:3], ray[3:])
        if h is None:
            assert who == -1
        else:
            assert (who, t, p, n, f) == (h.shape, h.t, list(h.point), list(h.normal), h.front_face), ray


def test_closest_hit_max_t(cornell):
    rng = np.random.default_rng(2)
    for ray in rays_cornell(rng, 300):
        for max_t in (200.0, 900.0):
            who, t, *_ = cornell.closest(ray, 0.001, max_t)
            h = cornell.o.closest_hit(ray[:3], ray[3:], 0.001, max_t)
            assert (who, t if who >= 0 else None) == ((h.shape, h.t) if h else (-1, None))


def test_ray_color_matches_oracle(H, cornell):
    rng = np.random.default_rng(8)
    out = (C.c_double * 3)()
    for i, ray in enumerate(rays_cornell(rng, 600)):
        st = C.c_uint64(int(rng.integers(0, 2 ** 63)))
        s0 = st.value
        H.h_ray_color(cornell.h, (C.c_double * 6)(*ray), C.byref(st), 8, out)
        want, s1 = cornell.o.ray_color(ray[:3], ray[3:], 8, s0)
        assert list(out) == list(want) and st.value == s1


@pytest.mark.parametrize("scene,depth,seed", [("cornell_box.json", 8, 1), ("spheres.json", 50, 3),
                                              ("cornell_box.json", 0, 2)])
def test_trace_pixels_match_oracle(H, scene, depth, seed):
    from conftest import scene_text
    pr = Pair(H, scene_text(scene), seed=seed)
    w, h = 1920, 1080
    rng = np.random.default_rng(seed)
    px = rng.choice(w * h, size=120, replace=False).astype(np.uint32)
    out = np.zeros((len(px), 3))
    H.h_trace_pixels(pr.h, w, h, 2, depth, seed, px.ctypes.data_as(C.POINTER(C.c_uint32)), len(px),
                     out.ctypes.data_as(C.POINTER(C.c_double)))
    ref = pr.o.render(w, h, 2, depth, seed, pixels=px)
    assert np.array_equal(out, ref)


def test_many_json_shapes_go_to_bvh(H):
    """Above LIN_MAX JSON shapes everything non-marched is in the BVH (config C5)."""
    shapes = [{"type": "Sphere", "name": "S%d" % i, "material": "M",
               "transform": {"translate": [i % 7 - 3.0, 0.3 * (i // 7), 5.0 + i * 0.01], "rotate": [0, 0, 0],
                             "scale": [0.2, 0.2, 0.2]}} for i in range(60)]
    js = {"camera": {"position": [0, 0, -5], "direction": [0, 0, 1], "up": [0, 1, 0], "fov": 60, "focal_length": 1},
          "shapes": shapes, "materials": {"M": {"type": "Metal", "albedo": {"type": "SolidColor", "color": [0.8, 0.7, 0.6]},
                                                "fuzz": 0.2}}, "background": [0, 0, 0]}
    pr = Pair(H, json.dumps(js), random_spheres=False)
    st = (C.c_int * 4)()
    H.h_accel_stats(pr.h, st)
    assert st[1] == 0 and st[3] == 60
    rng = np.random.default_rng(4)
    for _ in range(500):
        o = rng.uniform([-4, -1, -6], [4, 4, -4])
        d = rng.uniform([-4, -1, 4], [4, 4, 6]) - o
        d /= np.linalg.norm(d)
        who, t, *_ = pr.closest(np.concatenate([o, d]))
        h = pr.o.closest_hit(o, d)
        assert (who, t if who >= 0 else None) == ((h.shape, h.t) if h else (-1, None))


def test_synthetic_field_ground_sphere_uniform_and_octant_bvh(H):
    """C5's recipe at 3,000 spheres: the radius-1000 ground sphere leaves the
    BVH for the wave-uniform list (its box would inflate every ancestor), the
    rest sit in the 8 octant-ordered layouts; closest hits and pixel samples
    equal the oracle's linear scan bit for bit."""
    import sys
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "scenes"))
    import make_scenes
    text = json.dumps(make_scenes.synthetic(3000))
    pr = Pair(H, text, seed=1)
    st = (C.c_int * 4)()
    H.h_accel_stats(pr.h, st)
    nodes, nlin, nmarch, nleaf = list(st)
    assert nlin == 1 and nmarch == 0 and nleaf == pr.o.num_shapes - 1
    rng = np.random.default_rng(5)
    for _ in range(1500):
        o = rng.uniform([-15, 0.05, -15], [15, 3, 15])
        d = rng.normal(size=3)
        d[1] = -abs(d[1]) if rng.random() < 0.7 else d[1]
        d /= np.linalg.norm(d)
        who, t, p, n, f = pr.closest(np.concatenate([o, d]))
        h = pr.o.closest_hit(o, d)
        if h is None:
            assert who == -1
        else:
            assert (who, t, p, n, f) == (h.shape, h.t, list(h.point), list(h.normal), h.front_face)
    w, h = 320, 180
    px = rng.choice(w * h, size=60, replace=False).astype(np.uint32)
    out = np.zeros((len(px), 3))
    H.h_trace_pixels(pr.h, w, h, 2, 8, 3, px.ctypes.data_as(C.POINTER(C.c_uint32)), len(px),
                     out.ctypes.data_as(C.POINTER(C.c_double)))
    assert np.array_equal(out, pr.o.render(w, h, 2, 8, 3, pixels=px))


def test_bvh_walk_signed_zero_and_axis_rays(H):
    """The BVH stores each octant's boxes as near/far planes picked by the
    direction's sign bits and intersects them with t = fma(b, 1/d, -o/d): rays
    with +0 / -0 components (1/d = +-inf, NaN t's), axis-parallel rays and
    origins on the spheres' bounding planes must still find the oracle's
    closest hit (the cull has to stay conservative)."""
    import sys
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "scenes"))
    import make_scenes
    pr = Pair(H, json.dumps(make_scenes.synthetic(400)), seed=1)
    rng = np.random.default_rng(11)
    spheres = [s for s in make_scenes.synthetic(400)["shapes"][1:]]
    rays = []
    for _ in range(600):
        c = np.array(spheres[rng.integers(len(spheres))]["transform"]["translate"], float)
        # (not tangent to a sphere: a ray with disc == 0 takes the reference's unranged root, whose winner
        # depends on the visiting order)
        o = c + rng.choice([-0.2000001, 0.2000001, 0.1, 0.0], size=3) + rng.choice([0.0, 0.5, -0.5], size=3)
        o[1] = max(o[1], 0.05)
        d = np.zeros(3)
        k = rng.integers(3)
        d[k] = rng.choice([-1.0, 1.0])
        for j in range(3):
            if j != k:
                d[j] = rng.choice([0.0, -0.0, 1e-300, -1e-300, rng.normal() * 0.3])
        d /= np.linalg.norm(d)
        rays.append(np.concatenate([o, d]))
    hits = 0
    for ray in rays:
        who, t, p, n, f = pr.closest(ray)
        h = pr.o.closest_hit(ray[:3], ray[3:])
        if h is None:
            assert who == -1, ray
        else:
            hits += 1
            assert (who, t, p, n, f) == (h.shape, h.t, list(h.point), list(h.normal), h.front_face), ray
    assert hits > 100


def test_bvh_fma_slab_build_same_hits(H):
    """The bounce build for large BVHs computes the node planes' t as fma(b, 1/d, -o/d) (FMA_SLAB); on the
    synthetic field, with random and signed-zero / axis-parallel rays, it returns the same (shape, t) as the
    subtract-multiply build (the culls differ only in rounding, far inside the boxes' padding)."""
    import sys
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "scenes"))
    import make_scenes
    H.h_closest_nomarch.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_double)]
    scene = make_scenes.synthetic(3000)
    pr = Pair(H, json.dumps(scene), seed=1)
    rng = np.random.default_rng(17)
    centres = [np.array(s["transform"]["translate"], float) for s in scene["shapes"][1:]]
    hits = 0
    for i in range(4000):
        if i % 2:
            o = rng.uniform([-15, 0.05, -15], [15, 3, 15])
            d = rng.normal(size=3)
        else:
            o = centres[rng.integers(len(centres))] + rng.choice([-0.2000001, 0.2000001, 0.0], size=3)
            o[1] = max(o[1], 0.05)
            d = np.zeros(3)
            d[rng.integers(3)] = rng.choice([-1.0, 1.0])
            d = np.where(d == 0, rng.choice([0.0, -0.0, 1e-300, rng.normal() * 0.3], size=3), d)
        d /= np.linalg.norm(d)
        ray = (C.c_double * 6)(*np.concatenate([o, d]))
        t0, t1, t2 = C.c_double(), C.c_double(), C.c_double()
        w0 = H.h_closest_nomarch(pr.h, ray, 0, C.byref(t0))
        w1 = H.h_closest_nomarch(pr.h, ray, 1, C.byref(t1))
        w2 = H.h_closest_nomarch(pr.h, ray, 2, C.byref(t2))  # the quantized nodes (wf_walk)
        assert (w0, t0.value) == (w1, t1.value) == (w2, t2.value), (o, d)
        hits += w0 >= 0
    assert hits > 1000


def test_quantized_nodes_contain_the_boxes(H):
    """The 16-byte nodes of the large-tree walk (DNodeQ): every box on the per-axis grid contains the node's f64
    box (lo rounded down, hi up), interior links are the skips and leaf links decode to the leaf's shapes (a
    one-shape leaf through its 64-byte record, whose axis entries are the shape's)."""
    import sys
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "scenes"))
    import make_scenes
    H.h_qnode_check.argtypes = [C.c_void_p]
    pr = Pair(H, json.dumps(make_scenes.synthetic(3000)), seed=1)
    assert H.h_qnode_check(pr.h) == 0


def test_bvh_fma_slab_tiny_direction_component(H):
    """FMA_SLAB with a direction component so small that 1/d is finite but o/d
    overflows (|d| ~ 1e-308, |o| ~ 10): the plane t's of that axis must not
    become +-inf and cull the node that holds the hit.  Both
    builds must return the oracle's closest hit."""
    import sys
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "scenes"))
    import make_scenes
    H.h_closest_nomarch.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_double)]
    scene = make_scenes.synthetic(3000)
    pr = Pair(H, json.dumps(scene), seed=1)
    rng = np.random.default_rng(23)
    centres = [np.array(s["transform"]["translate"], float) for s in scene["shapes"][1:]]
    hits = 0
    for _ in range(600):
        c = centres[rng.integers(len(centres))]
        if max(abs(c[0]), abs(c[2])) < 3:
            continue
        ax = 0 if abs(c[2]) > abs(c[0]) else 2  # travel along an axis; the tiny component on the large one
        tiny = 2 - ax
        o = c.copy()
        o[ax] -= rng.choice([-1.0, 1.0]) * 1.5
        o[1] += rng.uniform(-0.1, 0.1)
        o[tiny] += rng.uniform(-0.1, 0.1)
        d = np.zeros(3)
        d[ax] = 1.0 if c[ax] > o[ax] else -1.0
        d[tiny] = rng.choice([1e-308, -1e-308, 3e-308, -5e-309])
        ray6 = np.concatenate([o, d])
        ray = (C.c_double * 6)(*ray6)
        ref = pr.o.closest_hit(o, d)
        for fma in (0, 1, 2):
            t = C.c_double()
            w = H.h_closest_nomarch(pr.h, ray, fma, C.byref(t))
            if ref is None:
                assert w == -1, (fma, ray6)
            else:
                assert (w, t.value) == (ref.shape, ref.t), (fma, ray6, w, ref.shape)
        hits += ref is not None
    assert hits > 200


def test_large_tree_walk_far_origins_and_grazing_rays(H):
    """The large-tree walk (fma = 1: FMA_SLAB, its f32 slab widened by the error bound; fma = 2:
    the quantized nodes, their grid folded into the widened offsets) keeps
    every node that holds the closest hit: rays from origins up to 1e5 away, aimed to graze spheres' silhouettes
    (|t| large, planes far from the origin), and rays leaving from sphere surfaces at shallow angles."""
    import sys
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "scenes"))
    import make_scenes
    H.h_closest_nomarch.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_double)]
    scene = make_scenes.synthetic(3000)
    pr = Pair(H, json.dumps(scene), seed=1)
    rng = np.random.default_rng(41)
    centres = [np.array(s["transform"]["translate"], float) for s in scene["shapes"][1:]]
    hits = 0
    for i in range(3000):
        c = centres[rng.integers(len(centres))]
        if i % 2:
            far = 10.0 ** rng.uniform(1, 5)
            o = c + rng.normal(size=3) * far
            o[1] = abs(o[1]) + 0.05
            side = np.cross(c - o, rng.normal(size=3))
            tgt = c + side / np.linalg.norm(side) * 0.2 * rng.uniform(0.999, 1.001)  # the silhouette
            d = tgt - o
        else:
            n = rng.normal(size=3)
            n /= np.linalg.norm(n)
            o = c + n * 0.2000001
            o[1] = max(o[1], 0.05)
            d = np.cross(n, rng.normal(size=3)) + n * rng.uniform(1e-9, 1e-3)  # nearly tangent
        d /= np.linalg.norm(d)
        ray = (C.c_double * 6)(*np.concatenate([o, d]))
        t0, t1, t2 = C.c_double(), C.c_double(), C.c_double()
        w0 = H.h_closest_nomarch(pr.h, ray, 0, C.byref(t0))
        w1 = H.h_closest_nomarch(pr.h, ray, 1, C.byref(t1))
        w2 = H.h_closest_nomarch(pr.h, ray, 2, C.byref(t2))  # the quantized nodes (wf_walk)
        assert (w0, t0.value) == (w1, t1.value) == (w2, t2.value), (o, d)
        hits += w0 >= 0
    assert hits > 500



def test_quantized_grid_refuses_unbounded_extents(H):
    """Shapes near +-1e308 make the root box's extent overflow to inf: the quantized grid is not built (the walk
    falls back to the 32-byte nodes) instead of the grid search looping forever, and hits still match."""
    import sys
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "scenes"))
    import make_scenes
    H.h_closest_nomarch.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_double)]
    scene = make_scenes.synthetic(400)
    far = json.loads(json.dumps(scene["shapes"][1]))
    for j in range(40):  # (more than the wave-uniform list takes: the rest go to the BVH)
        for sign in (1.0, -1.0):
            s2 = json.loads(json.dumps(far))
            s2["transform"]["translate"] = [sign * 1.5e308, 0.5 + j, 0.0]
            scene["shapes"].append(s2)
    pr = Pair(H, json.dumps(scene), seed=1)  # (returns: no endless loop in the grid builder)
    t = C.c_double()
    assert H.h_closest_nomarch(pr.h, (C.c_double * 6)(0, 2, 0, 0, -1, 0), 2, C.byref(t)) == -2  # no quantized nodes
    for fma in (0, 1):
        who = H.h_closest_nomarch(pr.h, (C.c_double * 6)(0, 2, 0, 0.01, -1, 0.02), fma, C.byref(t))
        assert who >= 0
