"""Every ray-marched ShapeFunction of the reference (Heart, Sine, Star,
DupinCyclide, HuntsSurface, Cushion; src/world/shapes/ray_marching.rs:121-520)
through the product's generic skipping march (pt_funcs.hpp + pt_march.hpp,
host build) against the oracle's literal march (oracle/pt_oracle.c), bit for
bit: closest hits on rays aimed at each shape and leaving its surface,
ray_color, whole pixels; plus the loader's handling of the functions' JSON.
Scene: scenes/marched.json (scenes/make_scenes.py)."""
import ctypes as C
import json

import numpy as np
import pytest

import oracle as O
from test_path_host import H, Pair  # noqa: F401  (fixture + helper)

FUNCS = {"DupinCyclide": 2, "Sine": 3, "Star": 4, "HuntsSurface": 5, "Cushion": 6, "Heart": 7}


@pytest.fixture(scope="module")
def marched_text():
    from conftest import scene_text
    return scene_text("marched.json")


@pytest.fixture(scope="module")
def marched(H, marched_text):  # noqa: F811
    return Pair(H, marched_text, random_spheres=False)


def shape_centre(pair, i):
    m = list(pair.o.shape(i).direct)
    return np.array([m[3], m[7], m[11]])


def rays_at(rng, centre, radius, n, eye=(0.0, 3.5, -16.0)):
    """Half camera-like rays aimed into the shape's ball, half from random
    points around it (bounce-like, including origins inside the bound)."""
    eye = np.asarray(eye, float)
    tgt = centre + rng.uniform(-radius, radius, size=(n, 3))
    o = np.tile(eye, (n, 1))
    o[n // 2:] = centre + rng.uniform(-1.6 * radius, 1.6 * radius, size=(n - n // 2, 3))
    d = tgt - o
    d[n // 2:] = rng.normal(size=(n - n // 2, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return np.concatenate([o, d], axis=1)


@pytest.mark.parametrize("name", list(FUNCS))
def test_function_closest_hits_exact(marched, name):
    i = FUNCS[name]
    rng = np.random.default_rng(100 + i)
    hits = 0
    for ray in rays_at(rng, shape_centre(marched, i), 2.0, 500):
        who, t, p, n, f = marched.closest(ray)
        h = marched.o.closest_hit(ray[:3], ray[3:])
        if h is None:
            assert who == -1, ray
        else:
            assert (who, t, p, n, f) == (h.shape, h.t, list(h.point), list(h.normal), h.front_face), ray
            hits += h.shape == i
    assert hits > 10, "too few rays reach the %s" % name


def test_function_ray_color_exact(H, marched):  # noqa: F811
    rng = np.random.default_rng(5)
    out = (C.c_double * 3)()
    for i in FUNCS.values():
        for ray in rays_at(rng, shape_centre(marched, i), 2.0, 60):
            st = C.c_uint64(int(rng.integers(0, 2 ** 63)))
            s0 = st.value
            H.h_ray_color(marched.h, (C.c_double * 6)(*ray), C.byref(st), 8, out)
            want, s1 = marched.o.ray_color(ray[:3], ray[3:], 8, s0)
            assert list(out) == list(want) and st.value == s1


def test_function_pixels_exact(H, marched):  # noqa: F811
    w, h = 320, 180
    rng = np.random.default_rng(4)
    px = rng.choice(w * h, size=160, replace=False).astype(np.uint32)
    out = np.zeros((len(px), 3))
    H.h_trace_pixels(marched.h, w, h, 2, 8, 7, px.ctypes.data_as(C.POINTER(C.c_uint32)), len(px),
                     out.ctypes.data_as(C.POINTER(C.c_double)))
    ref = marched.o.render(w, h, 2, 8, 7, pixels=px)
    assert np.array_equal(out, ref)
    assert out.max() > 0.0


def test_loader_function_parameters(pt, marched_text):
    """pt_scene_get_shape reports each function and its JSON parameters as the
    oracle's loader reads them."""
    ps = pt.Scene.from_json(marched_text, random_spheres=False)
    osc = O.Scene(marched_text, random_spheres=False)
    for i in FUNCS.values():
        g, o = ps.shape(i), osc.shape(i)
        assert g.type == O.MARCH and g.func == o.func
        assert (g.a, g.b, g.c, g.d, g.sphere_radius) == (o.fa, o.fb, o.fc, o.fd, o.fr)
        assert (g.step, g.depth) == (o.step, o.depth)
        assert list(g.inverse) == list(o.inverse)


@pytest.mark.parametrize("shape,code", [({"type": "Sine", "a": 1.0}, "PT_ERR_PARSE"),  # missing sphere_radius
                                         ({"type": "DupinCyclide", "a": 1, "b": 1, "c": 1, "sphere_radius": 2},
                                          "PT_ERR_PARSE"),  # missing d
                                         ({"type": "Teapot"}, "PT_ERR_PARSE")])
def test_loader_function_errors(pt, marched_text, shape, code):
    js = json.loads(marched_text)
    js["shapes"][2]["shape"] = shape
    with pytest.raises(pt.PtError) as e:
        pt.Scene.from_json(json.dumps(js), random_spheres=False)
    assert e.value.code == getattr(pt, code)
