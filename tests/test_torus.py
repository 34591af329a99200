"""Torus (src/world/shapes/mod.rs:400-494) and solve_quantic_equation
(src/algebra/equation.rs:17-67) on the CPU: the oracle's restatement against
the reference's own test inputs (equation.rs:69-122 and mod.rs:849-877, which
only print, so their results are checked here against numpy and geometry),
the product loader, and the product's device code compiled for the host
against the oracle, bit for bit."""
import ctypes as C
import json
import math
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle as O
from conftest import native_lib

ROOT = Path(__file__).resolve().parent.parent
NATIVE = ROOT / "tests" / "native"


def quartic(a, b, c, d, e):
    re, im = (C.c_double * 4)(), (C.c_double * 4)()
    O.lib().or_solve_quartic(a, b, c, d, e, re, im)
    return np.array(re[:]) + 1j * np.array(im[:])


@pytest.mark.parametrize("coef", [(3.0, 6.0, -123.0, -126.0, 1080.0), (-20.0, 5.0, 17.0, -29.0, 87.0),
                                  (1.0, -4.0, 6.48, -4.96, 1.0376)])
def test_quartic_on_the_reference_test_polynomials(coef):
    roots = quartic(*coef)
    want = np.roots(coef)
    # the closed form is ill-conditioned: compare as root sets, to 1e-6
    for r in roots:
        assert np.min(np.abs(want - r)) < 1e-6 * max(1.0, abs(r)), (roots, want)
    for w in want:
        assert np.min(np.abs(roots - w)) < 1e-6 * max(1.0, abs(w)), (roots, want)


def torus_scene(R=0.5, r=0.1, t=(0, 0, 0), rot=(0, 0, 0), s=(1, 1, 1)):
    return json.dumps({
        "camera": {"position": [0, 0, -5], "direction": [0, 0, 1], "up": [0, 1, 0], "fov": 40, "focal_length": 1},
        "shapes": [{"type": "Torus", "name": "Torus", "radius": R, "tube_radius": r,
                    "transform": {"translate": list(t), "rotate": list(rot), "scale": list(s)}, "material": "M"}],
        "materials": {"M": {"type": "EmptyMaterial"}}, "background": [0, 0, 0]})


def test_reference_test_torus_ray_misses():
    # test_torus (mod.rs:849-877): from (0, 0, -10) moving further away in z
    sc = O.Scene(torus_scene(), random_spheres=False)
    d = [0.42233513247717097, 0.26611434880691537, -0.86649650272494549]
    assert sc.closest_hit([0.0, 0.0, -10.0], d) is None


def test_axis_ray_hits_the_outer_equator():
    sc = O.Scene(torus_scene(R=1.0, r=0.3), random_spheres=False)
    h = sc.closest_hit([-5.0, 0.0, 0.0], [1.0, 0.0, 0.0])
    assert h is not None and abs(h.t - 3.7) < 1e-6
    assert np.allclose(list(h.normal), [-1.0, 0.0, 0.0], atol=1e-6)
    # u, v of mod.rs:466-467 at p = (-1.3, 0, 0): theta = 0, phi = acos(0) + pi
    assert abs(h.v) < 1e-9 and abs(h.u - (math.acos(0.0) + math.pi) / (2 * math.pi)) < 1e-9
    # through the hole along z: no hit
    assert sc.closest_hit([0.0, 0.0, -5.0], [0.0, 0.0, 1.0]) is None
    # Reference quirk, reproduced: along z through the tube's centre line
    # (true roots 4.7 and 5.3) the closed form returns four complex roots
    # (5 +- 1.38i), so approx_equal(im, 0) rejects them all and the ray misses.
    roots = quartic(1.0, -20.0, 153.82, -538.2, 720.1481)  # the coefficients of mod.rs:434-447 for that ray
    assert np.all(np.abs(roots.imag) > 1.0)
    assert sc.closest_hit([1.0, 0.0, -5.0], [0.0, 0.0, 1.0]) is None


def test_loader_takes_torus(pt):
    a = pt.Scene.from_json(torus_scene(R=0.7, r=0.2), random_spheres=False)
    info = a.shape(0)
    assert info.type == pt.TORUS and info.radius == 0.7 and info.tube_radius == 0.2
    o = O.Scene(torus_scene(R=0.7, r=0.2), random_spheres=False)
    assert list(info.direct) == list(o.shape(0).direct)


def test_host_build_matches_oracle_on_torus_frames():
    subprocess.run(["make", "-s", "-C", str(NATIVE)], check=True)
    H = C.CDLL(native_lib("libpath.so"))
    d = C.POINTER(C.c_double)
    H.h_scene_new.restype = C.c_void_p
    H.h_scene_new.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_uint64]
    H.h_scene_free.argtypes = [C.c_void_p]
    H.h_trace_pixels.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64,
                                 C.POINTER(C.c_uint32), C.c_size_t, d]
    text = (ROOT / "scenes" / "torus.json").read_text()
    raw = text.encode()
    h = H.h_scene_new(raw, len(raw), 1, 2)
    try:
        w, hh, spp, depth = 64, 36, 3, 8
        px = np.arange(w * hh, dtype=np.uint32)
        out = np.zeros((len(px), 3))
        H.h_trace_pixels(h, w, hh, spp, depth, 5, px.ctypes.data_as(C.POINTER(C.c_uint32)), len(px),
                         out.ctypes.data_as(d))
        ref = O.Scene(text, seed=2).render(w, hh, spp, depth, 5)
        assert np.array_equal(out, ref)
    finally:
        H.h_scene_free(h)
