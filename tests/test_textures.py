"""Textures (src/world/texture.rs) and Perlin noise (src/algebra/noise.rs) on
the CPU: the oracle's restatement against independent pure-Python
restatements of the reference formulas, the product loader (ImageTexture via
the built-in PPM reader and via a host loader), and the product's device code
compiled for the host (tests/native) against the oracle, bit for bit.

Parity status: no reference test pins any texture value, and the Perlin tables
come from the unseedable thread_rng (noise.rs:25), so the noise realisation is
the RNG spec's, distributionally the reference's."""
import ctypes as C
import math
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle as O
from conftest import native_lib

ROOT = Path(__file__).resolve().parent.parent
NATIVE = ROOT / "tests" / "native"


@pytest.fixture(autouse=True)
def _repo_cwd(monkeypatch):
    monkeypatch.chdir(ROOT)  # the scenes name their image as ./scenes/textures/grid.ppm


@pytest.fixture(scope="module")
def textured_text():
    return (ROOT / "scenes" / "textured.json").read_text()


@pytest.fixture(scope="module")
def noise_text():
    return (ROOT / "scenes" / "noise.json").read_text()


def perlin_tables(seed, k):
    perm, rv = (C.c_int32 * 768)(), (C.c_double * 768)()
    O.lib().or_perlin_tables(seed, k, perm, rv)
    return np.array(perm[:]).reshape(3, 256), np.array(rv[:]).reshape(256, 3)


def py_noise(perm, rv, p):
    """Perlin::noise, noise.rs:44-74, in plain Python floats."""
    x, y, z = (int(math.floor(c)) for c in p)
    u, v, w = (c - math.floor(c) for c in p)
    u2, v2, w2 = u * u * (3.0 - 2.0 * u), v * v * (3.0 - 2.0 * v), w * w * (3.0 - 2.0 * w)
    s = 0.0
    for a in (0, 1):
        for b in (0, 1):
            for c in (0, 1):
                g = rv[perm[0][(a + x) & 255] ^ perm[1][(b + y) & 255] ^ perm[2][(c + z) & 255]]
                s = s + ((a * u2 + (1 - a) * (1.0 - u2)) * (b * v2 + (1 - b) * (1.0 - v2))
                         * (c * w2 + (1 - c) * (1.0 - w2)) * (g[0] * (u - a) + g[1] * (v - b) + g[2] * (w - c)))
    return s


def test_perlin_tables_are_the_reference_shape():
    perm, rv = perlin_tables(1, 0)
    for a in range(3):
        assert sorted(perm[a]) == list(range(256))  # shuffles of 0..256
    assert not np.array_equal(perm[0], perm[1])  # three independent shuffles
    assert np.all(np.abs(rv) <= 1.0)  # Vector3d::random(-1, 1), not normalised
    assert np.std(np.linalg.norm(rv, axis=1)) > 0.1
    p2, _ = perlin_tables(1, 1)
    assert not np.array_equal(perm, p2)  # a stream per NoiseTexture
    p3, _ = perlin_tables(2, 0)
    assert not np.array_equal(perm, p3)  # and per scene seed


def test_turb_matches_python_restatement():
    perm, rv = perlin_tables(7, 0)
    rng = np.random.default_rng(0)
    for p in rng.uniform(-300, 300, size=(500, 3)):
        n = py_noise(perm, rv, p)
        acc, wt = 0.0, 1.0
        for _ in range(7):  # turb's scan: weight * noise(p) of the unscaled p every octave
            acc = acc + wt * n
            wt *= 0.5
        assert O.lib().or_perlin_turb(7, 0, (C.c_double * 3)(*p)) == abs(acc)


def test_noise_lattice_points_are_zero():
    perm, rv = perlin_tables(3, 0)
    for p in [(0.0, 0.0, 0.0), (5.0, -2.0, 17.0), (-255.0, 256.0, 1.0)]:
        assert py_noise(perm, rv, p) == 0.0  # every corner dot product with (u, v, w) = 0


def scene_with_material(mat, shape=None):
    shape = shape or {"type": "Sphere", "name": "S", "transform": {"translate": [0, 0, 0], "rotate": [0, 0, 0],
                                                                  "scale": [1, 1, 1]}, "material": "M"}
    import json
    return json.dumps({"camera": {"position": [0, 0, -5], "direction": [0, 0, 1], "up": [0, 1, 0], "fov": 40,
                                  "focal_length": 1},
                       "shapes": [shape], "materials": {"M": mat}, "background": [0, 0, 0]})


def test_checker_and_uvchecker_values():
    odd, even = [0.1, 0.2, 0.8], [0.9, 0.2, 0.1]
    chk = {"type": "CheckerTexture", "scale": 4.0, "odd": {"type": "SolidColor", "color": odd},
           "even": {"type": "SolidColor", "color": even}, "multipliers": {"x": 5, "y": 5, "z": 5}}
    sc = O.Scene(scene_with_material({"type": "Metal", "albedo": chk, "fuzz": 0.0}), random_spheres=False)
    assert sc.material(0).tex == 0
    rng = np.random.default_rng(1)
    for p in rng.uniform(-3, 3, size=(300, 3)):
        sines = math.sin(5 * p[0]) * math.sin(5 * p[1]) * math.sin(5 * p[2])  # texture.rs:42-45
        want = odd if sines < 0.0 else even
        assert list(sc.texture_value(0, 0.3, 0.7, p)) == want
    uvc = {"type": "UVChecker", "odd": {"type": "SolidColor", "color": odd},
           "even": {"type": "SolidColor", "color": even}, "multipliers": [40.0, 30.0]}
    sc = O.Scene(scene_with_material({"type": "Lambertian", "albedo": uvc}), random_spheres=False)
    for u, v in rng.uniform(0, 1, size=(300, 2)):
        sines = math.sin(v * 40.0 * math.pi) * math.sin(u * 30.0 * math.pi)  # texture.rs:78-79
        want = odd if sines < 0.0 else even
        assert list(sc.texture_value(0, u, v, [0, 0, 0])) == want


def test_image_texture_texels_and_clamp():
    w, h = 5, 3
    rgba = bytes(c for y in range(h) for x in range(w) for c in (x * 40, y * 80, 7, 255))
    img = {"type": "ImageTexture", "image_filename": "mem.png"}
    sc = O.Scene(scene_with_material({"type": "Lambertian", "albedo": img}), random_spheres=False,
                 images={"mem.png": (w, h, rgba)})
    cs = 1.0 / 255.0
    for u, v in [(0.0, 1.0), (0.5, 0.5), (0.99, 0.01), (0.21, 0.66), (-3.0, 7.0)]:
        uc, vc = min(max(u, 0.0), 1.0), 1.0 - min(max(v, 0.0), 1.0)  # texture.rs:98-102
        x, y = min(int(uc * w), w - 1), min(int(vc * h), h - 1)
        want = [x * 40 * cs, y * 80 * cs, 7 * cs]
        assert list(sc.texture_value(0, u, v, [0, 0, 0])) == want


def test_ppm_reader_and_loader_agree(pt):
    text = scene_with_material({"type": "Metal", "albedo": {"type": "ImageTexture",
                                                           "image_filename": "./scenes/textures/grid.ppm"},
                                "fuzz": 1.0})
    a = pt.Scene.from_json(text, random_spheres=False)
    assert a.material(0).texture == 0
    w, h, rgba = O.read_ppm(ROOT / "scenes" / "textures" / "grid.ppm")
    assert (w, h) == (64, 32) and len(rgba) == w * h * 4
    b = pt.Scene.from_json(text, random_spheres=False, images={"./scenes/textures/grid.ppm": (w, h, rgba)})
    assert b.material(0).texture == 0
    missing = text.replace("grid.ppm", "nope.ppm")
    with pytest.raises(pt.PtError) as e:
        pt.Scene.from_json(missing, random_spheres=False)
    assert e.value.code == pt.PT_ERR_UNSUPPORTED and "nope.ppm" in str(e.value)
    with pytest.raises(pt.PtError) as e:
        pt.Scene.from_json(missing, random_spheres=False, images={"./scenes/textures/nope.ppm": (2, 2, b"x")})
    assert e.value.code == pt.PT_ERR_INVALID  # a loader's malformed image is an error, not a fallback


def test_loader_rejects_bad_textures(pt):
    bad = scene_with_material({"type": "Lambertian", "albedo": {"type": "Marble"}})
    with pytest.raises(pt.PtError) as e:
        pt.Scene.from_json(bad)
    assert e.value.code == pt.PT_ERR_PARSE
    bad = scene_with_material({"type": "Lambertian", "albedo": {"type": "UVChecker", "odd": {"type": "SolidColor",
                               "color": [1, 1, 1]}, "even": {"type": "SolidColor", "color": [0, 0, 0]},
                               "multipliers": [1.0, 2.0, 3.0]}})
    with pytest.raises(pt.PtError):
        pt.Scene.from_json(bad)


@pytest.fixture(scope="module")
def H():
    subprocess.run(["make", "-s", "-C", str(NATIVE)], check=True)
    L = C.CDLL(native_lib("libpath.so"))
    d = C.POINTER(C.c_double)
    L.h_scene_new.restype = C.c_void_p
    L.h_scene_new.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_uint64]
    L.h_scene_free.argtypes = [C.c_void_p]
    L.h_trace_pixels.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64,
                                 C.POINTER(C.c_uint32), C.c_size_t, d]
    L.h_ray_color.argtypes = [C.c_void_p, d, C.POINTER(C.c_uint64), C.c_uint32, d]
    return L


@pytest.mark.parametrize("name,seed,depth", [("textured.json", 1, 8), ("noise.json", 2, 8), ("textured.json", 5, 50)])
def test_host_build_matches_oracle_on_textured_frames(H, name, seed, depth):
    text = (ROOT / "scenes" / name).read_text()
    raw = text.encode()
    h = H.h_scene_new(raw, len(raw), 1, seed)
    assert h
    try:
        w, hh, spp = 48, 27, 3
        px = np.arange(w * hh, dtype=np.uint32)
        out = np.zeros((len(px), 3))
        H.h_trace_pixels(h, w, hh, spp, depth, 4, px.ctypes.data_as(C.POINTER(C.c_uint32)), len(px),
                         out.ctypes.data_as(C.POINTER(C.c_double)))
        ref = O.Scene(text, seed=seed).render(w, hh, spp, depth, 4)
        assert np.array_equal(out, ref)
        assert out.mean() > 0.05
    finally:
        H.h_scene_free(h)
