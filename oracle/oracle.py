"""ctypes wrapper around the C restatement (oracle/pt_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.

Scene JSON is turned into oracle records with Python's own json module (the
reference's serde/typetag schema, src/world/json_models.rs:15-48), so the
oracle does not share the product's C++ JSON loader.
"""
from __future__ import annotations

import ctypes as C
import json
import math
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
# PT_ORACLE_LIB: another build of the same source (the sanitizer build, scripts/san.sh)
LIB_PATH = Path(os.environ["PT_ORACLE_LIB"]) if os.environ.get("PT_ORACLE_LIB") else HERE / "_build" / "liboracle.so"

SPHERE, RECT, CUBE, MARCH, TORUS = 0, 1, 2, 3, 4
FUNC_HEART, FUNC_SINE, FUNC_STAR, FUNC_DUPIN, FUNC_HUNTS, FUNC_CUSHION = 0, 1, 2, 3, 4, 5
FUNC_IDS = {"Heart": FUNC_HEART, "Sine": FUNC_SINE, "Star": FUNC_STAR, "DupinCyclide": FUNC_DUPIN,
            "HuntsSurface": FUNC_HUNTS, "Cushion": FUNC_CUSHION}
LAMBERTIAN, METAL, DIELECTRIC, DIFFUSE_LIGHT, EMPTY = 0, 1, 2, 3, 4


class ShapeIn(C.Structure):
    _fields_ = [("type", C.c_int32), ("material", C.c_int32), ("inverse_normal", C.c_int32),
                ("depth", C.c_int32), ("func", C.c_int32), ("pad0", C.c_int32),
                ("translate", C.c_double * 3), ("rotate", C.c_double * 3), ("scale", C.c_double * 3),
                ("x0", C.c_double), ("y0", C.c_double), ("x1", C.c_double), ("y1", C.c_double),
                ("step", C.c_double), ("fa", C.c_double), ("fb", C.c_double), ("fc", C.c_double),
                ("fd", C.c_double), ("fr", C.c_double), ("radius", C.c_double), ("tube_radius", C.c_double)]


class MaterialIn(C.Structure):
    _fields_ = [("type", C.c_int32), ("tex", C.c_int32), ("albedo", C.c_double * 3),
                ("fuzz", C.c_double), ("ior", C.c_double), ("emit", C.c_double * 3)]


TEX_SOLID, TEX_CHECKER, TEX_UVCHECKER, TEX_NOISE, TEX_IMAGE = 0, 1, 2, 3, 4


class TextureIn(C.Structure):
    _fields_ = [("type", C.c_int32), ("odd", C.c_int32), ("even", C.c_int32), ("aux", C.c_int32),
                ("c", C.c_double * 3)]


class ShapeOut(C.Structure):
    _fields_ = [("type", C.c_int32), ("material", C.c_int32), ("inverse_normal", C.c_int32),
                ("depth", C.c_int32), ("func", C.c_int32), ("pad0", C.c_int32),
                ("direct", C.c_double * 16), ("inverse", C.c_double * 16),
                ("x0", C.c_double), ("y0", C.c_double), ("x1", C.c_double), ("y1", C.c_double),
                ("step", C.c_double), ("fa", C.c_double), ("fb", C.c_double), ("fc", C.c_double),
                ("fd", C.c_double), ("fr", C.c_double), ("radius", C.c_double), ("tube_radius", C.c_double)]


class Hit(C.Structure):
    _fields_ = [("t", C.c_double), ("point", C.c_double * 3), ("normal", C.c_double * 3),
                ("front_face", C.c_int32), ("shape", C.c_int32), ("material", C.c_int32),
                ("pad0", C.c_int32), ("u", C.c_double), ("v", C.c_double)]


class Stats(C.Structure):
    _fields_ = [("shape_tests", C.c_uint64 * 4), ("march_steps", C.c_uint64),
                ("march_bounds", C.c_uint64), ("bounces", C.c_uint64),
                ("rejection_tries", C.c_uint64), ("samples", C.c_uint64),
                ("scatters", C.c_uint64 * 5)]

    def as_dict(self):
        return {"shape_tests": list(self.shape_tests), "march_steps": self.march_steps,
                "march_bounds": self.march_bounds, "bounces": self.bounces,
                "rejection_tries": self.rejection_tries, "samples": self.samples,
                "scatters": list(self.scatters)}


class Camera(C.Structure):
    _fields_ = [("position", C.c_double * 3), ("direction", C.c_double * 3), ("up", C.c_double * 3),
                ("right", C.c_double * 3), ("fov", C.c_double), ("focal_length", C.c_double)]


class Caster(C.Structure):
    _fields_ = [("position", C.c_double * 3), ("right", C.c_double * 3), ("up", C.c_double * 3),
                ("left_top", C.c_double * 3), ("pixel_resolution", C.c_double),
                ("width", C.c_uint32), ("height", C.c_uint32)]


def build():
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        build()
    L = C.CDLL(str(LIB_PATH))
    d3 = C.POINTER(C.c_double)
    L.or_scene_new.restype = C.c_void_p
    L.or_scene_new.argtypes = [C.POINTER(ShapeIn), C.c_int, C.POINTER(MaterialIn), C.c_int, C.c_int,
                               C.c_uint64]
    L.or_scene_free.argtypes = [C.c_void_p]
    L.or_scene_set_textures.argtypes = [C.c_void_p, C.POINTER(TextureIn), C.c_int, C.c_uint64]
    L.or_scene_add_image.restype = C.c_int
    L.or_scene_add_image.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint8)]
    L.or_perlin_tables.argtypes = [C.c_uint64, C.c_uint32, C.POINTER(C.c_int32), d3]
    L.or_perlin_turb.restype = C.c_double
    L.or_perlin_turb.argtypes = [C.c_uint64, C.c_uint32, d3]
    L.or_solve_quartic.argtypes = [C.c_double] * 5 + [d3, d3]
    L.or_texture_value.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_double, d3, d3]
    L.or_scene_num_shapes.argtypes = [C.c_void_p]
    L.or_scene_num_materials.argtypes = [C.c_void_p]
    L.or_scene_get_shape.argtypes = [C.c_void_p, C.c_int, C.POINTER(ShapeOut)]
    L.or_scene_get_material.argtypes = [C.c_void_p, C.c_int, C.POINTER(MaterialIn)]
    L.or_scene_use_bvh.argtypes = [C.c_void_p, C.c_int, C.c_uint64]
    L.or_transform_new.argtypes = [d3, d3, d3, d3, d3]
    L.or_rotate.argtypes = [d3, d3]
    L.or_mat_mul.argtypes = [d3, d3, d3]
    L.or_aabb_transform.argtypes = [d3, d3, d3, d3, d3]
    L.or_camera_new.argtypes = [d3, d3, d3, C.c_double, C.c_double, C.POINTER(Camera)]
    L.or_to_radians.restype = C.c_double
    L.or_to_radians.argtypes = [C.c_double]
    L.or_caster_new.argtypes = [C.POINTER(Camera), C.c_uint32, C.c_uint32, C.POINTER(Caster)]
    L.or_caster_ray.argtypes = [C.POINTER(Caster), C.c_double, C.c_double, d3, d3]
    L.or_mix64.restype = C.c_uint64
    L.or_mix64.argtypes = [C.c_uint64]
    L.or_sample_key.restype = C.c_uint64
    L.or_sample_key.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
    L.or_rng_next.restype = C.c_uint64
    L.or_rng_next.argtypes = [C.POINTER(C.c_uint64)]
    L.or_gen_f64.restype = C.c_double
    L.or_gen_f64.argtypes = [C.POINTER(C.c_uint64)]
    L.or_uniform_incl_scale.restype = C.c_double
    L.or_uniform_incl_scale.argtypes = [C.c_double, C.c_double]
    L.or_gen_range_incl.restype = C.c_double
    L.or_gen_range_incl.argtypes = [C.POINTER(C.c_uint64), C.c_double, C.c_double]
    L.or_shape_hit.argtypes = [C.c_void_p, C.c_int, d3, d3, C.c_double, C.c_double, C.POINTER(Hit)]
    L.or_closest_hit.argtypes = [C.c_void_p, d3, d3, C.c_double, C.c_double, C.POINTER(Hit),
                                 C.POINTER(Stats)]
    L.or_ray_color.argtypes = [C.c_void_p, d3, d3, C.c_uint32, C.POINTER(C.c_uint64), d3,
                               C.POINTER(Stats)]
    L.or_trace_pixel.argtypes = [C.c_void_p, C.POINTER(Caster), C.c_uint32, C.c_uint32, C.c_uint32,
                                 C.c_uint32, C.c_uint64, d3, C.POINTER(Stats)]
    L.or_render.argtypes = [C.c_void_p, C.POINTER(Caster), C.c_uint32, C.c_uint32, C.c_uint64,
                            C.POINTER(C.c_uint32), C.c_size_t, C.c_int, d3, C.POINTER(Stats)]
    _lib = L
    return L


def _d3(v):
    return (C.c_double * 3)(*[float(x) for x in v])


def vec3(v):
    """Vector3d accepts [x, y, z] or {"x","y","z"} (serde derive on Vector3d)."""
    if isinstance(v, dict):
        return [float(v["x"]), float(v["y"]), float(v["z"])]
    if len(v) != 3:
        raise ValueError("Vector3d needs 3 components")
    return [float(x) for x in v]


def read_ppm(path):
    """Binary PPM (P6, maxval 255) -> (width, height, RGBA8 bytes), alpha 255."""
    data = Path(path).read_bytes()
    fields, pos = [], 0
    while len(fields) < 4:
        while data[pos:pos + 1].isspace():
            pos += 1
        if data[pos:pos + 1] == b"#":
            pos = data.index(b"\n", pos) + 1
            continue
        end = pos
        while not data[end:end + 1].isspace():
            end += 1
        fields.append(data[pos:end])
        pos = end
    pos += 1  # the single whitespace byte after maxval
    if fields[0] != b"P6" or fields[3] != b"255":
        raise ValueError("not a P6/255 PPM: %s" % path)
    w, h = int(fields[1]), int(fields[2])
    rgb = np.frombuffer(data, np.uint8, w * h * 3, pos).reshape(-1, 3)
    rgba = np.concatenate([rgb, np.full((w * h, 1), 255, np.uint8)], axis=1)
    return w, h, rgba.tobytes()


class _Textures:
    """Texture trees (src/world/texture.rs) flattened in pre-order: a node,
    then its odd subtree, then its even one.  SolidColor at a material's root
    stays inline (tex = -1)."""

    def __init__(self, images):
        self.nodes, self.image_list, self.images = [], [], images or {}

    def node(self, tex):
        t = tex["type"]
        i = len(self.nodes)
        rec = {"type": None, "odd": -1, "even": -1, "aux": -1, "c": [0.0, 0.0, 0.0]}
        self.nodes.append(rec)
        if t == "SolidColor":
            rec["type"], rec["c"] = TEX_SOLID, vec3(tex["color"])
        elif t == "CheckerTexture":
            rec["type"], rec["c"] = TEX_CHECKER, vec3(tex["multipliers"])
            rec["odd"] = self.node(tex["odd"])
            rec["even"] = self.node(tex["even"])
        elif t == "UVChecker":
            m = tex["multipliers"]
            rec["type"], rec["c"] = TEX_UVCHECKER, [float(m[0]), float(m[1]), 0.0]
            rec["odd"] = self.node(tex["odd"])
            rec["even"] = self.node(tex["even"])
        elif t == "NoiseTexture":
            rec["type"], rec["c"] = TEX_NOISE, [float(tex["scale"]), 0.0, 0.0]
        elif t == "ImageTexture":
            fn = tex["image_filename"]
            rec["type"], rec["aux"] = TEX_IMAGE, len(self.image_list)
            self.image_list.append(self.images[fn] if fn in self.images else read_ppm(fn))
        else:
            raise NotImplementedError(t)
        return i

    def root(self, tex):
        """(tex index or -1, solid colour)"""
        if tex["type"] == "SolidColor":
            return -1, vec3(tex["color"])
        return self.node(tex), [0.0, 0.0, 0.0]


def records_from_json(text: str, images=None):
    """Scene JSON -> (shape records, material records, camera dict, textures).

    Follows SceneJson (json_models.rs:23-29): materials map (name -> typetag
    "type"), shapes in file order, camera with fov in degrees.  images maps
    ImageTexture file names to (width, height, RGBA8 bytes); other files are
    read as binary PPM.
    """
    js = json.loads(text)
    names = list(js["materials"].keys())
    index = {n: i for i, n in enumerate(names)}
    mats = (MaterialIn * max(1, len(names)))()
    tx = _Textures(images)
    for i, n in enumerate(names):
        m = js["materials"][n]
        t = m["type"]
        mats[i].tex = -1
        if t == "Lambertian":
            mats[i].type = LAMBERTIAN
            mats[i].tex, mats[i].albedo[:] = tx.root(m["albedo"])
        elif t == "Metal":
            mats[i].type = METAL
            mats[i].tex, mats[i].albedo[:] = tx.root(m["albedo"])
            mats[i].fuzz = float(m["fuzz"])
        elif t == "Dielectric":
            mats[i].type = DIELECTRIC
            mats[i].ior = float(m["index_of_refraction"])
        elif t == "DiffuseLight":
            mats[i].type = DIFFUSE_LIGHT
            mats[i].tex, mats[i].emit[:] = tx.root(m["emit"])
        elif t == "EmptyMaterial":
            mats[i].type = EMPTY
        else:
            raise NotImplementedError(t)
    shapes = js["shapes"]
    recs = (ShapeIn * max(1, len(shapes)))()
    for i, s in enumerate(shapes):
        r = recs[i]
        tr = s["transform"]
        r.translate[:] = vec3(tr["translate"])
        r.rotate[:] = vec3(tr["rotate"])
        r.scale[:] = vec3(tr["scale"])
        r.material = index[s["material"]]
        t = s["type"]
        if t == "Sphere":
            r.type = SPHERE
            r.inverse_normal = 1 if s.get("inverse_normal", False) else 0
        elif t == "Rectangle":
            r.type = RECT
            r.x0, r.y0, r.x1, r.y1 = (float(s[k]) for k in ("x0", "y0", "x1", "y1"))
        elif t == "Cube":
            r.type = CUBE
        elif t == "Torus":
            r.type = TORUS
            r.radius, r.tube_radius = float(s["radius"]), float(s["tube_radius"])
        elif t == "BruteForsableShape":
            fn = s["shape"]
            if fn["type"] not in FUNC_IDS:
                raise NotImplementedError(fn["type"])
            r.type = MARCH
            r.func = FUNC_IDS[fn["type"]]
            # BruteForceShapeJson fields (ray_marching.rs:559-670); the Heart has none
            for k, fld in (("a", "fa"), ("b", "fb"), ("c", "fc"), ("d", "fd"), ("sphere_radius", "fr")):
                if k in fn and r.func != FUNC_HEART:
                    setattr(r, fld, float(fn[k]))
            r.step = float(s["step"])
            r.depth = int(s.get("depth", 4))
        else:
            raise NotImplementedError(t)
    cam = js["camera"]
    camera = {"position": vec3(cam["position"]), "direction": vec3(cam["direction"]),
              "up": vec3(cam["up"]), "fov_deg": float(cam["fov"]),
              "focal_length": float(cam["focal_length"])}
    return recs, len(shapes), mats, len(names), camera, tx


class Scene:
    def __init__(self, json_text: str, random_spheres: bool = True, seed: int = 1, images=None):
        L = lib()
        recs, n, mats, nm, cam, tx = records_from_json(json_text, images)
        self._keep = (recs, mats)
        self.ptr = L.or_scene_new(recs, n, mats, nm, 1 if random_spheres else 0, seed)
        if tx.nodes:
            arr = (TextureIn * len(tx.nodes))()
            for i, r in enumerate(tx.nodes):
                arr[i].type, arr[i].odd, arr[i].even, arr[i].aux = r["type"], r["odd"], r["even"], r["aux"]
                arr[i].c[:] = r["c"]
            L.or_scene_set_textures(self.ptr, arr, len(tx.nodes), seed)
            for w, h, rgba in tx.image_list:
                buf = (C.c_uint8 * len(rgba)).from_buffer_copy(rgba)
                L.or_scene_add_image(self.ptr, w, h, buf)
        self.camera_json = cam
        self.n_json_shapes = n

    def __del__(self):
        if getattr(self, "ptr", None) and _lib is not None:
            _lib.or_scene_free(self.ptr)
            self.ptr = None

    def use_bvh(self, enable: bool = True, seed: int = 7):
        """Reference BvhNode traversal (CPU baseline); default is the linear scan."""
        lib().or_scene_use_bvh(self.ptr, 1 if enable else 0, seed)
        return self

    @property
    def num_shapes(self):
        return lib().or_scene_num_shapes(self.ptr)

    @property
    def num_materials(self):
        return lib().or_scene_num_materials(self.ptr)

    def shape(self, i) -> ShapeOut:
        out = ShapeOut()
        lib().or_scene_get_shape(self.ptr, i, C.byref(out))
        return out

    def material(self, i) -> MaterialIn:
        out = MaterialIn()
        lib().or_scene_get_material(self.ptr, i, C.byref(out))
        return out

    def camera(self) -> Camera:
        c = self.camera_json
        out = Camera()
        L = lib()
        L.or_camera_new(_d3(c["position"]), _d3(c["direction"]), _d3(c["up"]), c["focal_length"],
                        L.or_to_radians(c["fov_deg"]), C.byref(out))
        return out

    def caster(self, width, height, camera: Camera | None = None) -> Caster:
        k = Caster()
        lib().or_caster_new(C.byref(camera or self.camera()), width, height, C.byref(k))
        return k

    def closest_hit(self, o, d, min_t=0.001, max_t=math.inf):
        h = Hit()
        ok = lib().or_closest_hit(self.ptr, _d3(o), _d3(d), min_t, max_t, C.byref(h), None)
        return h if ok else None

    def shape_hit(self, i, o, d, min_t=0.001, max_t=math.inf):
        h = Hit()
        ok = lib().or_shape_hit(self.ptr, i, _d3(o), _d3(d), min_t, max_t, C.byref(h))
        return h if ok else None

    def texture_value(self, tex, u, v, p):
        out = (C.c_double * 3)()
        lib().or_texture_value(self.ptr, tex, u, v, _d3(p), out)
        return np.array(out[:])

    def ray_color(self, o, d, depth, rng_state: int):
        st = C.c_uint64(rng_state)
        out = (C.c_double * 3)()
        lib().or_ray_color(self.ptr, _d3(o), _d3(d), depth, C.byref(st), out, None)
        return np.array(out[:]), st.value

    def render(self, width, height, spp, depth, seed, pixels=None, threads=None, camera=None,
               stats=False):
        """Per-pixel means (npix, 3) for the given pixel indices (default: the whole frame)."""
        k = self.caster(width, height, camera)
        if pixels is None:
            pixels = np.arange(width * height, dtype=np.uint32)
        pixels = np.ascontiguousarray(pixels, dtype=np.uint32)
        out = np.zeros((len(pixels), 3), dtype=np.float64)
        st = Stats() if stats else None
        threads = threads or min(16, os.cpu_count() or 1)
        lib().or_render(self.ptr, C.byref(k), spp, depth, seed,
                        pixels.ctypes.data_as(C.POINTER(C.c_uint32)), len(pixels), threads,
                        out.ctypes.data_as(C.POINTER(C.c_double)),
                        C.byref(st) if st is not None else None)
        return (out, st.as_dict()) if stats else out
