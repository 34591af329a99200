"""rs_pathtracing_amd — MI355X-native sample loop behind the reference's interfaces.

Python mirror of the reference's host API over the C-ABI in
include/rs_pathtracing.h (librs_pathtracing_amd.so, built in-tree):

    Scene.from_json(data)                       src/world/mod.rs:46-49
    Scene.camera()                              src/world/mod.rs:193-197
    Camera.new(position, direction, up, focal_length, fov)   src/camera/mod.rs:71-88
    ImageParams(width, height)                  src/camera/ray_caster.rs:10-14
    Renderer: start_rendering / render_step / stop_rendering   src/renderer/mod.rs:47-56
    HipRenderer(scene, device, depth)           ThreadPoolRenderer::new, step_by_step.rs:37
    ray_color / trace_pixel_samples             src/renderer/mod.rs:23-45, 151-155
    closest_hit                                 src/world/mod.rs:42-44

The colour buffer is the reference's Vec<Vector3d>: a (w*h, 3) float64 array,
row-major, index x + y*w.  There is no CPU fallback: if the library or a GPU
is missing, construction fails loudly.
"""
from __future__ import annotations

import abc
import ctypes as C
import hashlib
import os
import struct
from dataclasses import dataclass
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "librs_pathtracing_amd.so"

PT_OK = 0
PT_ERR_INVALID, PT_ERR_PARSE, PT_ERR_UNSUPPORTED, PT_ERR_HIP, PT_ERR_STATE, PT_ERR_IO = -1, -2, -3, -4, -5, -6
SPHERE, RECTANGLE, CUBE, MARCH, TORUS = 0, 1, 2, 3, 4
LAMBERTIAN, METAL, DIELECTRIC, DIFFUSE_LIGHT, EMPTY = 0, 1, 2, 3, 4
TILE = 16

# every symbol include/rs_pathtracing.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "pt_scene_create_from_json", "pt_scene_destroy", "pt_scene_camera", "pt_scene_num_shapes",
    "pt_scene_get_shape", "pt_scene_num_materials", "pt_scene_get_material", "pt_camera_new",
    "pt_renderer_create", "pt_renderer_create_multi", "pt_renderer_num_devices", "pt_renderer_destroy",
    "pt_renderer_set_option", "pt_renderer_get_option", "pt_option_name",
    "pt_render_start", "pt_render_step", "pt_render_step_rgba8", "pt_render_stop",
    "pt_render_device", "pt_render_frame_device", "pt_shard_tiles", "pt_unshard_device", "pt_closest_hit",
    "pt_ray_color", "pt_trace_pixel_samples", "pt_count_work", "pt_profile_phases", "pt_march_jobs", "pt_march_guard_drops", "pt_render_stop_stats", "pt_wave_diag",
    "pt_kernel_timing", "pt_encode_rgba8", "pt_encode_rgba8_device", "pt_write_png", "pt_write_ppm",
    "pt_sample_key", "pt_last_error", "pt_version", "pt_abi_version", "pt_abi_layout", "pt_renderer_peer_access",
    "pt_render_device_samples", "pt_checkpoint_save", "pt_checkpoint_load",
]
ABI_VERSION = 4  # PT_ABI_VERSION this binding is written for


class PtError(RuntimeError):
    """A non-zero status from the C-ABI (the reference panics or returns serde_json::Error)."""

    def __init__(self, code: int, msg: str):
        super().__init__("%s (status %d)" % (msg, code))
        self.code = code


# pt_image_loader: (user, filename, *width, *height, *rgba8) -> status
ImageLoader = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_char_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                          C.POINTER(C.POINTER(C.c_uint8)))


class SceneOpts(C.Structure):
    _fields_ = [("random_spheres", C.c_uint32), ("struct_size", C.c_uint32), ("seed", C.c_uint64),
                ("load_image", ImageLoader), ("image_user", C.c_void_p)]


class CameraStruct(C.Structure):
    _fields_ = [("position", C.c_double * 3), ("direction", C.c_double * 3), ("up", C.c_double * 3),
                ("right", C.c_double * 3), ("fov", C.c_double), ("focal_length", C.c_double)]


class ShapeInfo(C.Structure):
    _fields_ = [("type", C.c_int32), ("material", C.c_int32), ("inverse_normal", C.c_int32),
                ("depth", C.c_int32), ("func", C.c_int32), ("pad0", C.c_int32),
                ("direct", C.c_double * 16), ("inverse", C.c_double * 16),
                ("x0", C.c_double), ("y0", C.c_double), ("x1", C.c_double), ("y1", C.c_double),
                ("step", C.c_double), ("a", C.c_double), ("b", C.c_double), ("c", C.c_double), ("d", C.c_double),
                ("sphere_radius", C.c_double), ("radius", C.c_double), ("tube_radius", C.c_double)]


class MaterialInfo(C.Structure):
    _fields_ = [("type", C.c_int32), ("texture", C.c_int32), ("albedo", C.c_double * 3),
                ("fuzz", C.c_double), ("ior", C.c_double), ("emit", C.c_double * 3)]


class HitStruct(C.Structure):
    _fields_ = [("t", C.c_double), ("point", C.c_double * 3), ("normal", C.c_double * 3),
                ("front_face", C.c_int32), ("shape", C.c_int32), ("material", C.c_int32),
                ("pad0", C.c_int32)]


class CheckpointStruct(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("samples_number", C.c_uint32),
                ("samples_done", C.c_uint32), ("rank", C.c_uint32), ("world", C.c_uint32), ("depth", C.c_uint32),
                ("reserved", C.c_uint32), ("seed", C.c_uint64), ("scene_key", C.c_uint64), ("count", C.c_uint64)]


HIT_DTYPE = np.dtype([("t", "<f8"), ("point", "<f8", 3), ("normal", "<f8", 3), ("front_face", "<i4"),
                      ("shape", "<i4"), ("material", "<i4"), ("pad0", "<i4")])
assert HIT_DTYPE.itemsize == C.sizeof(HitStruct)

_lib = None


def lib():
    """Load the in-tree HIP library; fails loudly if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ImportError("%s is missing: build it with `make -C rs-pathtracing_amd` or "
                          "`python -c 'import __graft_entry__ as g; g.build()'` (there is no CPU fallback)"
                          % LIB_PATH)
    try:
        # One HIP runtime per process: torch bundles its own libamdhip64.so.7.
        # Loading it first lets our NEEDED libamdhip64.so.7 resolve to the same
        # copy (same SONAME), so torch tensors / streams and our kernels share
        # one runtime instead of two runtimes fighting over the device.
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(os.environ.get("PT_AMD_LIB") or str(LIB_PATH))  # PT_AMD_LIB: an alternate build (tuning)
    vp, d = C.c_void_p, C.POINTER(C.c_double)
    u32, u64, sz = C.c_uint32, C.c_uint64, C.c_size_t
    sig = {
        "pt_scene_create_from_json": (C.c_int, [C.c_char_p, sz, C.POINTER(SceneOpts), C.POINTER(vp)]),
        "pt_scene_destroy": (None, [vp]),
        "pt_scene_camera": (C.c_int, [vp, C.POINTER(CameraStruct)]),
        "pt_scene_num_shapes": (C.c_int, [vp]),
        "pt_scene_get_shape": (C.c_int, [vp, C.c_int, C.POINTER(ShapeInfo)]),
        "pt_scene_num_materials": (C.c_int, [vp]),
        "pt_scene_get_material": (C.c_int, [vp, C.c_int, C.POINTER(MaterialInfo)]),
        "pt_camera_new": (C.c_int, [d, d, d, C.c_double, C.c_double, C.POINTER(CameraStruct)]),
        "pt_renderer_create": (C.c_int, [vp, C.c_int, u32, C.POINTER(vp)]),
        "pt_renderer_create_multi": (C.c_int, [vp, C.POINTER(C.c_int), C.c_int, u32, C.POINTER(vp)]),
        "pt_renderer_num_devices": (C.c_int, [vp]),
        "pt_renderer_set_option": (C.c_int, [vp, C.c_char_p, C.c_int64]),
        "pt_renderer_get_option": (C.c_int, [vp, C.c_char_p, C.POINTER(C.c_int64)]),
        "pt_option_name": (C.c_char_p, [C.c_int]),
        "pt_renderer_destroy": (None, [vp]),
        "pt_render_start": (C.c_int, [vp, C.POINTER(CameraStruct), u32, u32, u32, u64]),
        "pt_render_step": (C.c_int, [vp, d, C.c_int]),
        "pt_render_step_rgba8": (C.c_int, [vp, d, C.POINTER(C.c_uint8), C.c_int]),
        "pt_render_stop": (C.c_int, [vp]),
        "pt_render_device": (C.c_int, [vp, C.POINTER(CameraStruct), u32, u32, u32, u64, u32, u32, vp, vp]),
        "pt_render_frame_device": (C.c_int, [vp, C.POINTER(CameraStruct), u32, u32, u32, u64, vp, vp]),
        "pt_render_device_samples": (C.c_int, [vp, C.POINTER(CameraStruct), u32, u32, u32, u64, u32, u32, u32, u32,
                                               vp, vp]),
        "pt_checkpoint_save": (C.c_int, [C.c_char_p, C.POINTER(CheckpointStruct), d]),
        "pt_checkpoint_load": (C.c_int, [C.c_char_p, C.POINTER(CheckpointStruct), d, u64]),
        "pt_shard_tiles": (u32, [u32, u32, u32, u32]),
        "pt_unshard_device": (C.c_int, [C.c_int, vp, u32, u32, u32, vp, vp]),
        "pt_closest_hit": (C.c_int, [vp, d, sz, C.c_double, C.c_double, vp]),
        "pt_ray_color": (C.c_int, [vp, d, C.POINTER(u64), sz, u32, d]),
        "pt_trace_pixel_samples": (C.c_int, [vp, C.POINTER(CameraStruct), u32, u32, u32, u64,
                                             C.POINTER(u32), sz, d]),
        "pt_count_work": (C.c_int, [vp, C.POINTER(CameraStruct), u32, u32, u32, u64, C.POINTER(u32), sz,
                                    C.POINTER(u64)]),
        "pt_march_jobs": (C.c_int, [vp, C.POINTER(C.c_double), sz, C.POINTER(C.c_double), C.POINTER(C.c_int32),
                                    C.POINTER(C.c_uint32)]),
        "pt_kernel_timing": (C.c_int, [vp, C.c_int, C.POINTER(C.c_double), C.POINTER(u32), sz]),
        "pt_march_guard_drops": (C.c_int, [vp, C.POINTER(u64)]),
        "pt_render_stop_stats": (C.c_int, [vp, C.POINTER(u64), C.POINTER(u64)]),
        "pt_wave_diag": (C.c_int, [vp, C.c_int, C.POINTER(u64), sz]),
        "pt_profile_phases": (C.c_int, [vp, C.POINTER(CameraStruct), u32, u32, u32, u64, C.POINTER(u64)]),
        "pt_encode_rgba8": (C.c_int, [d, sz, C.POINTER(C.c_uint8)]),
        "pt_encode_rgba8_device": (C.c_int, [C.c_int, vp, sz, vp, vp]),
        "pt_write_png": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint8), u32, u32]),
        "pt_write_ppm": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint8), u32, u32]),
        "pt_sample_key": (u64, [u64, u64, u64]),
        "pt_last_error": (C.c_char_p, []),
        "pt_version": (C.c_char_p, []),
        "pt_abi_version": (u32, []),
        "pt_abi_layout": (C.c_int, [C.c_int, C.POINTER(u32), sz]),
        "pt_renderer_peer_access": (C.c_int, [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("PT_AMD_LIB") and not hasattr(L, name):
            continue  # an older alternate build (tuning comparisons)
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if not os.environ.get("PT_AMD_LIB") and L.pt_abi_version() != ABI_VERSION:
        raise ImportError("%s has ABI version %d; this binding is written for %d (rebuild the library)"
                          % (LIB_PATH, L.pt_abi_version(), ABI_VERSION))
    _lib = L
    return L


def _check(status: int) -> int:
    if status < 0:
        raise PtError(status, lib().pt_last_error().decode("utf-8", "replace"))
    return status


def _d3(v):
    return (C.c_double * 3)(*[float(x) for x in v])


def _dptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_double))


@dataclass
class ImageParams:
    """src/camera/ray_caster.rs:10-14"""
    width: int
    height: int


class Camera:
    """Camera (src/camera/mod.rs:36-46); fov in radians as Camera::new takes it."""

    def __init__(self, c: CameraStruct):
        self._c = c

    @classmethod
    def new(cls, position, direction, up, focal_length: float, fov: float) -> "Camera":
        c = CameraStruct()
        _check(lib().pt_camera_new(_d3(position), _d3(direction), _d3(up), float(focal_length), float(fov),
                                   C.byref(c)))
        return cls(c)

    position = property(lambda s: np.array(s._c.position[:]))
    direction = property(lambda s: np.array(s._c.direction[:]))
    up = property(lambda s: np.array(s._c.up[:]))
    right = property(lambda s: np.array(s._c.right[:]))
    fov = property(lambda s: s._c.fov)
    focal_length = property(lambda s: s._c.focal_length)


class Scene:
    """Realized scene: JSON shapes in file order, then add_random_spheres."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def from_json(cls, data: str | bytes, random_spheres: bool = True, seed: int = 1,
                  images: dict | None = None) -> "Scene":
        """images: ImageTexture file name -> (width, height, RGBA8 bytes), the
        decoded pixels the reference gets from image::open(..).into_rgba8()
        (src/world/texture.rs:119-130).  Names not in it are read by the
        library's built-in binary-PPM reader."""
        raw = data.encode("utf-8") if isinstance(data, str) else bytes(data)
        opts = SceneOpts(1 if random_spheres else 0, C.sizeof(SceneOpts), seed)
        keep = []
        if images:
            def load(_user, name, w, h, px):
                img = images.get(name.decode("utf-8"))
                if img is None:
                    return PT_ERR_UNSUPPORTED  # declined: the built-in PPM reader takes it
                iw, ih, rgba = img
                if len(rgba) != iw * ih * 4:
                    return PT_ERR_INVALID
                buf = (C.c_uint8 * len(rgba)).from_buffer_copy(rgba)
                keep.append(buf)
                w[0], h[0] = iw, ih
                px[0] = C.cast(buf, C.POINTER(C.c_uint8))
                return PT_OK
            opts.load_image = ImageLoader(load)
        h = C.c_void_p()
        _check(lib().pt_scene_create_from_json(raw, len(raw), C.byref(opts), C.byref(h)))
        return cls(h)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.pt_scene_destroy(h)
            self._h = None

    def camera(self) -> Camera:
        c = CameraStruct()
        _check(lib().pt_scene_camera(self._h, C.byref(c)))
        return Camera(c)

    @property
    def num_shapes(self) -> int:
        return _check(lib().pt_scene_num_shapes(self._h))

    @property
    def num_materials(self) -> int:
        return _check(lib().pt_scene_num_materials(self._h))

    def shape(self, i: int) -> ShapeInfo:
        s = ShapeInfo()
        _check(lib().pt_scene_get_shape(self._h, i, C.byref(s)))
        return s

    def material(self, i: int) -> MaterialInfo:
        m = MaterialInfo()
        _check(lib().pt_scene_get_material(self._h, i, C.byref(m)))
        return m


class Renderer(abc.ABC):
    """trait Renderer (src/renderer/mod.rs:47-56)."""

    @abc.abstractmethod
    def start_rendering(self, camera: Camera, img_params: ImageParams, samples_number: int): ...

    @abc.abstractmethod
    def render_step(self, buffer: np.ndarray) -> bool: ...

    @abc.abstractmethod
    def stop_rendering(self): ...


class HipRenderer(Renderer):
    """The MI355X renderer: ThreadPoolRenderer::new(scene, thread_number, depth)
    with HIP devices in place of the thread pool.  `device` is one HIP ordinal
    (-1 = current); `devices` (a list of ordinals, may repeat) spreads the
    frame's tiles over several (pt_renderer_create_multi).  `seed` keys the
    per-(pixel, sample) RNG; render_step(blocking=False) is step_by_step's
    non-blocking drain, blocking=True is thread_pool_new's."""

    def __init__(self, scene: Scene, device: int = -1, depth: int = 50, seed: int = 1, devices=None):
        self.scene = scene  # must outlive the renderer
        self.depth = int(depth)
        self.seed = int(seed)
        h = C.c_void_p()
        if devices is None:
            _check(lib().pt_renderer_create(scene._h, int(device), self.depth, C.byref(h)))
        else:
            dv = (C.c_int * len(devices))(*[int(x) for x in devices])
            _check(lib().pt_renderer_create_multi(scene._h, dv, len(devices), self.depth, C.byref(h)))
        self._h = h
        self._shape = None

    @property
    def num_devices(self) -> int:
        return _check(lib().pt_renderer_num_devices(self._h))

    def peer_access(self) -> tuple:
        """(distinct device pairs with devices[0], pairs with peer access enabled both ways)."""
        p, e = C.c_int(), C.c_int()
        _check(lib().pt_renderer_peer_access(self._h, C.byref(p), C.byref(e)))
        return p.value, e.value

    def set_option(self, name: str, value: int):
        """A tuning knob (pt_renderer_set_option): "engine" 0 auto / 1 megakernel / 2 wavefront, "wf_slots", ..."""
        _check(lib().pt_renderer_set_option(self._h, name.encode(), int(value)))

    def get_option(self, name: str) -> int:
        v = C.c_int64()
        _check(lib().pt_renderer_get_option(self._h, name.encode(), C.byref(v)))
        return v.value

    def options(self) -> dict:
        """Every tuning knob and its current value."""
        return {n: self.get_option(n) for n in option_names()}

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.pt_renderer_destroy(h)
            self._h = None

    def start_rendering(self, camera: Camera, img_params: ImageParams, samples_number: int, seed=None):
        s = self.seed if seed is None else int(seed)
        _check(lib().pt_render_start(self._h, C.byref(camera._c), img_params.width, img_params.height,
                                     int(samples_number), s))
        self._shape = (img_params.width * img_params.height, 3)

    def render_step(self, buffer: np.ndarray, blocking: bool = False) -> bool:
        if self._shape is None:
            raise PtError(PT_ERR_STATE, "render_step before start_rendering")
        if buffer.shape != self._shape or buffer.dtype != np.float64 or not buffer.flags.c_contiguous:
            raise ValueError("buffer must be a C-contiguous float64 array of shape %r" % (self._shape,))
        return _check(lib().pt_render_step(self._h, _dptr(buffer), 1 if blocking else 0)) == 1

    def render_step_rgba8(self, rgba: np.ndarray, buffer: np.ndarray | None = None, blocking: bool = False) -> bool:
        """render_step with the GPU's display encode of every finished band in
        rgba ((w*h, 4) uint8); buffer (optional) gets the linear rows too."""
        if self._shape is None:
            raise PtError(PT_ERR_STATE, "render_step before start_rendering")
        if rgba.shape != (self._shape[0], 4) or rgba.dtype != np.uint8 or not rgba.flags.c_contiguous:
            raise ValueError("rgba must be a C-contiguous uint8 array of shape (%d, 4)" % self._shape[0])
        bp = None
        if buffer is not None:
            if buffer.shape != self._shape or buffer.dtype != np.float64 or not buffer.flags.c_contiguous:
                raise ValueError("buffer must be a C-contiguous float64 array of shape %r" % (self._shape,))
            bp = _dptr(buffer)
        return _check(lib().pt_render_step_rgba8(self._h, bp, rgba.ctypes.data_as(C.POINTER(C.c_uint8)),
                                                 1 if blocking else 0)) == 1

    def stop_rendering(self):
        _check(lib().pt_render_stop(self._h))

    def render(self, camera: Camera, img_params: ImageParams, samples_number: int, seed=None) -> np.ndarray:
        buf = np.zeros((img_params.width * img_params.height, 3), dtype=np.float64)
        self.start_rendering(camera, img_params, samples_number, seed)
        self.render_step(buf, blocking=True)
        return buf

    def render_device(self, camera: Camera, width: int, height: int, spp: int, seed: int, rank: int,
                      world: int, out_ptr: int, stream_ptr: int = 0):
        """Render this rank's tiles into device memory at out_ptr on the HIP stream stream_ptr
        (0 = the null stream; see pt_render_device)."""
        _check(lib().pt_render_device(self._h, C.byref(camera._c), width, height, spp, seed, rank, world,
                                      C.c_void_p(out_ptr), C.c_void_p(stream_ptr)))

    def render_device_samples(self, camera: Camera, width: int, height: int, spp: int, seed: int, rank: int,
                              world: int, s_begin: int, s_end: int, out_ptr: int, stream_ptr: int = 0):
        """Samples [s_begin, s_end) of the frame render_device renders, added to the running sums at out_ptr
        (read when s_begin > 0; sums stored, or the means once s_end == spp; see pt_render_device_samples)."""
        _check(lib().pt_render_device_samples(self._h, C.byref(camera._c), width, height, spp, seed, rank, world,
                                              int(s_begin), int(s_end), C.c_void_p(out_ptr),
                                              C.c_void_p(stream_ptr)))

    def render_frame_device(self, camera: Camera, width: int, height: int, spp: int, seed: int, frame_ptr: int,
                            stream_ptr: int = 0):
        """The whole frame over all of the renderer's devices into device memory at frame_ptr (first
        device), ordered after stream_ptr's queued work (pt_render_frame_device)."""
        _check(lib().pt_render_frame_device(self._h, C.byref(camera._c), width, height, spp, seed,
                                            C.c_void_p(frame_ptr), C.c_void_p(stream_ptr)))

    # ---- probes --------------------------------------------------------
    def closest_hit(self, rays: np.ndarray, min_t: float = 0.001, max_t: float = float("inf")) -> np.ndarray:
        rays = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 6)
        out = np.zeros(len(rays), dtype=HIT_DTYPE)
        _check(lib().pt_closest_hit(self._h, _dptr(rays), len(rays), min_t, max_t, out.ctypes.data))
        return out

    def ray_color(self, rays: np.ndarray, rng_states: np.ndarray, depth: int | None = None) -> np.ndarray:
        rays = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 6)
        states = np.ascontiguousarray(rng_states, dtype=np.uint64)
        out = np.zeros((len(rays), 3), dtype=np.float64)
        _check(lib().pt_ray_color(self._h, _dptr(rays), states.ctypes.data_as(C.POINTER(C.c_uint64)),
                                  len(rays), self.depth if depth is None else int(depth), _dptr(out)))
        rng_states[...] = states
        return out

    def trace_pixel_samples(self, camera: Camera, img_params: ImageParams, samples_number: int,
                            pixels: np.ndarray, seed=None) -> np.ndarray:
        pixels = np.ascontiguousarray(pixels, dtype=np.uint32)
        out = np.zeros((len(pixels), 3), dtype=np.float64)
        s = self.seed if seed is None else int(seed)
        _check(lib().pt_trace_pixel_samples(self._h, C.byref(camera._c), img_params.width, img_params.height,
                                            int(samples_number), s,
                                            pixels.ctypes.data_as(C.POINTER(C.c_uint32)), len(pixels),
                                            _dptr(out)))
        return out


COUNTERS = ["samples", "bounces", "test_sphere", "test_rect", "test_cube", "test_march", "node_slabs",
            "march_slabs", "march_steps", "march_tries", "march_blocks", "hits", "lambert", "metal",
            "dielectric", "reject_tries", "unwind", "test_torus", "march_guard"]


def count_work(renderer: "HipRenderer", camera: Camera, img_params: ImageParams, samples_number: int,
               pixels: np.ndarray, seed=None) -> dict:
    """Event counts of the kernel's own traversal over the given pixels (pt_count_work)."""
    pixels = np.ascontiguousarray(pixels, dtype=np.uint32)
    out = (C.c_uint64 * len(COUNTERS))()
    s = renderer.seed if seed is None else int(seed)
    _check(lib().pt_count_work(renderer._h, C.byref(camera._c), img_params.width, img_params.height,
                               int(samples_number), s, pixels.ctypes.data_as(C.POINTER(C.c_uint32)), len(pixels),
                               out))
    return dict(zip(COUNTERS, list(out)))


def march_guard_drops(renderer: "HipRenderer") -> int:
    """Marches dropped by the 2^24-iteration guard since the last call (pt_march_guard_drops)."""
    n = C.c_uint64()
    _check(lib().pt_march_guard_drops(renderer._h, C.byref(n)))
    return n.value


def render_stop_stats(renderer: "HipRenderer"):
    """(skipped, worked) since the last call (pt_render_stop_stats): stop-gated launches that found their frame
    stopped, and those of them that still had work (0 unless the stop gate is broken)."""
    s, w = C.c_uint64(), C.c_uint64()
    _check(lib().pt_render_stop_stats(renderer._h, C.byref(s), C.byref(w)))
    return s.value, w.value


def march_jobs(renderer: "HipRenderer", jobs, status=False):
    """The skipping Heart march alone on the GPU (pt_march_jobs): jobs is an
    (n, 8) float64 array {step, passes, o, d}; returns (t, hit, iters), or
    (t, status, iters) with status 1 hit / 0 miss / 2 dropped by the guard."""
    import numpy as np
    jobs = np.ascontiguousarray(jobs, dtype=np.float64).reshape(-1, 8)
    n = len(jobs)
    t = np.zeros(n)
    st = np.zeros(n, np.int32)
    it = np.zeros(n, np.uint32)
    dp = C.POINTER(C.c_double)
    _check(lib().pt_march_jobs(renderer._h, jobs.ctypes.data_as(dp), n, t.ctypes.data_as(dp),
                               st.ctypes.data_as(C.POINTER(C.c_int32)), it.ctypes.data_as(C.POINTER(C.c_uint32))))
    return (t, st, it) if status else (t, st == 1, it)


# (slot 5 was the wavefront tail kernel until round 6; it now times the per-slot unwind, wf_unwind)
KERNEL_KINDS = ["bounce", "march", "select", "reduce", "megakernel", "unwind", "walk"]


def kernel_timing(renderer: "HipRenderer", enable: bool = True) -> dict:
    """Summed HIP-event time (ms) and launches per render-path kernel since the
    last call (pt_kernel_timing); enable/disable recording for what follows."""
    ms = (C.c_double * len(KERNEL_KINDS))()
    n = (C.c_uint32 * len(KERNEL_KINDS))()
    _check(lib().pt_kernel_timing(renderer._h, 1 if enable else 0, ms, n, len(KERNEL_KINDS)))
    return {k: (ms[i], n[i]) for i, k in enumerate(KERNEL_KINDS) if k}


def wave_diag(renderer: "HipRenderer", enable: bool = True):
    """Read-and-clear the wavefront march kernel's phase diagnostics (pt_wave_diag)."""
    out = (C.c_uint64 * 64)()
    _check(lib().pt_wave_diag(renderer._h, 1 if enable else 0, out, 64))
    return list(out)


def profile_phases(renderer: "HipRenderer", camera: Camera, img_params: ImageParams, samples_number: int,
                   seed=None) -> dict:
    """Wave-level phase timing of the megakernel's per-lane loop (pt_profile_phases)."""
    out = (C.c_uint64 * 10)()
    s = renderer.seed if seed is None else int(seed)
    _check(lib().pt_profile_phases(renderer._h, C.byref(camera._c), img_params.width, img_params.height,
                                   int(samples_number), s, out))
    return dict(zip(["trace", "march", "select", "shade", "passes", "march_passes", "max_passes",
                    "shade_finish", "shade_scatter", "shade_restart"], list(out)))


def option_names() -> list:
    out, i = [], 0
    while True:
        n = lib().pt_option_name(i)
        if n is None:
            return out
        out.append(n.decode())
        i += 1


# the defaults (pt_kernel.hpp Tuning): bench.py reports knobs that differ
OPTION_DEFAULTS = {"engine": 0, "mega_waves": 4, "diag": 0, "wf_slots": 2, "wf_paths": 0, "wf_min_chunks": 1,
                   "wf_bounce_waves": 3, "wf_march_slice": 256, "wf_walk": 5, "bvh_leaf": 1}


def shard_tiles(width: int, height: int, rank: int, world: int) -> int:
    return lib().pt_shard_tiles(width, height, rank, world)


def shard_pixels(width: int, height: int, rank: int, world: int) -> np.ndarray:
    """Pixel index (x + y*w) of each slot of rank's compact shard, -1 outside
    the frame: logical tile k (16x16) belongs to rank k % world, tiles in
    order, pixels row-major inside a tile (render_tiles' layout).  For world > 1
    logical tile k sits at column (k % tiles_x + row) % tiles_x of its row
    (dev::tile_position, a diagonal deal); world == 1 is row-major."""
    tx = (width + TILE - 1) // TILE
    ty = (height + TILE - 1) // TILE
    k = np.arange(rank, tx * ty, world)
    if world > 1:
        row = k // tx
        k = row * tx + (k % tx + row) % tx
    ly, lx = np.divmod(np.arange(TILE * TILE), TILE)
    x = (k % tx)[:, None] * TILE + lx[None, :]
    y = (k // tx)[:, None] * TILE + ly[None, :]
    idx = np.where((x < width) & (y < height), y * width + x, -1)
    return idx.ravel()


def unshard_host(gathered: np.ndarray, width: int, height: int, world: int) -> np.ndarray:
    """Host mirror of pt_unshard_device: (world, per*256, 3) shards -> (w*h, 3) frame."""
    frame = np.zeros((width * height, 3), dtype=gathered.dtype)
    for rank in range(world):
        idx = shard_pixels(width, height, rank, world)
        ok = idx >= 0
        frame[idx[ok]] = gathered[rank, : len(idx)][ok]
    return frame


def unshard_device(gathered_ptr: int, width: int, height: int, world: int, frame_ptr: int, stream_ptr: int = 0,
                   device: int = -1):
    _check(lib().pt_unshard_device(int(device), C.c_void_p(gathered_ptr), width, height, world,
                                   C.c_void_p(frame_ptr), C.c_void_p(stream_ptr)))


def encode_rgba8(buffer: np.ndarray) -> np.ndarray:
    """Display encode of src/bin/main.rs:281-289 (gamma 2, clamp, u8)."""
    buf = np.ascontiguousarray(buffer, dtype=np.float64).reshape(-1, 3)
    out = np.zeros((len(buf), 4), dtype=np.uint8)
    _check(lib().pt_encode_rgba8(_dptr(buf), len(buf), out.ctypes.data_as(C.POINTER(C.c_uint8))))
    return out


def encode_rgba8_device(rgb_ptr: int, npix: int, rgba_ptr: int, stream_ptr: int = 0, device: int = -1):
    """The display encode on the GPU (pt_encode_rgba8_device): device pointers."""
    _check(lib().pt_encode_rgba8_device(int(device), C.c_void_p(rgb_ptr), int(npix), C.c_void_p(rgba_ptr),
                                        C.c_void_p(stream_ptr)))


def _image_args(rgba: np.ndarray, width: int, height: int):
    rgba = np.ascontiguousarray(rgba, dtype=np.uint8).reshape(-1)
    if rgba.size != width * height * 4:
        raise ValueError("rgba must hold width*height*4 bytes")
    return rgba, rgba.ctypes.data_as(C.POINTER(C.c_uint8))


def write_png(path, rgba: np.ndarray, width: int, height: int):
    """image::save_buffer(path, rgba, w, h, ColorType::Rgba8) (src/bin/main.rs:71-82)."""
    buf, p = _image_args(rgba, width, height)
    _check(lib().pt_write_png(str(path).encode(), p, width, height))


def write_ppm(path, rgba: np.ndarray, width: int, height: int):
    buf, p = _image_args(rgba, width, height)
    _check(lib().pt_write_ppm(str(path).encode(), p, width, height))


# ---- resumable frames -------------------------------------------------------
def frame_key(scene_json: bytes, camera: Camera, depth: int, random_spheres: int = 1, scene_seed: int = 1) -> int:
    """A 64-bit name for what a checkpoint's sums belong to: the scene text, the scene options, the camera
    and the depth (pt_checkpoint.scene_key)."""
    h = hashlib.blake2b(digest_size=8)
    h.update(bytes(scene_json))
    h.update(struct.pack("<IQI", int(random_spheres), int(scene_seed), int(depth)))
    h.update(bytes(camera._c))
    return int.from_bytes(h.digest(), "little")


def checkpoint_count(width: int, height: int, rank: int = 0, world: int = 1) -> int:
    """Doubles in a rank's running sums (pt_render_device's d_out layout)."""
    return width * height * 3 if world == 1 else shard_tiles(width, height, rank, world) * TILE * TILE * 3


def save_checkpoint(path, sums: np.ndarray, *, width: int, height: int, samples_number: int, samples_done: int,
                    seed: int, depth: int, scene_key: int = 0, rank: int = 0, world: int = 1):
    """Write a rank's running sums after samples [0, samples_done) (pt_checkpoint_save)."""
    sums = np.ascontiguousarray(sums, dtype=np.float64).reshape(-1)
    c = CheckpointStruct(width, height, samples_number, samples_done, rank, world, depth, 0, seed, scene_key,
                         sums.size)
    _check(lib().pt_checkpoint_save(str(path).encode(), C.byref(c), _dptr(sums)))


def load_checkpoint(path, with_sums: bool = True):
    """(header as a dict, sums as a float64 array or None) of a checkpoint file (pt_checkpoint_load)."""
    c = CheckpointStruct()
    _check(lib().pt_checkpoint_load(str(path).encode(), C.byref(c), None, 0))
    sums = None
    if with_sums:
        sums = np.empty(c.count, dtype=np.float64)
        _check(lib().pt_checkpoint_load(str(path).encode(), C.byref(c), _dptr(sums), sums.size))
    return {k: getattr(c, k) for k, _ in CheckpointStruct._fields_}, sums


def sample_key(seed: int, pixel: int, sample: int) -> int:
    return lib().pt_sample_key(seed, pixel, sample)


def version() -> str:
    return lib().pt_version().decode()


def source_id() -> str:
    """The loaded build's source hash (pt_version's "src ..." field, rs-pathtracing_amd/Makefile)."""
    v = version()
    return v.split("src ", 1)[1].rstrip(")") if "src " in v else "unknown"


# pt_abi_layout struct ids and the ctypes mirror of each
ABI_STRUCTS = {0: SceneOpts, 1: CameraStruct, 2: ShapeInfo, 3: MaterialInfo, 4: HitStruct, 5: CheckpointStruct}


def abi_layout(which: int) -> list:
    """[sizeof, offsetof(field 0), ...] of a boundary struct as the library was compiled (pt_abi_layout)."""
    out = (C.c_uint32 * 64)()
    n = _check(lib().pt_abi_layout(int(which), out, 64))
    return list(out[:n])
