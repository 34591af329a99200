"""GPU parity: the HIP path (through the C-ABI) against the C oracle on the
same realized scene and the same counter-based RNG stream.

The bar: bit-exact f64 (the kernel is compiled with -ffp-contract=off and
follows the reference's operation order); the north_star tolerance
(per-channel RMS <= 1e-4 on linear radiance) is asserted as well, so a
single exact-tie difference cannot hide a systematic error.
"""
import math

import numpy as np
import pytest

import oracle as O
from conftest import native_lib

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-4


def rms(a, b):
    return np.sqrt(np.mean((a - b) ** 2, axis=0))


@pytest.fixture(scope="module")
def cornell(pt, cornell_text):
    return pt.Scene.from_json(cornell_text, seed=1), O.Scene(cornell_text, seed=1)


@pytest.fixture(scope="module")
def spheres(pt, spheres_text):
    return pt.Scene.from_json(spheres_text, seed=3), O.Scene(spheres_text, seed=3)


def random_rays(n, rng, box_lo, box_hi, eye=None):
    o = rng.uniform(box_lo, box_hi, size=(n, 3))
    if eye is not None:
        o[: n // 2] = eye
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return np.concatenate([o, d], axis=1)


def test_closest_hit_bit_exact(pt, cornell):
    ps, osc = cornell
    r = pt.HipRenderer(ps, depth=8)
    rng = np.random.default_rng(11)
    rays = random_rays(6000, rng, [-20, 0, -20], [555, 555, 555], eye=[278, 278, -800])
    # add rays aimed at the Heart and the random-sphere corner
    tgt = np.concatenate([rng.uniform([140, 130, 80], [285, 270, 215], size=(1500, 3)),
                          rng.uniform([-11, 0, -11], [11, 0.5, 11], size=(500, 3))])
    org = np.concatenate([np.tile([278.0, 278.0, -800.0], (1500, 1)), rng.uniform([-30, 1, -30], [30, 5, 30], (500, 3))])
    d = tgt - org
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([rays, np.concatenate([org, d], axis=1)])
    got = r.closest_hit(rays)
    mism = 0
    for i, ray in enumerate(rays):
        h = osc.closest_hit(ray[:3], ray[3:])
        g = got[i]
        if h is None:
            assert g["shape"] == -1, i
            continue
        same = (g["shape"] == h.shape and g["t"] == h.t and list(g["point"]) == list(h.point)
                and list(g["normal"]) == list(h.normal) and bool(g["front_face"]) == bool(h.front_face))
        mism += not same
    assert mism == 0, "%d of %d closest hits differ" % (mism, len(rays))


def test_ray_color_bit_exact(pt, cornell):
    ps, osc = cornell
    r = pt.HipRenderer(ps, depth=8)
    rng = np.random.default_rng(5)
    rays = random_rays(3000, rng, [50, 50, 50], [500, 500, 500], eye=[278, 278, -800])
    states = rng.integers(0, 2 ** 63, size=len(rays), dtype=np.uint64)
    st_gpu = states.copy()
    col = r.ray_color(rays, st_gpu, depth=8)
    for i in range(len(rays)):
        c, s = osc.ray_color(rays[i, :3], rays[i, 3:], 8, int(states[i]))
        assert list(col[i]) == list(c), i
        assert int(st_gpu[i]) == s, i


def render_pair(pt, scenes, w, h, spp, depth, seed, **opts):
    ps, osc = scenes
    r = pt.HipRenderer(ps, depth=depth)
    for k, v in opts.items():
        r.set_option(k, v)
    cam = ps.camera()
    img = r.render(cam, pt.ImageParams(w, h), spp, seed=seed)
    ref = osc.render(w, h, spp, depth, seed)
    return img, ref


def check_image(img, ref):
    assert np.all(np.isfinite(img))
    assert np.all(rms(img, ref) <= RMS_TOL), rms(img, ref)
    exact = np.mean(np.all(img == ref, axis=1))
    assert exact == 1.0, "bit-exact pixels: %.6f" % exact


def test_cornell_frame_parity(pt, cornell):
    img, ref = render_pair(pt, cornell, 64, 36, 4, 8, seed=1)
    check_image(img, ref)
    assert img.mean() > 0.05  # not a black frame


def test_cornell_partial_tiles_and_odd_size(pt, cornell):
    img, ref = render_pair(pt, cornell, 37, 21, 2, 8, seed=9)  # tiles cut by the frame edge
    check_image(img, ref)


def test_spheres_frame_gui_depth(pt, spheres):
    img, ref = render_pair(pt, spheres, 48, 27, 3, 50, seed=2)  # depth 50 = the bins' depth
    check_image(img, ref)


@pytest.mark.parametrize("depth", [0, 1, 2])
def test_shallow_depths(pt, cornell, depth):
    img, ref = render_pair(pt, cornell, 32, 18, 2, depth, seed=4)
    check_image(img, ref)
    if depth == 0:  # every hit is black at depth 0; only sky survives
        assert img.max() <= 1.0


def test_trace_pixel_samples_probe(pt, cornell):
    ps, osc = cornell
    r = pt.HipRenderer(ps, depth=8)
    w, h = 1920, 1080
    rng = np.random.default_rng(3)
    pixels = rng.choice(w * h, size=400, replace=False).astype(np.uint32)
    # include pixels that look at the Heart (screen centre-left) and the corner spheres
    pixels = np.concatenate([pixels, np.array([560 * 1920 + 820, 700 * 1920 + 860, 1070 * 1920 + 300], np.uint32)])
    got = r.trace_pixel_samples(ps.camera(), pt.ImageParams(w, h), 3, pixels, seed=7)
    ref = osc.render(w, h, 3, 8, 7, pixels=pixels)
    assert np.array_equal(got, ref)


def test_nonblocking_render_step(pt, cornell):
    ps, _ = cornell
    r = pt.HipRenderer(ps, depth=8)
    cam, ip = ps.camera(), pt.ImageParams(96, 64)
    want = r.render(cam, ip, 2, seed=5)
    buf = np.zeros_like(want)
    r.start_rendering(cam, ip, 2, seed=5)
    polls = 0
    while not r.render_step(buf):
        polls += 1
        assert polls < 10_000_000
    assert np.array_equal(buf, want)
    with pytest.raises(pt.PtError) as e:
        r.render_step(buf)  # the frame was consumed; step before a new start
    assert e.value.code == pt.PT_ERR_STATE


def test_device_shards_and_unshard(pt, cornell):
    import torch
    ps, _ = cornell
    r = pt.HipRenderer(ps, depth=8)
    cam = ps.camera()
    w, h, spp = 70, 45, 2
    stream = torch.cuda.current_stream().cuda_stream  # order after torch's zero-fills
    full = torch.zeros(w * h * 3, dtype=torch.float64, device="cuda")
    r.render_device(cam, w, h, spp, 3, 0, 1, full.data_ptr(), stream)
    torch.cuda.synchronize()
    world = 3
    per = pt.shard_tiles(w, h, 0, world)
    g = torch.zeros(world * per * 256 * 3, dtype=torch.float64, device="cuda")
    for rank in range(world):
        r.render_device(cam, w, h, spp, 3, rank, world, g.data_ptr() + rank * per * 256 * 3 * 8, stream)
    torch.cuda.synchronize()
    frame = torch.zeros_like(full)
    pt.unshard_device(g.data_ptr(), w, h, world, frame.data_ptr(), stream)
    torch.cuda.synchronize()
    assert torch.equal(frame, full)
    host = r.render(cam, pt.ImageParams(w, h), spp, seed=3)
    assert np.array_equal(full.cpu().numpy().reshape(-1, 3), host)


def test_count_work_diagnostic(pt, cornell):
    """The STATS build of the kernel counts its own events and renders nothing
    different: samples = pixels x spp, and rays aimed at the Heart march."""
    ps, _ = cornell
    r = pt.HipRenderer(ps, depth=8)
    w, h = 1920, 1080
    pixels = np.array([560 * w + 820, 600 * w + 900, 10 * w + 10, 900 * w + 1500], np.uint32)
    cnt = pt.count_work(r, ps.camera(), pt.ImageParams(w, h), 8, pixels, seed=3)
    assert cnt["samples"] == 8 * len(pixels)
    assert cnt["bounces"] >= cnt["samples"]
    assert cnt["test_rect"] >= 6 * cnt["bounces"]  # the 6 uniform rectangles are tested every bounce
    assert cnt["test_march"] > 0 and cnt["march_tries"] > 0


def test_engines_agree_with_oracle(pt, cornell):
    """Cornell has the ray-marched Heart, so the default engine is the
    wavefront one; the megakernel must give the same bits, and both the
    oracle's."""
    ps, osc = cornell
    r = pt.HipRenderer(ps, depth=8)
    cam, ip = ps.camera(), pt.ImageParams(80, 45)
    wave = r.render(cam, ip, 3, seed=21)
    r.set_option("engine", 1)  # megakernel
    mega = r.render(cam, ip, 3, seed=21)
    assert np.array_equal(wave, mega)
    check_image(wave, osc.render(80, 45, 3, 8, 21))


def test_wavefront_chunk_size_invariance(pt, cornell):
    """The wavefront frame is the same bits whatever its chunking: the default chunks against tiny chunks and
    tile groups (768 path slots), and both against the oracle.  (The fused-bounce mode this test also covered
    until round 4 was removed in round 5: measured slower, and the path state no longer stores the depth.)"""
    ps, osc = cornell
    r = pt.HipRenderer(ps, depth=8)
    cam, ip = ps.camera(), pt.ImageParams(96, 54)
    r.set_option("engine", 2)  # wavefront
    split = r.render(cam, ip, 4, seed=31)
    r.set_option("wf_paths", 256 * 3)
    small = r.render(cam, ip, 4, seed=31)
    assert np.array_equal(split, small)
    check_image(split, osc.render(96, 54, 4, 8, 31))


@pytest.mark.parametrize("waves", [2, 4, 5, 6, 8])
def test_bounce_register_budgets(pt, cornell, waves):
    """Every register budget of the bounce kernel (wf_bounce_waves; the 5-, 6- and 8-wave builds spill) renders
    the oracle's pixels on the marched scene (the default 3 is every other test of this file)."""
    img, ref = render_pair(pt, cornell, 64, 36, 3, 8, seed=21, wf_bounce_waves=waves, engine=2)
    check_image(img, ref)


def test_wavefront_chunks_and_tile_groups(pt, cornell):
    """A tiny path budget forces one-tile groups and one-sample chunks: the
    running per-pixel sums must still add samples in order."""
    img, ref = render_pair(pt, cornell, 37, 21, 3, 8, seed=9, wf_paths=300)
    check_image(img, ref)
    # 7 tiles x 1 spp per chunk, ragged last group; one slot and three slots in flight
    for slots in (1, 3):
        img, ref = render_pair(pt, cornell, 70, 45, 2, 8, seed=10, wf_paths=256 * 7, wf_slots=slots)
        check_image(img, ref)
    # uneven sample chunks: 6 tiles, 2 spp per chunk at most, 5 spp -> 3 chunks,
    # rounded up to 4 for two streams and balanced to 2, 1, 1, 1 samples
    img, ref = render_pair(pt, cornell, 37, 21, 5, 8, seed=12, wf_paths=256 * 6 * 2, wf_slots=2)
    check_image(img, ref)


def test_wavefront_deep_paths(pt, spheres, cornell):
    """Depth 50 (the bins' depth) through the wavefront engine: 32-word stacks."""
    img, ref = render_pair(pt, spheres, 40, 24, 2, 50, seed=6, engine=2)
    check_image(img, ref)
    img, ref = render_pair(pt, cornell, 24, 16, 2, 20, seed=6, engine=2)
    check_image(img, ref)


def test_wavefront_shards(pt, cornell):
    """Compact per-rank shards from the wavefront engine un-interleave to the
    single-rank frame."""
    import torch
    ps, _ = cornell
    r = pt.HipRenderer(ps, depth=8)
    cam = ps.camera()
    w, h, spp, world = 53, 40, 2, 2
    stream = torch.cuda.current_stream().cuda_stream
    per = pt.shard_tiles(w, h, 0, world)
    g = torch.zeros(world * per * 256 * 3, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    for rank in range(world):
        r.render_device(cam, w, h, spp, 8, rank, world, g.data_ptr() + rank * per * 256 * 3 * 8, stream)
    frame = torch.zeros(w * h * 3, dtype=torch.float64, device="cuda")
    # render_device and unshard_device queue on the same (torch current) stream: ordered
    pt.unshard_device(g.data_ptr(), w, h, world, frame.data_ptr(), stream)
    torch.cuda.synchronize()
    r.set_option("engine", 1)  # megakernel
    want = r.render(cam, pt.ImageParams(w, h), spp, seed=8)
    assert np.array_equal(frame.cpu().numpy().reshape(-1, 3), want)


def test_heart_march_many_rays(pt, cornell):
    """Tens of thousands of rays through the Heart's bound (camera rays and
    rays leaving its surface), closest hit on the GPU vs the oracle: catches
    device-only numerics in the skipping march (hardware reciprocals etc.)."""
    ps, osc = cornell
    r = pt.HipRenderer(ps, depth=8)
    rng = np.random.default_rng(17)
    n = 12000
    eye = np.tile([278.0, 278.0, -800.0], (n, 1))
    tgt = rng.uniform([120, 120, 60], [310, 280, 240], size=(n, 3))
    d1 = tgt - eye
    d1 /= np.linalg.norm(d1, axis=1, keepdims=True)
    # origins on / near the Heart, random directions (bounce rays)
    o2 = rng.uniform([150, 140, 90], [280, 260, 210], size=(n, 3))
    d2 = rng.normal(size=(n, 3))
    d2 /= np.linalg.norm(d2, axis=1, keepdims=True)
    rays = np.concatenate([np.concatenate([eye, d1], 1), np.concatenate([o2, d2], 1)])
    got = r.closest_hit(rays)
    bad = 0
    for i, ray in enumerate(rays):
        h = osc.closest_hit(ray[:3], ray[3:])
        g = got[i]
        if h is None:
            bad += g["shape"] != -1
        else:
            bad += not (g["shape"] == h.shape and g["t"] == h.t)
    assert bad == 0, "%d of %d rays differ" % (bad, len(rays))


def test_count_work_matches_host_build(pt, cornell, cornell_text):
    """The GPU's STATS counters equal the host build's of the same code,
    event for event (the FLOP side of the roofline rests on them)."""
    import ctypes as C
    import subprocess
    from pathlib import Path
    native = Path(__file__).resolve().parent / "native"
    subprocess.run(["make", "-s", "-C", str(native)], check=True)
    L = C.CDLL(native_lib("libpath.so"))
    L.h_scene_new.restype = C.c_void_p
    L.h_scene_new.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_uint64]
    L.h_count_work.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64,
                               C.POINTER(C.c_uint32), C.c_size_t, C.POINTER(C.c_uint64)]
    raw = cornell_text.encode()
    h = L.h_scene_new(raw, len(raw), 1, 1)
    ps, _ = cornell
    r = pt.HipRenderer(ps, depth=8)
    w, hh = 1920, 1080
    rng = np.random.default_rng(9)
    px = np.concatenate([rng.choice(w * hh, 200, replace=False),
                         np.arange(64) * 12 + 1688069]).astype(np.uint32)
    got = pt.count_work(r, ps.camera(), pt.ImageParams(w, hh), 4, px, seed=1)
    want = (C.c_uint64 * len(pt.COUNTERS))()
    L.h_count_work(h, w, hh, 4, 8, 1, px.ctypes.data_as(C.POINTER(C.c_uint32)), len(px), want)
    assert got == dict(zip(pt.COUNTERS, list(want)))


def test_marched_functions_frame_and_hits(pt):
    """scenes/marched.json: every reference ShapeFunction (Heart, Sine, Star,
    DupinCyclide, HuntsSurface, Cushion) through the GPU's generic skipping
    march, both engines, against the oracle's literal march."""
    from conftest import scene_text
    text = scene_text("marched.json")
    ps = pt.Scene.from_json(text, random_spheres=False)
    osc = O.Scene(text, random_spheres=False)
    img, ref = render_pair(pt, (ps, osc), 96, 54, 2, 8, seed=3)
    check_image(img, ref)
    r = pt.HipRenderer(ps, depth=8)
    r.set_option("engine", 1)  # megakernel
    mega = r.render(ps.camera(), pt.ImageParams(96, 54), 2, seed=3)
    assert np.array_equal(mega, img)
    rng = np.random.default_rng(31)
    rays = []
    for i in range(2, 8):
        m = list(osc.shape(i).direct)
        c = np.array([m[3], m[7], m[11]])
        tgt = c + rng.uniform(-2, 2, size=(800, 3))
        o = np.tile([0.0, 3.5, -16.0], (800, 1))
        o[400:] = c + rng.uniform(-3, 3, size=(400, 3))
        d = tgt - o
        d[400:] = rng.normal(size=(400, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        rays.append(np.concatenate([o, d], 1))
    rays = np.concatenate(rays)
    got = r.closest_hit(rays)
    bad = 0
    for i, ray in enumerate(rays):
        h = osc.closest_hit(ray[:3], ray[3:])
        g = got[i]
        bad += (g["shape"] != -1) if h is None else not (g["shape"] == h.shape and g["t"] == h.t)
    assert bad == 0, "%d of %d rays differ" % (bad, len(rays))


def test_kernel_timing_from_first_frame(pt, cornell):
    """Timing enabled on a fresh renderer (before its workspace exists) covers
    the first frame; timing and the image do not depend on each other."""
    ps, _ = cornell
    r = pt.HipRenderer(ps, depth=8)
    cam, ip = ps.camera(), pt.ImageParams(48, 32)
    pt.kernel_timing(r, True)
    img = r.render(cam, ip, 2, seed=4)
    kt = pt.kernel_timing(r, False)
    assert kt["bounce"][1] > 0 and kt["bounce"][0] > 0.0
    assert kt["march"][1] > 0 and kt["select"][1] > 0 and kt["reduce"][1] > 0
    assert kt["unwind"][1] == kt["reduce"][1]  # a frame this small unwinds its slots in their own pass
    assert np.array_equal(img, r.render(cam, ip, 2, seed=4))


# ---------------------------------------------------------------- textures
# The texture lookups call sin / acos / atan2, which the GPU evaluates with
# the ROCm device math library and the oracle with glibc (as the reference
# does through Rust's std).  Both are faithful to within an ulp but not always
# equal: a NoiseTexture value (a sin) can differ in its last bit (measured:
# <= 2.2e-15 relative, 1-4 % of pixels), and a checker or texel boundary could
# flip for a rare sample.  The bar: the north_star RMS tolerance, and all but a
# rare pixel within 1e-12 relative of the oracle.
TEX_REL = 1e-12
TEX_CLOSE_MIN = 0.998


@pytest.mark.parametrize("name,seed,depth", [("textured.json", 1, 8), ("noise.json", 2, 8),
                                             ("textured.json", 3, 50), ("torus.json", 2, 8)])
def test_textured_frames(pt, name, seed, depth, monkeypatch):
    """Textured scenes and the Torus (extended builds).  The Torus' quartic
    (equation.rs:17-67) runs through hypot / atan2 / sin / cos / cbrt, so it
    shares the texture tolerance."""
    from conftest import ROOT, scene_text
    monkeypatch.chdir(ROOT)
    text = scene_text(name)
    scenes = (pt.Scene.from_json(text, seed=seed), O.Scene(text, seed=seed))
    img, ref = render_pair(pt, scenes, 64, 36, 4, depth, seed=seed)
    check_image_tol(img, ref)
    assert img.mean() > 0.05


def test_textured_deep_frame_fits_device_memory(pt, monkeypatch):
    """A textured scene at the reference GUI's depth 50, 1920x1080, 128 spp: each path slot carries
    (depth + 1) * 24 B of textured attenuation values, so the by-depth chunk (256M paths since round 6; 128M before)
    would need ~430 GB per chunk stream; the engine sizes its chunks to the device memory instead and the frame
    renders.  A sample of
    pixels is checked against the oracle at the texture tolerance."""
    import torch
    from conftest import ROOT, host_threads, scene_text
    monkeypatch.chdir(ROOT)
    text = scene_text("textured.json")
    w, h, spp, depth, seed = 1920, 1080, 128, 50, 5
    ps, osc = pt.Scene.from_json(text, seed=1), O.Scene(text, seed=1)
    r = pt.HipRenderer(ps, depth=depth)
    frame = torch.zeros(w * h * 3, dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    r.render_device(ps.camera(), w, h, spp, seed, 0, 1, frame.data_ptr(), stream)
    torch.cuda.synchronize()
    img = frame.view(-1, 3).cpu().numpy()
    assert np.all(np.isfinite(img)) and img.mean() > 0.05
    px = np.random.default_rng(12).choice(w * h, size=96, replace=False).astype(np.uint32)
    ref = osc.render(w, h, spp, depth, seed, pixels=px, threads=host_threads())
    check_image_tol(img[px], ref)


def check_image_tol(img, ref):
    assert np.all(np.isfinite(img))
    assert np.all(rms(img, ref) <= RMS_TOL), rms(img, ref)
    close = np.mean(np.all(np.abs(img - ref) <= TEX_REL * np.abs(ref), axis=1))
    assert close >= TEX_CLOSE_MIN, "pixels within %g relative: %.6f" % (TEX_REL, close)


def test_textured_probes_and_shards(pt, monkeypatch):
    from conftest import ROOT, scene_text
    monkeypatch.chdir(ROOT)
    text = scene_text("textured.json")
    ps, osc = pt.Scene.from_json(text, seed=4), O.Scene(text, seed=4)
    r = pt.HipRenderer(ps, depth=8)
    cam = ps.camera()
    w, h = 96, 54
    rng = np.random.default_rng(8)
    pixels = rng.choice(w * h, size=300, replace=False).astype(np.uint32)
    got = r.trace_pixel_samples(cam, pt.ImageParams(w, h), 3, pixels, seed=6)
    ref = osc.render(w, h, 3, 8, 6, pixels=pixels)
    check_image_tol(got, ref)
    rays = random_rays(500, rng, [-3, 0.1, -4], [3, 3, 3], eye=[0, 2.2, -9])
    states = rng.integers(0, 2 ** 63, size=len(rays), dtype=np.uint64)
    st_gpu = states.copy()
    col = r.ray_color(rays, st_gpu, depth=8)
    refc = np.array([osc.ray_color(ray[:3], ray[3:], 8, int(s))[0] for ray, s in zip(rays, states)])
    check_image_tol(col, refc)
    # tile shards of a textured frame reassemble to the single-GPU frame
    full = r.render(cam, pt.ImageParams(w, h), 2, seed=1)
    world = 3
    per = pt.shard_tiles(w, h, 0, world)
    import torch
    stream = torch.cuda.current_stream().cuda_stream  # order after torch's zero-fills
    shards = torch.zeros(world * per * 256 * 3, dtype=torch.float64, device="cuda")
    frame = torch.zeros(w * h * 3, dtype=torch.float64, device="cuda")
    for k in range(world):
        r.render_device(cam, w, h, 2, 1, k, world, shards.data_ptr() + k * per * 256 * 3 * 8, stream)
    pt.unshard_device(shards.data_ptr(), w, h, world, frame.data_ptr(), stream)
    torch.cuda.synchronize()
    assert np.array_equal(frame.view(-1, 3).cpu().numpy(), full)
    cnt = pt.count_work(r, cam, pt.ImageParams(w, h), 2, pixels, seed=1)
    assert cnt["samples"] == 2 * len(pixels)


def test_bvh_signed_zero_and_axis_rays_on_device(pt):
    """The device BVH walk (near/far planes per octant layout, octant from the direction's sign bits) on rays
    with +0 / -0 / denormal components and origins around the spheres' bounding planes: the GPU's closest hits
    equal the oracle's linear scan (the host build runs the same rays in tests/test_path_host.py)."""
    import json
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "scenes"))
    import make_scenes
    scene = make_scenes.synthetic(400)
    text = json.dumps(scene)
    ps, osc = pt.Scene.from_json(text, seed=1), O.Scene(text, seed=1)
    r = pt.HipRenderer(ps, depth=8)
    rng = np.random.default_rng(11)
    centres = [np.array(s["transform"]["translate"], float) for s in scene["shapes"][1:]]
    rays = []
    for _ in range(2000):
        o = centres[rng.integers(len(centres))] + rng.choice([-0.2000001, 0.2000001, 0.1, 0.0], size=3) \
            + rng.choice([0.0, 0.5, -0.5], size=3)
        o[1] = max(o[1], 0.05)
        d = np.zeros(3)
        k = rng.integers(3)
        d[k] = rng.choice([-1.0, 1.0])
        for j in range(3):
            if j != k:
                d[j] = rng.choice([0.0, -0.0, 1e-300, -1e-300, rng.normal() * 0.3])
        d /= np.linalg.norm(d)
        rays.append(np.concatenate([o, d]))
    rays = np.array(rays)
    got = r.closest_hit(rays)
    hits = 0
    for i, ray in enumerate(rays):
        h = osc.closest_hit(ray[:3], ray[3:])
        g = got[i]
        if h is None:
            assert g["shape"] == -1, ray
            continue
        hits += 1
        assert (g["shape"], g["t"], list(g["point"])) == (h.shape, h.t, list(h.point)), ray
    assert hits > 300
