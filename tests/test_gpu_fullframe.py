"""Whole-frame parity at the headline size, and adversarial march rays, on the GPU.

* The full C2 frame (cornell_box 1920x1080, depth 8, seed 1) at 2 spp from the
  HIP renderer, compared with the oracle's ShapeCollection linear scan
  (src/world/shapes/mod.rs:573-597 with the literal march of
  ray_marching.rs:20-74) on every one of its 2,073,600 pixels: bit-exact, and
  the north_star's per-channel RMS <= 1e-4 over the frame.
* Adversarial rays for the skipping march (tests/adversarial.py: grazing,
  frozen / zero-crossing coordinates, binade edges; several step / depth
  settings) through the GPU's closest-hit and ray_color kernels against the
  oracle.
"""
import numpy as np
import pytest

import adversarial as A
import oracle as O
from conftest import host_threads

pytestmark = pytest.mark.gpu


def test_c2_full_frame_every_pixel(pt, cornell_text):
    import torch
    w, h, spp, depth, seed = 1920, 1080, 2, 8, 1
    ps = pt.Scene.from_json(cornell_text, seed=1)
    r = pt.HipRenderer(ps, depth=depth)
    frame = torch.zeros(w * h * 3, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    r.render_device(ps.camera(), w, h, spp, seed, 0, 1, frame.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    img = frame.view(-1, 3).cpu().numpy()
    ref = O.Scene(cornell_text, seed=1).render(w, h, spp, depth, seed, threads=host_threads())
    rms = np.sqrt(np.mean((img - ref) ** 2, axis=0))
    assert np.all(rms <= 1e-4), rms
    bad = np.nonzero(np.any(img != ref, axis=1))[0]
    assert len(bad) == 0, "%d of %d pixels differ, first %s" % (len(bad), w * h, bad[:10])


def _every_pixel(img, ref):
    rms = np.sqrt(np.mean((img - ref) ** 2, axis=0))
    assert np.all(rms <= 1e-4), rms
    bad = np.nonzero(np.any(img != ref, axis=1))[0]
    assert len(bad) == 0, "%d of %d pixels differ, first %s" % (len(bad), len(img), bad[:10])


def test_c2_multichunk_two_streams_every_pixel(pt, cornell_text):
    """The timed frame's structure at the headline size: several sample chunks
    on two chunk streams, per-pixel sums chained across the streams in chunk
    order (pt_wave.hip render_wave_nw) — here 4 chunks of 2 spp (wf_paths =
    2^22) in two rounds of the 2 streams — every pixel against the oracle
    (src/renderer/mod.rs:151-155: the in-order per-pixel sum)."""
    import torch
    w, h, spp, depth, seed = 1920, 1080, 8, 8, 1
    ps = pt.Scene.from_json(cornell_text, seed=1)
    r = pt.HipRenderer(ps, depth=depth)
    r.set_option("wf_paths", 1 << 22)
    assert r.get_option("wf_slots") == 2
    frame = torch.zeros(w * h * 3, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    pt.kernel_timing(r, True)
    r.render_device(ps.camera(), w, h, spp, seed, 0, 1, frame.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    kt = pt.kernel_timing(r, False)
    assert kt["reduce"][1] == 4  # four chunks, one per-pixel reduce each
    img = frame.view(-1, 3).cpu().numpy()
    ref = O.Scene(cornell_text, seed=1).use_bvh(True, 7).render(w, h, spp, depth, seed, threads=host_threads())
    _every_pixel(img, ref)


def test_c3_full_frame_every_pixel(pt, cornell_text):
    """C3's 3840x2160 frame (BASELINE configs[2]) at 2 spp, every pixel."""
    import torch
    w, h, spp, depth, seed = 3840, 2160, 2, 8, 3
    ps = pt.Scene.from_json(cornell_text, seed=1)
    r = pt.HipRenderer(ps, depth=depth)
    frame = torch.zeros(w * h * 3, dtype=torch.float64, device="cuda")
    r.render_device(ps.camera(), w, h, spp, seed, 0, 1, frame.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    img = frame.view(-1, 3).cpu().numpy()
    del frame
    ref = O.Scene(cornell_text, seed=1).use_bvh(True, 7).render(w, h, spp, depth, seed, threads=host_threads())
    _every_pixel(img, ref)


def test_c5_full_frame_every_pixel(pt):
    """C5's synthetic 100k-sphere scene (BASELINE configs[4]) at 1920x1080, 2 spp,
    every pixel against the oracle's reference BvhNode traversal
    (src/world/shapes/mod.rs:620-729)."""
    import json
    import sys
    from pathlib import Path
    import torch
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "scenes"))
    import make_scenes
    text = json.dumps(make_scenes.synthetic(100000))
    w, h, spp, depth, seed = 1920, 1080, 2, 8, 2
    ps = pt.Scene.from_json(text, seed=1)
    r = pt.HipRenderer(ps, depth=depth)
    frame = torch.zeros(w * h * 3, dtype=torch.float64, device="cuda")
    r.render_device(ps.camera(), w, h, spp, seed, 0, 1, frame.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    img = frame.view(-1, 3).cpu().numpy()
    ref = O.Scene(text, seed=1).use_bvh(True, 7).render(w, h, spp, depth, seed, threads=host_threads())
    _every_pixel(img, ref)


def test_c1_full_frame_every_pixel(pt, spheres_text):
    """C1 at its own size (BASELINE configs[0]: spheres.json 256x256, 16 spp, depth 8, the bench's scene seed 1):
    the frame through the C-ABI renderer against the oracle's linear scan with the literal march, every pixel
    (1,048,576 samples, two marched Hearts)."""
    w, h, spp, depth, seed = 256, 256, 16, 8, 1
    ps = pt.Scene.from_json(spheres_text, seed=1)
    r = pt.HipRenderer(ps, depth=depth)
    img = r.render(ps.camera(), pt.ImageParams(w, h), spp, seed=seed)
    ref = O.Scene(spheres_text, seed=1).render(w, h, spp, depth, seed, threads=host_threads())
    _every_pixel(img, ref)
    assert img.mean() > 0.05  # not a black frame


def _compare_hits(got, osc, rays):
    bad = []
    for i, ray in enumerate(rays):
        hh = osc.closest_hit(ray[:3], ray[3:])
        g = got[i]
        if hh is None:
            ok = g["shape"] == -1
        else:
            ok = (g["shape"] == hh.shape and g["t"] == hh.t and list(g["normal"]) == list(hh.normal))
        if not ok:
            bad.append(i)
    return bad


@pytest.mark.parametrize("xf,step,depth", [
    ("cornell", 0.01, None), ("unit", 0.01, None), ("scaled", 0.01, None),
    ("unit", 0.05, 4), ("unit", 0.003, 4), ("unit", 0.01, 1), ("unit", 0.01, 0), ("unit", 0.02, 5),
    ("unit", -0.01, 4), ("cornell", 0.003, 4)])
def test_adversarial_march_rays_closest_hit(pt, xf, step, depth):
    tr = {"cornell": A.HEART_XF, "unit": A.UNIT_XF, "scaled": A.SCALED_XF}[xf]
    js = A.heart_json(tr, step=step, depth=depth)
    ps = pt.Scene.from_json(js, random_spheres=False)
    osc = O.Scene(js, random_spheres=False)
    rays = A.world_rays(ps.shape(0).direct, A.object_rays(np.random.default_rng(47)))
    got = pt.HipRenderer(ps, depth=8).closest_hit(rays)
    bad = _compare_hits(got, osc, rays)
    assert not bad, "%d of %d rays differ: %s" % (len(bad), len(rays), rays[bad[:3]])


def test_adversarial_rays_in_the_cornell_scene(pt, cornell_text):
    """The same families aimed at cornell's Heart inside the full scene (walls,
    cubes, random spheres): closest hit, and whole paths (ray_color, depth 8)."""
    ps = pt.Scene.from_json(cornell_text, seed=1)
    osc = O.Scene(cornell_text, seed=1)
    k = next(i for i in range(ps.num_shapes) if ps.shape(i).type == pt.MARCH)
    rng = np.random.default_rng(53)
    rays = A.world_rays(ps.shape(k).direct, A.object_rays(rng))
    r = pt.HipRenderer(ps, depth=8)
    bad = _compare_hits(r.closest_hit(rays), osc, rays)
    assert not bad, "%d of %d closest hits differ" % (len(bad), len(rays))
    states = rng.integers(0, 2 ** 63, size=len(rays), dtype=np.uint64)
    st = states.copy()
    col = r.ray_color(rays, st, depth=8)
    for i in range(len(rays)):
        c, s = osc.ray_color(rays[i, :3], rays[i, 3:], 8, int(states[i]))
        assert list(col[i]) == list(c) and int(st[i]) == s, i


def test_march_guard_counts_sub_ulp_step(pt):
    """A step below the rounding of t (t + step == t): the reference's march
    (ray_marching.rs:37-51) never ends.  Here the march guard drops it after
    2^24 skipping iterations, the ray is a miss for that shape, and the drop is
    counted (pt_march_guard_drops) instead of passing silently."""
    js = A.heart_json(A.UNIT_XF, step=1e-30, depth=4)
    ps = pt.Scene.from_json(js, random_spheres=False)
    r = pt.HipRenderer(ps, depth=8)
    assert pt.march_guard_drops(r) == 0
    rng = np.random.default_rng(59)
    n = 64
    o = np.tile([0.0, 0.0, -5.0], (n, 1))
    d = rng.uniform(-0.3, 0.3, size=(n, 3)) - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    hits = r.closest_hit(np.concatenate([o, d], 1))
    assert np.all(hits["shape"] == -1)
    assert pt.march_guard_drops(r) == n
    assert pt.march_guard_drops(r) == 0  # read and cleared
    jobs = np.concatenate([np.tile([1e-30, 4.0], (n, 1)), o, d], 1)  # {step, passes, o, d}
    t, st, it = pt.march_jobs(r, jobs, status=True)
    assert np.all(st == 2) and np.all(it >= 2 ** 24 - 1)
    # a whole frame (wavefront engine) still finishes, and counts its drops
    img = r.render(ps.camera(), pt.ImageParams(4, 4), 1, seed=1)
    assert np.all(np.isfinite(img))
    # A grazing ray at 7 passes (the last pass steps by 2e-14): f stays inside
    # the rounding band around 0 for so many steps that the reference's literal
    # march (the oracle) does not end within minutes; the skipping march hits
    # the guard after 2^24 iterations and counts it.
    js7 = A.heart_json(A.UNIT_XF, step=0.02, depth=7)
    ps7 = pt.Scene.from_json(js7, random_spheres=False)
    r7 = pt.HipRenderer(ps7, depth=8)
    ray = A.world_rays(ps7.shape(0).direct, A.object_rays(np.random.default_rng(47)))[97:98]
    assert r7.closest_hit(ray)["shape"][0] == -1
    assert pt.march_guard_drops(r7) == 1
    # a normal scene drops nothing
    js2 = A.heart_json(A.HEART_XF)
    r2 = pt.HipRenderer(pt.Scene.from_json(js2, random_spheres=False), depth=8)
    r2.render(r2.scene.camera(), pt.ImageParams(64, 36), 2, seed=1)
    assert pt.march_guard_drops(r2) == 0
