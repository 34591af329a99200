"""BASELINE.json configs beyond the headline one, on the GPU, through the
C-ABI (the bench measures c2; these are parity cases):

* C3 — cornell 3840x2160: the full-size frame at low spp, sampled pixels
  against the oracle, and the spp-chunked wavefront against one chunk;
* C4 — cornell 3840x2160 dealt to 8 ranks: the 8 tile shards rendered in one
  process reassemble to the single-GPU frame bit for bit (the partition is
  exact for any N because the RNG is keyed per (pixel, sample));
* C5 — the synthetic 100k-sphere scene (scenes/make_scenes.py synthetic):
  GPU BVH traversal against the oracle's reference BvhNode traversal.
"""
import json
import os
import sys
from pathlib import Path

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


@pytest.fixture(scope="module")
def cornell(pt, cornell_text):
    return pt.Scene.from_json(cornell_text, seed=1), O.Scene(cornell_text, seed=1).use_bvh(True, 7)


def test_c3_full_size_frame(pt, cornell):
    import torch
    ps, osc = cornell
    r = pt.HipRenderer(ps, depth=8)
    cam = ps.camera()
    w, h, spp = 3840, 2160, 2
    stream = torch.cuda.current_stream().cuda_stream
    frame = torch.zeros(w * h * 3, dtype=torch.float64, device="cuda")
    r.render_device(cam, w, h, spp, 1, 0, 1, frame.data_ptr(), stream)
    torch.cuda.synchronize()
    img = frame.view(-1, 3).cpu().numpy()
    assert np.all(np.isfinite(img)) and img.mean() > 0.05
    rng = np.random.default_rng(2)
    px = rng.choice(w * h, size=64, replace=False).astype(np.uint32)
    ref = osc.render(w, h, spp, 8, 1, pixels=px)
    assert np.array_equal(img[px], ref)


def test_c3_chunked_equals_unchunked(pt, cornell):
    """The full-size frame cut into 1-spp chunks and tile groups (the wf_paths option)
    sums the same samples in the same order as one chunk."""
    ps, _ = cornell
    cam = ps.camera()
    w, h, spp = 3840, 2160, 2
    r = pt.HipRenderer(ps, depth=8)
    a = r.render(cam, pt.ImageParams(w, h), spp, seed=3)
    r2 = pt.HipRenderer(ps, depth=8)
    r2.set_option("wf_paths", 1 << 22)  # 4M paths: tile groups of 16384 tiles, one sample per chunk
    b = r2.render(cam, pt.ImageParams(w, h), spp, seed=3)
    assert np.array_equal(a, b)


def test_c4_eight_rank_tiling(pt, cornell):
    import torch
    ps, _ = cornell
    r = pt.HipRenderer(ps, depth=8)
    cam = ps.camera()
    w, h, spp, world = 3840, 2160, 1, 8
    stream = torch.cuda.current_stream().cuda_stream
    full = torch.zeros(w * h * 3, dtype=torch.float64, device="cuda")
    r.render_device(cam, w, h, spp, 5, 0, 1, full.data_ptr(), stream)
    per = pt.shard_tiles(w, h, 0, world)
    assert per * world >= -(-w // 16) * -(-h // 16)  # every tile has a rank
    g = torch.zeros(world * per * 256 * 3, dtype=torch.float64, device="cuda")
    for rank in range(world):
        assert pt.shard_tiles(w, h, rank, world) <= per
        r.render_device(cam, w, h, spp, 5, rank, world, g.data_ptr() + rank * per * 256 * 3 * 8, stream)
    frame = torch.zeros_like(full)
    pt.unshard_device(g.data_ptr(), w, h, world, frame.data_ptr(), stream)
    torch.cuda.synchronize()
    assert torch.equal(frame, full)


@pytest.fixture(scope="module")
def c5(pt):
    sys.path.insert(0, str(ROOT / "scenes"))
    import make_scenes
    text = json.dumps(make_scenes.synthetic(100000))
    return text, pt.Scene.from_json(text, seed=1), O.Scene(text, seed=1).use_bvh(True, 7)


def test_c5_synthetic_100k_spheres(pt, c5):
    text, ps, osc = c5
    assert ps.num_shapes > 100000
    r = pt.HipRenderer(ps, depth=8)
    cam = ps.camera()
    w, h = 1920, 1080
    rng = np.random.default_rng(4)
    px = rng.choice(w * h, size=400, replace=False).astype(np.uint32)
    got = r.trace_pixel_samples(cam, pt.ImageParams(w, h), 4, px, seed=2)
    ref = osc.render(w, h, 4, 8, 2, pixels=px)
    assert np.array_equal(got, ref)
    img = r.render(cam, pt.ImageParams(160, 90), 2, seed=2)
    ref = osc.render(160, 90, 2, 8, 2)
    assert np.array_equal(img, ref)
    assert img.mean() > 0.05
    r.set_option("bvh_leaf", 3)  # the BVH rebuilt with 3 shapes per leaf: the same closest hits
    assert np.array_equal(r.render(cam, pt.ImageParams(160, 90), 2, seed=2), ref)
    r.set_option("bvh_leaf", 1)
    # the wavefront engine (this frame is below its automatic threshold), with the BVH walk in the bounce kernel
    # (wf_walk 0) and in its own kernel at each register budget
    r.set_option("engine", 2)
    for walk in (0, 4, 5, 6, 8):
        r.set_option("wf_walk", walk)
        assert np.array_equal(r.render(cam, pt.ImageParams(160, 90), 2, seed=2), ref), walk
    r.set_option("wf_walk", 5)
    r.set_option("bvh_leaf", 3)  # multi-shape leaves in the quantized nodes' links
    assert np.array_equal(r.render(cam, pt.ImageParams(160, 90), 2, seed=2), ref)


def test_shard_pixels_matches_device_deal(pt, cornell):
    # the host map (shard_pixels, used by unshard_host) and the kernels' diagonal deal
    # (dev::tile_position) place every shard slot on the same frame pixel
    import torch
    ps, _ = cornell
    r = pt.HipRenderer(ps, depth=8)
    cam = ps.camera()
    w, h, spp, world = 200, 72, 1, 4   # ragged edge tiles, 13 tiles per row
    stream = torch.cuda.current_stream().cuda_stream
    full = torch.zeros(w * h * 3, dtype=torch.float64, device="cuda")
    r.render_device(cam, w, h, spp, 9, 0, 1, full.data_ptr(), stream)
    per = pt.shard_tiles(w, h, 0, world)
    full_h = None
    for rank in range(world):
        s = torch.zeros(per * 256 * 3, dtype=torch.float64, device="cuda")
        r.render_device(cam, w, h, spp, 9, rank, world, s.data_ptr(), stream)
        torch.cuda.synchronize()
        if full_h is None:
            full_h = full.view(-1, 3).cpu().numpy()
        idx = pt.shard_pixels(w, h, rank, world)
        got = s.view(-1, 3).cpu().numpy()[: len(idx)]
        ok = idx >= 0
        assert np.array_equal(got[ok], full_h[idx[ok]])
