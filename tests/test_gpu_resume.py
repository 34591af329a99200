"""Resumable frames on the GPU (pt_render_device_samples + checkpoint files).

A frame cut into sample windows [0, a), [a, b), ..., [z, spp) -- with the
running sums written to a checkpoint file, the renderer destroyed and a new one
created between windows -- must leave the frame buffer bit-identical to one
pt_render_device call, and so to the oracle (the sums add samples in index
order and every sample keeps its frame-wide RNG key; the reference renders the
frame in one go, src/renderer/mod.rs:67-114).  Covered: one rank and shards of
a 2- and 3-rank frame, a ray-marched scene, windows split over several tile
groups and sample chunks (a small wf_paths), and invalid windows.
"""
import numpy as np
import pytest

import oracle as O
from conftest import ROOT, host_threads

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cornell(pt, cornell_text):
    return pt.Scene.from_json(cornell_text, seed=1), O.Scene(cornell_text, seed=1).use_bvh(True, 7)


def one_shot(pt, r, cam, w, h, spp, seed, rank, world):
    import torch
    out = torch.zeros(pt.checkpoint_count(w, h, rank, world), dtype=torch.float64, device="cuda")
    r.render_device(cam, w, h, spp, seed, rank, world, out.data_ptr())
    torch.cuda.synchronize()
    return out.cpu().numpy()


def windowed(pt, make_renderer, cam, w, h, spp, seed, rank, world, cuts, ckpt=None, key=0):
    """Render [0, spp) in the windows `cuts` splits it into; with ckpt, every window but the last ends in a
    checkpoint file and the next window starts from a new renderer and the file's sums."""
    import torch
    n = pt.checkpoint_count(w, h, rank, world)
    out = torch.full((n,), float("nan"), dtype=torch.float64, device="cuda")  # s_begin 0 must not read it
    r = make_renderer()
    edges = [0] + list(cuts) + [spp]
    for a, b in zip(edges, edges[1:]):
        r.render_device_samples(cam, w, h, spp, seed, rank, world, a, b, out.data_ptr())
        torch.cuda.synchronize()
        if ckpt is not None and b < spp:
            pt.save_checkpoint(ckpt, out.cpu().numpy(), width=w, height=h, samples_number=spp, samples_done=b,
                               seed=seed, depth=r.depth, scene_key=key, rank=rank, world=world)
            del out, r
            hd, sums = pt.load_checkpoint(ckpt)
            assert (hd["samples_done"], hd["scene_key"], hd["rank"], hd["world"]) == (b, key, rank, world)
            out = torch.from_numpy(sums).to("cuda")
            r = make_renderer()
    return out.cpu().numpy()


def bits(a):
    return np.ascontiguousarray(a).view(np.uint64)


def test_windows_equal_one_launch_and_the_oracle(pt, cornell, tmp_path, cornell_text):
    ps, osc = cornell
    cam = ps.camera()
    w, h, spp, seed = 96, 64, 12, 3
    mk = lambda: pt.HipRenderer(ps, depth=8)  # noqa: E731
    full = one_shot(pt, mk(), cam, w, h, spp, seed, 0, 1)
    key = pt.frame_key(cornell_text.encode(), cam, 8)
    got = windowed(pt, mk, cam, w, h, spp, seed, 0, 1, [1, 5, 11], ckpt=tmp_path / "f.ckpt", key=key)
    assert np.array_equal(bits(got), bits(full))
    ref = osc.render(w, h, spp, 8, seed, threads=host_threads())
    assert np.array_equal(got.reshape(-1, 3), ref)


@pytest.mark.parametrize("world", [2, 3])
def test_shard_windows_equal_one_launch(pt, cornell, tmp_path, world):
    ps, _ = cornell
    cam = ps.camera()
    w, h, spp, seed = 120, 72, 9, 5
    mk = lambda: pt.HipRenderer(ps, depth=8)  # noqa: E731
    for rank in range(world):
        full = one_shot(pt, mk(), cam, w, h, spp, seed, rank, world)
        got = windowed(pt, mk, cam, w, h, spp, seed, rank, world, [4], ckpt=tmp_path / ("r%d.ckpt" % rank))
        assert np.array_equal(bits(got), bits(full)), rank


def test_windows_over_tile_groups_and_chunks(pt, cornell):
    """wf_paths small: each window runs as several tile groups of several sample chunks (each group's first
    chunk reads the running sums, its last one stores them)."""
    ps, _ = cornell
    cam = ps.camera()
    w, h, spp, seed = 80, 48, 10, 9

    def mk():
        r = pt.HipRenderer(ps, depth=8)
        r.set_option("wf_paths", 1024)  # 4 tiles per group, 1 sample per chunk
        return r
    full = one_shot(pt, pt.HipRenderer(ps, depth=8), cam, w, h, spp, seed, 0, 1)
    for cuts in ([3], [1, 2, 3, 9], list(range(1, 10))):
        got = windowed(pt, mk, cam, w, h, spp, seed, 0, 1, cuts)
        assert np.array_equal(bits(got), bits(full)), cuts


def test_marched_scene_windows(pt, tmp_path):
    """A ray-marched heart (the persistent march kernel between bounces): windows == one launch."""
    text = (ROOT / "scenes" / "marched.json").read_text()
    ps = pt.Scene.from_json(text, seed=1)
    cam = ps.camera()
    w, h, spp, seed = 64, 48, 6, 2
    mk = lambda: pt.HipRenderer(ps, depth=8)  # noqa: E731
    full = one_shot(pt, mk(), cam, w, h, spp, seed, 0, 1)
    got = windowed(pt, mk, cam, w, h, spp, seed, 0, 1, [2, 3], ckpt=tmp_path / "m.ckpt")
    assert np.array_equal(bits(got), bits(full))


def test_invalid_windows(pt, cornell):
    import torch
    ps, _ = cornell
    cam = ps.camera()
    r = pt.HipRenderer(ps, depth=8)
    out = torch.zeros(64 * 32 * 3, dtype=torch.float64, device="cuda")
    for a, b in [(0, 0), (5, 3), (4, 4), (0, 9)]:
        with pytest.raises(pt.PtError) as e:
            r.render_device_samples(cam, 64, 32, 8, 1, 0, 1, a, b, out.data_ptr())
        assert e.value.code == pt.PT_ERR_INVALID


def test_cli_render_interrupted_and_resumed(tmp_path):
    """tools/pt_render (the headless CLI over the C-ABI): a frame stopped after its first window (-x 1, exit 3,
    checkpoint kept) and resumed by a second process equals the frame rendered in one go, bit for bit; the
    checkpoint is removed when the frame completes, and the image is a PNG."""
    import subprocess
    exe = str(ROOT / "tools" / "pt_render")
    scene = str(ROOT / "scenes" / "cornell_box.json")
    args = [exe, scene, "12", "96", "64", "-d", "8", "-s", "3"]
    one = subprocess.run(args + ["-f", str(tmp_path / "one.f64"), "-o", str(tmp_path / "one.png")],
                         capture_output=True, text=True, timeout=120)
    assert one.returncode == 0, one.stderr
    ck = tmp_path / "frame.ckpt"
    first = subprocess.run(args + ["-c", str(ck), "-n", "5", "-x", "1", "-o", ""], capture_output=True, text=True,
                           timeout=120)
    assert first.returncode == 3, first.stderr
    assert ck.exists()
    second = subprocess.run(args + ["-c", str(ck), "-n", "5", "-f", str(tmp_path / "res.f64"), "-o", ""],
                            capture_output=True, text=True, timeout=120)
    assert second.returncode == 0, second.stderr
    assert "resuming at sample 5 of 12" in second.stderr
    assert not ck.exists()
    assert (tmp_path / "one.f64").read_bytes() == (tmp_path / "res.f64").read_bytes()
    assert (tmp_path / "one.png").read_bytes()[:8] == b"\x89PNG\r\n\x1a\n"


def test_cli_refuses_an_unloadable_checkpoint(tmp_path):
    """An existing checkpoint file that does not load (here: not a checkpoint) stops the CLI with exit 1 and the
    library's message; the file is left as it was, never overwritten by a frame started from sample 0."""
    import subprocess
    exe = str(ROOT / "tools" / "pt_render")
    ck = tmp_path / "frame.ckpt"
    ck.write_bytes(b"not a checkpoint at all")
    r = subprocess.run([exe, str(ROOT / "scenes" / "cornell_box.json"), "4", "32", "16", "-c", str(ck), "-n", "2",
                        "-o", ""], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1, r.stderr
    assert "not a checkpoint file" in r.stderr
    assert ck.read_bytes() == b"not a checkpoint at all"
