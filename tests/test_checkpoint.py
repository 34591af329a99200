"""Checkpoint files of resumable frames (pt_checkpoint_save / pt_checkpoint_load,
rs-pathtracing_amd/csrc/pt_checkpoint.cpp).  The reference has no checkpoint
(Renderer::render runs a frame in one go, src/renderer/mod.rs:67-114); SURVEY
§5 names checkpoint / resume as the hot path's auxiliary subsystem.  Host code
only: the GPU side (sample windows resumed from these files) is
tests/test_gpu_resume.py."""
import ctypes as C

import numpy as np
import pytest


def header(pt, w=64, h=40, rank=0, world=1, done=8, spp=32):
    return dict(width=w, height=h, samples_number=spp, samples_done=done, seed=5, depth=50, scene_key=0xabc,
                rank=rank, world=world)


@pytest.mark.parametrize("rank,world", [(0, 1), (0, 2), (1, 2), (5, 8)])
def test_round_trip_is_bit_exact(pt, tmp_path, rank, world):
    hd = header(pt, w=200, h=120, rank=rank, world=world)
    n = pt.checkpoint_count(200, 120, rank, world)
    rng = np.random.default_rng(rank + 10 * world)
    sums = rng.standard_normal(n) * 1e3
    sums[:6] = [0.0, -0.0, np.inf, -np.inf, 5e-324, np.nan]  # every bit pattern survives
    path = tmp_path / "frame.ckpt"
    pt.save_checkpoint(path, sums, **hd)
    got, back = pt.load_checkpoint(path)
    assert back.view(np.uint64).tolist() == sums.view(np.uint64).tolist()
    for k, v in hd.items():
        assert got[k] == v
    assert got["count"] == n and got["reserved"] == 0
    assert path.stat().st_size == 8 + 56 + 8 * n + 8
    assert [p.name for p in tmp_path.iterdir()] == ["frame.ckpt"]  # the temporary was renamed away


def test_save_overwrites_atomically(pt, tmp_path):
    path = tmp_path / "f.ckpt"
    n = pt.checkpoint_count(64, 40)
    pt.save_checkpoint(path, np.zeros(n), **header(pt, done=4))
    pt.save_checkpoint(path, np.ones(n), **header(pt, done=12))
    got, sums = pt.load_checkpoint(path)
    assert got["samples_done"] == 12 and np.all(sums == 1.0)


@pytest.mark.parametrize("change", ["done_past_spp", "rank_ge_world", "count", "empty", "world0"])
def test_inconsistent_header_is_refused(pt, tmp_path, change):
    hd = header(pt)
    n = pt.checkpoint_count(64, 40)
    if change == "done_past_spp":
        hd["samples_done"] = 33
    elif change == "rank_ge_world":
        hd["rank"], hd["world"] = 2, 2
    elif change == "count":
        n -= 3
    elif change == "empty":
        hd["width"] = 0
    elif change == "world0":
        hd["world"] = 0
    with pytest.raises(pt.PtError) as e:
        pt.save_checkpoint(tmp_path / "x.ckpt", np.zeros(max(n, 1)), **hd)
    assert e.value.code == pt.PT_ERR_INVALID
    assert not (tmp_path / "x.ckpt").exists()


def corrupt(path, fn):
    raw = bytearray(path.read_bytes())
    path.write_bytes(bytes(fn(raw)))


def _flip(at):
    def f(raw):
        raw[at] ^= 0x40
        return raw
    return f


@pytest.mark.parametrize("how", ["truncated", "longer", "magic", "sum_byte", "checksum", "header_key",
                                 "header_count", "empty_file"])
def test_corrupt_files_fail_with_io_status(pt, tmp_path, how):
    path = tmp_path / "f.ckpt"
    n = pt.checkpoint_count(64, 40)
    pt.save_checkpoint(path, np.arange(n, dtype=np.float64), **header(pt))
    size = path.stat().st_size
    fn = {"truncated": lambda r: r[:-9], "longer": lambda r: r + b"\0" * 8, "magic": _flip(2),
          "sum_byte": _flip(64 + 8 * 17 + 5), "checksum": _flip(size - 1), "header_key": _flip(8 + 40),
          "header_count": _flip(8 + 48), "empty_file": lambda r: b""}[how]
    corrupt(path, fn)
    with pytest.raises(pt.PtError) as e:
        pt.load_checkpoint(path)
    assert e.value.code == pt.PT_ERR_IO, str(e.value)


def test_checksum_failure_zeroes_the_sums(pt, tmp_path):
    path = tmp_path / "f.ckpt"
    n = pt.checkpoint_count(64, 40)
    pt.save_checkpoint(path, np.full(n, 2.5), **header(pt))
    corrupt(path, _flip(64 + 8 * 3))
    c = pt.CheckpointStruct()
    buf = np.full(n, 7.0)
    rc = pt.lib().pt_checkpoint_load(str(path).encode(), C.byref(c), buf.ctypes.data_as(C.POINTER(C.c_double)), n)
    assert rc == pt.PT_ERR_IO and np.all(buf == 0.0)


def test_small_buffer_and_missing_file(pt, tmp_path):
    path = tmp_path / "f.ckpt"
    n = pt.checkpoint_count(64, 40)
    pt.save_checkpoint(path, np.zeros(n), **header(pt))
    c = pt.CheckpointStruct()
    buf = np.zeros(n - 1)
    rc = pt.lib().pt_checkpoint_load(str(path).encode(), C.byref(c), buf.ctypes.data_as(C.POINTER(C.c_double)),
                                     n - 1)
    assert rc == pt.PT_ERR_INVALID
    with pytest.raises(pt.PtError) as e:
        pt.load_checkpoint(tmp_path / "nope.ckpt")
    assert e.value.code == pt.PT_ERR_IO
    hd, sums = pt.load_checkpoint(path, with_sums=False)  # header only
    assert sums is None and hd["count"] == n


def test_frame_key_names_scene_camera_and_depth(pt, cornell_text):
    sc = pt.Scene.from_json(cornell_text, seed=1)
    cam = sc.camera()
    raw = cornell_text.encode()
    k = pt.frame_key(raw, cam, 50)
    assert k == pt.frame_key(raw, cam, 50)
    assert k != pt.frame_key(raw, cam, 8)
    assert k != pt.frame_key(raw + b" ", cam, 50)
    assert k != pt.frame_key(raw, cam, 50, scene_seed=2)
    moved = pt.Camera.new([0.0, 1.0, 2.0], [0.0, 0.0, -1.0], [0.0, 1.0, 0.0], 1.0, 0.5)
    assert k != pt.frame_key(raw, moved, 50)
