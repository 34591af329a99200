"""The C-ABI library loads and exports every symbol include/rs_pathtracing.h
declares; host-side entry points behave as specified.  No GPU needed."""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

import oracle as O

ROOT = Path(__file__).resolve().parent.parent


def declared():
    text = (ROOT / "include" / "rs_pathtracing.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pt_[a-z0-9_]+)\s*\(", text)))


def test_header_matches_binding_list(pt):
    assert declared() == sorted(pt.EXPORTS)


def test_library_exports_every_declared_symbol(pt):
    L = C.CDLL(str(pt.LIB_PATH))
    for name in declared():
        assert hasattr(L, name), name


def test_version(pt):
    assert "gfx950" in pt.version()


def test_sample_key_matches_oracle(pt):
    L = O.lib()
    for seed, px, s in [(1, 0, 0), (1, 2073599, 255), (0xDEADBEEF, 12345, 7)]:
        assert pt.sample_key(seed, px, s) == L.or_sample_key(seed, px, s)


def test_shard_tiles(pt):
    w, h = 1920, 1080
    total = 120 * 68
    for world in (1, 2, 3, 8):
        counts = [pt.shard_tiles(w, h, r, world) for r in range(world)]
        assert sum(counts) == total
        assert max(counts) - min(counts) <= 1
    assert pt.shard_tiles(w, h, 3, 2) == 0


def test_encode_rgba8(pt):
    """src/bin/main.rs:281-289: sqrt, clamp [0, 0.999], *256, as u8 (NaN -> 0)."""
    buf = np.array([[0.0, 0.25, 1.0], [4.0, -1.0, np.nan], [0.5, 1e-6, 0.998]])
    out = pt.encode_rgba8(buf)
    want = []
    for r in buf:
        px = []
        for v in r:
            s = np.sqrt(v) if v >= 0 else np.nan
            s = np.nan if np.isnan(s) else min(max(s, 0.0), 0.999)
            px.append(0 if np.isnan(s) else int(s * 256.0))
        want.append(px + [255])
    assert out.tolist() == want


def test_renderer_without_gpu_fails_loudly(pt, cornell_text):
    """No CPU fallback: without a HIP device, creating a renderer is an error."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    sc = pt.Scene.from_json(cornell_text)
    with pytest.raises(pt.PtError) as e:
        pt.HipRenderer(sc, depth=8)
    assert e.value.code == pt.PT_ERR_HIP


# ---- struct layout across the boundary (a 16-byte Rust struct was read as 32) ----

NATIVE = ROOT / "tests" / "native"


def abi_check_bin():
    import fcntl
    import subprocess
    (NATIVE / "_build").mkdir(exist_ok=True)
    with open(NATIVE / "_build" / ".lock", "w") as lk:  # pytest-xdist workers: one make at a time
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", str(NATIVE), "_build/abi_check"], check=True)
    return str(NATIVE / "_build" / "abi_check")


def test_abi_version(pt):
    assert pt.lib().pt_abi_version() == pt.ABI_VERSION == 4


@pytest.mark.parametrize("which", [0, 1, 2, 3, 4, 5])
def test_abi_layout_matches_ctypes(pt, which):
    """pt_abi_layout (the library's own sizeof / offsetof) == the ctypes mirror."""
    S = pt.ABI_STRUCTS[which]
    assert pt.abi_layout(which) == [C.sizeof(S)] + [getattr(S, f[0]).offset for f in S._fields_]


def test_abi_layout_unknown_struct(pt):
    with pytest.raises(pt.PtError) as e:
        pt.abi_layout(99)
    assert e.value.code == pt.PT_ERR_INVALID


def test_plain_c_caller_layout():
    """A gcc-compiled C program, header only: every struct's sizeof / offsetof
    as C lays it out equals the library's."""
    import subprocess
    out = subprocess.run([abi_check_bin(), "layout"], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    assert out.stdout.count("match") == 6


def test_legacy_opts_are_not_read_past():
    """A 0.1.0 caller's 16-byte pt_scene_opts (`reserved` = 0 where struct_size
    sits now) placed against an unreadable page loads the scene (with an
    ImageTexture) without touching the page; a 0.2.0 caller's 32-byte struct
    (struct_size 0, a loader set) loads it without calling the loader (0 cannot
    tell the two apart, ADVICE r4: ABI 4); the current struct calls its loader;
    a 16-byte struct (struct_size 16) loads without touching the page;
    struct_size 8 is refused (no silent fallback for old callers)."""
    import subprocess
    out = subprocess.run([abi_check_bin(), "legacy", "scenes/textured.json"], capture_output=True, text=True,
                         cwd=str(ROOT))
    assert out.returncode == 0, (out.returncode, out.stderr)
    assert "struct_size 8 refused" in out.stdout
    assert "0.1.0 opts" in out.stdout and "loader not called" in out.stdout
    assert "loader called" in out.stdout and "16-byte opts" in out.stdout


def test_opts_struct_size_from_python(pt, cornell_text):
    raw = cornell_text.encode()
    L = pt.lib()
    for size, ok in [(0, True), (16, True), (24, True), (32, True), (64, True), (8, False), (15, False)]:
        o = pt.SceneOpts(0, size, 3)
        h = C.c_void_p()
        rc = L.pt_scene_create_from_json(raw, len(raw), C.byref(o), C.byref(h))
        assert (rc == 0) == ok, (size, rc)
        if rc == 0:
            assert L.pt_scene_num_shapes(h) == 9  # random_spheres = 0
            L.pt_scene_destroy(h)


def test_plain_c_caller_checkpoint(tmp_path):
    """The C caller writes a checkpoint of a 2-rank shard and reads it back
    bit for bit; a flipped byte fails the checksum with PT_ERR_IO and zeroed sums."""
    import subprocess
    out = subprocess.run([abi_check_bin(), "checkpoint", str(tmp_path / "f.ckpt")], capture_output=True, text=True)
    assert out.returncode == 0, (out.returncode, out.stderr)
    assert "checkpoint round trip" in out.stdout and "corrupt file refused" in out.stdout


def test_option_names_match_the_python_defaults(pt):
    """Every tuning knob the library names (pt_option_name) has a default in the Python mirror and vice versa
    (no GPU needed)."""
    assert set(pt.option_names()) == set(pt.OPTION_DEFAULTS)
