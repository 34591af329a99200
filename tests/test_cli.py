"""tools/pt_render, the headless CLI over the C-ABI (the reference binaries' `scene [spp [w h]]` arguments,
src/bin/main_raylib.rs:22-41): argument errors, unreadable and malformed scenes, and no CPU fallback.  Host
only; the GPU renders (one go, interrupted and resumed) are tests/test_gpu_resume.py."""
import subprocess

import pytest

from conftest import ROOT

EXE = ROOT / "tools" / "pt_render"


@pytest.fixture(scope="module")
def exe():
    import fcntl
    with open(ROOT / "tools" / ".build.lock", "w") as lk:  # pytest-xdist workers: one make at a time
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", str(ROOT / "tools"), "pt_render"], check=True)
    return str(EXE)


def run(exe, *args):
    return subprocess.run([exe, *args], capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize("args", [[], ["a.json", "4", "64"], ["a.json", "1", "2", "3", "4"], ["a.json", "-q"],
                                  ["a.json", "-d"], ["a.json", "-c", "x.ckpt"]])
def test_usage_errors(exe, args):
    r = run(exe, *args)
    assert r.returncode == 2 and "usage" in r.stderr


def test_unreadable_and_malformed_scenes(exe, tmp_path):
    r = run(exe, str(tmp_path / "missing.json"))
    assert r.returncode == 1 and "cannot read" in r.stderr
    bad = tmp_path / "bad.json"
    bad.write_text('{"camera": ')
    r = run(exe, str(bad), "1", "8", "8")
    assert r.returncode == 1 and "status -2" in r.stderr  # PT_ERR_PARSE, serde_json's error in the reference


def test_no_cpu_fallback(exe, tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    r = run(exe, str(ROOT / "scenes" / "cornell_box.json"), "1", "8", "8", "-o", str(tmp_path / "x.png"))
    assert r.returncode == 1 and "status -4" in r.stderr  # PT_ERR_HIP
    assert not (tmp_path / "x.png").exists()
