"""Compile gate: the product sources of the working tree must compile with the Makefile's own flags.

The CPU suite loads the prebuilt library, so on its own it cannot see a source change that no longer compiles
(round 5 shipped such a default build for a few commits).  Here every product source is compiled for gfx950 and the
host with `hipcc -fsyntax-only` (semantic analysis of both sides, every template the kernel launches instantiate:
a few seconds per file), with the FLAGS `make print-flags` reports; and a scratch copy of the sources with one
undefined macro in pt_wave.hip must fail, so the gate is known to bite."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "rs-pathtracing_amd"
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"

pytestmark = pytest.mark.skipif(not Path(HIPCC).exists(), reason="hipcc not installed")


def make_var(target):
    r = subprocess.run(["make", "-s", "-C", str(PKG), target], capture_output=True, text=True, check=True)
    return r.stdout.split()


def syntax_check(src_dir, src):
    flags = make_var("print-flags")
    path = Path(src_dir) / src
    lang = [] if path.suffix == ".hip" else ["-x", "hip"]
    return subprocess.run([HIPCC, *flags, "-fsyntax-only", *lang, str(path)], capture_output=True, text=True,
                          timeout=300)


@pytest.mark.parametrize("src", make_var("print-src") if Path(HIPCC).exists() else [])
def test_product_sources_compile(src):
    r = syntax_check(PKG, src)
    assert r.returncode == 0, r.stderr[-4000:]


def test_gate_rejects_an_undefined_macro(tmp_path):
    """The same check on a scratch copy whose pt_wave.hip uses a macro nothing defines fails."""
    shutil.copytree(PKG / "csrc", tmp_path / "csrc")
    shutil.copytree(ROOT / "include", tmp_path.parent / "include", dirs_exist_ok=True)
    w = tmp_path / "csrc" / "pt_wave.hip"
    w.write_text(w.read_text() + "\nstatic int pt_gate_probe = PT_GATE_UNDEFINED_MACRO;\n")
    r = syntax_check(tmp_path, "csrc/pt_wave.hip")
    assert r.returncode != 0 and "PT_GATE_UNDEFINED_MACRO" in r.stderr
