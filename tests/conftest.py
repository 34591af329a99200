import importlib.util
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT))


def load_package():
    """Import rs-pathtracing_amd/ (hyphenated dir) as `rs_pathtracing_amd`."""
    if "rs_pathtracing_amd" in sys.modules:
        return sys.modules["rs_pathtracing_amd"]
    pkg = ROOT / "rs-pathtracing_amd"
    spec = importlib.util.spec_from_file_location("rs_pathtracing_amd", pkg / "__init__.py",
                                                  submodule_search_locations=[str(pkg)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["rs_pathtracing_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session")
def pt():
    return load_package()


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    return oracle


# the host builds of tests/native: _build, or the sanitizer build _build_san (scripts/san.sh sets PT_NATIVE_BUILD)
NATIVE_BUILD = ROOT / "tests" / "native" / __import__("os").environ.get("PT_NATIVE_BUILD", "_build")


def native_lib(name):
    return str(NATIVE_BUILD / name)


def scene_text(name):
    return (ROOT / "scenes" / name).read_text()


@pytest.fixture(scope="session")
def cornell_text():
    return scene_text("cornell_box.json")


@pytest.fixture(scope="session")
def spheres_text():
    return scene_text("spheres.json")


def host_threads(cap=16):
    """Oracle threads: the CPUs this process may run on, at most `cap` (the GPU
    box shows the whole machine in os.cpu_count() but grants one GPU's share)."""
    import os
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(cap, n))
