"""Work counts of the device walk compiled for the host (tests/native libpath.so, h_count_work): BVH node tests,
sphere tests and bounces per sample on C5's synthetic field and on cornell, for comparing BVH builds on the CPU
before a GPU A/B (profiles/r4/ab_round4_experiments.txt r4n).

    python scripts/bvh_count.py [libpath.so ...]     (default: tests/native/_build/libpath.so)
"""
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "scenes"))
import make_scenes  # noqa: E402

COUNTERS = ["samples", "bounces", "test_sphere", "test_rect", "test_cube", "test_march", "node_slabs",
            "march_slabs", "march_steps", "march_tries", "march_blocks", "hits", "lambert", "metal",
            "dielectric", "reject_tries", "unwind", "test_torus", "march_guard"]


def counts(lib, text, w=1920, h=1080, n=6000, spp=2, depth=8):
    L = C.CDLL(str(lib))
    L.h_scene_new.restype = C.c_void_p
    L.h_scene_new.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_uint64]
    L.h_count_work.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64,
                               C.POINTER(C.c_uint32), C.c_size_t, C.POINTER(C.c_uint64)]
    L.h_scene_free.argtypes = [C.c_void_p]
    raw = text.encode()
    hd = L.h_scene_new(raw, len(raw), 1, 1)
    px = np.random.default_rng(5).choice(w * h, n, replace=False).astype(np.uint32)
    out = (C.c_uint64 * len(COUNTERS))()
    L.h_count_work(hd, w, h, spp, depth, 1, px.ctypes.data_as(C.POINTER(C.c_uint32)), len(px), out)
    L.h_scene_free(hd)
    d = dict(zip(COUNTERS, list(out)))
    return {k: round(d[k] / d["samples"], 3) for k in ("bounces", "node_slabs", "test_sphere", "test_rect",
                                                         "test_cube")}


def main():
    libs = sys.argv[1:] or [str(ROOT / "tests" / "native" / "_build" / "libpath.so")]
    scenes = {"c5 synthetic_100000": json.dumps(make_scenes.synthetic(100000)),
              "c2 cornell_box": (ROOT / "scenes" / "cornell_box.json").read_text()}
    for name, text in scenes.items():
        for lib in libs:
            print(name, lib, counts(lib, text))


if __name__ == "__main__":
    main()
