"""The reference GUI's own workload through the drop-in boundary (VERDICT r4 ask 5).

src/bin/main.rs renders a 1600x900 window (:26) with step_by_step::ThreadPoolRenderer::new(scene, 12, 50)
(:229-240): depth 50, 1 spp per redraw, 100 spp after Space (:264).  Each GUI frame calls the non-blocking
render_step (step_by_step.rs:101-121) and gamma-encodes the buffer (:281-289).  This script does the same through
pt_render_start / pt_render_step_rgba8 (non-blocking, display encode on the GPU): per spp setting it times
start_rendering -> the render_step that returns true (the complete buffer), counts the polls, and checks a stratified
pixel set of the finished buffer against the oracle at depth 50.

    python scripts/interactive_bench.py [--scene cornell_box.json] [--reps 3] [--spp 1 100] [--out file.json]

Prints one JSON line per spp setting (and writes them to --out).
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

W, H, DEPTH = 1600, 900, 50  # src/bin/main.rs:26, 229-240


def host_threads(cap=16):
    """The CPUs this process may run on, at most cap (the GPU box grants one GPU's share of the machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(cap, n))


def parity_pixels(w, h, n_grid=32):
    """A grid of pixels plus a full row through the Heart (cornell: y ~ 757/1080 of the frame)."""
    gy = np.linspace(3, h - 4, n_grid).astype(int)
    gx = np.linspace(5, w - 6, n_grid).astype(int)
    grid = (gy[:, None] * w + gx[None, :]).ravel()
    row = (h * 757 // 1080) * w + np.arange(0, w, 4)
    return np.unique(np.concatenate([grid, row])).astype(np.uint32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="cornell_box.json")
    ap.add_argument("--spp", type=int, nargs="+", default=[1, 100])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--display-only", action="store_true",
                    help="poll with the display buffer only (no linear f64 copy per band), as a GUI that only "
                         "shows the frame; parity then compares the RGBA8 bytes with the oracle's encoded pixels")
    ap.add_argument("--out", default=None)
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE", help="renderer option (A/B)")
    a = ap.parse_args()

    import __graft_entry__ as ge
    pt = ge.load_package()
    text = (ROOT / "scenes" / a.scene).read_text()
    scene = pt.Scene.from_json(text, seed=1)
    r = pt.HipRenderer(scene, depth=DEPTH)
    for o in a.option:
        k, v = o.split("=")
        r.set_option(k, int(v))
    cam = scene.camera()
    buf = np.zeros((W * H, 3))
    rgba = np.zeros((W * H, 4), dtype=np.uint8)
    recs = []
    for spp in a.spp:
        # warm-up frame (workspace, streams, code objects)
        r.start_rendering(cam, pt.ImageParams(W, H), spp, seed=a.seed)
        lin = None if a.display_only else buf
        while not r.render_step_rgba8(rgba, lin):
            pass
        times, polls = [], []
        for _ in range(a.reps):
            r.stop_rendering()  # RendererState::render: stop, then start (main.rs:268-271)
            t0 = time.perf_counter()
            r.start_rendering(cam, pt.ImageParams(W, H), spp, seed=a.seed)
            n = 0
            while True:
                n += 1
                if r.render_step_rgba8(rgba, lin):  # non-blocking; the encoded frame of what is done so far
                    break
            times.append(time.perf_counter() - t0)
            polls.append(n)
        samples = W * H * spp
        best = min(times)
        rec = {"workload": "%s %dx%d %dspp depth %d (reference GUI: src/bin/main.rs:26, 229-240, 264)"
                           % (a.scene, W, H, spp, DEPTH),
               "path": "pt_render_start + non-blocking pt_render_step_rgba8 polled until the buffer is complete"
                       + (" (display buffer only)" if a.display_only else " (display and linear buffers)"),
               "ms_to_complete_buffer": [round(t * 1e3, 3) for t in times], "ms_best": round(best * 1e3, 3),
               "msamples_per_s_best": round(samples / best / 1e6, 2), "polls": polls}
        if not a.no_parity:
            import oracle
            px = parity_pixels(W, H)
            osc = oracle.Scene(text, seed=1)
            t = time.perf_counter()
            ref = osc.render(W, H, spp, DEPTH, a.seed, pixels=px, threads=host_threads())
            if a.display_only:  # the RGBA8 bytes against the oracle's pixels through the host encode
                enc_ref = pt.encode_rgba8(np.ascontiguousarray(ref))
                rec["parity"] = {"pixels": int(len(px)),
                                 "rgba8_exact_frac": float(np.mean(np.all(rgba[px] == enc_ref, axis=1))),
                                 "oracle_s": round(time.perf_counter() - t, 1)}
            else:
                got = buf[px]
                rec["parity"] = {"pixels": int(len(px)), "exact_frac": float(np.mean(np.all(got == ref, axis=1))),
                                 "rms": float(np.sqrt(np.mean((got - ref) ** 2))),
                                 "oracle_s": round(time.perf_counter() - t, 1)}
                enc = pt.encode_rgba8(buf)
                rec["parity"]["rgba8_equal_host_encode"] = bool(np.array_equal(enc, rgba))
        recs.append(rec)
        print(json.dumps(rec), flush=True)
    if a.out:
        Path(a.out).write_text("\n".join(json.dumps(x) for x in recs) + "\n")


if __name__ == "__main__":
    main()
