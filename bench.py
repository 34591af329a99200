"""Benchmark: Msamples/s on cornell_box 1920x1080, 256 spp, 8 bounces (BASELINE.json configs[1]).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One step = one full frame (all W*H*spp camera samples, every bounce) rendered
from scene data resident in HBM into an HBM frame buffer.  For N > 1 the
frame's 16x16 tiles are dealt round-robin to the ranks (tile k -> rank k % N),
each rank renders its tiles into a compact shard, the shards are gathered to
rank 0 over RCCL (torch.distributed "nccl") and un-interleaved there: the same
frame at every N ("scaling": "strong").  Rank 0 prints one JSON line.
"""
import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "Msamples/sec cornell_box 1920x1080x256spp at 1/2/4/8 MI355X; RMS pixel delta"
FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector (FMA = 2 FLOP); no-FMA instruction peak is half of it
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: 8 TB/s spec

# FLOPs per event of the kernels' own traversal (counted in pt_device.hpp /
# pt_march.hpp; f64 add/sub/mul/div/sqrt = 1 FLOP, compares, min/max and
# integer ops not counted).  Event counts come from the GPU itself
# (pt_count_work, a diagnostic build of the same device functions) on a pixel
# sample.  The march events run in the wavefront engine's march kernel, the
# rest in its bounce kernel.
FLOP_WEIGHTS = {
    "samples": 31,        # jittered camera ray + normalize (28), accumulate (3)
    "bounces": 11,        # reciprocal direction (3), background on a miss (8)
    "test_sphere": 52,    # inverse transform of the ray (33) + quadratic (19)
    "test_rect": 37, "test_cube": 45,
    "test_march": 64,     # transform (33) + bounding-ellipsoid quadratic (31)
    "node_slabs": 12, "march_slabs": 12,
    "march_steps": 19,    # literal step: t, p adds (4) + heart_f (15)
    "march_tries": 400,   # degree-6 expansion (140), root guess (20), Bernstein prefix
                          # setup + margin (95), ~3 de Casteljau halvings (145)
    "march_blocks": 135,  # exact advance of t, p over ~2.5 binade segments each + heart_f
    "hits": 100,          # object point/normal, normalisations, world transforms
    "lambert": 20, "metal": 25, "dielectric": 40, "reject_tries": 14, "unwind": 3,
}
MARCH_EVENTS = ("test_march", "march_slabs", "march_steps", "march_tries", "march_blocks")


def flops_per_sample(cnt, keys=None):
    keys = FLOP_WEIGHTS if keys is None else keys
    return sum(FLOP_WEIGHTS[k] * cnt[k] for k in keys) / max(1, cnt["samples"])


# BASELINE.json configs[1..4] (configs[0] is the reference's own CPU case):
# scene, width, height, spp.  c2 is the headline (the default); c5's scene is
# generated (scenes/make_scenes.py synthetic(100000)), not a file.
CONFIGS = {
    "c2": ("cornell_box.json", 1920, 1080, 256),
    "c3": ("cornell_box.json", 3840, 2160, 1024),
    "c4": ("cornell_box.json", 3840, 2160, 4096),
    "c5": ("synthetic_100000", 1920, 1080, 256),
}


def scene_text(name):
    if name.startswith("synthetic_"):
        sys.path.insert(0, str(ROOT / "scenes"))
        import make_scenes
        return json.dumps(make_scenes.synthetic(int(name.split("_")[1])))
    return (ROOT / "scenes" / name).read_text()


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", choices=sorted(CONFIGS), default=None,
                    help="a BASELINE.json config (default: c2 through the flags below)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="cornell_box.json")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--scene-seed", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--parity-pixels", type=int, default=48)
    a = ap.parse_args()
    if a.config:
        a.scene, a.width, a.height, a.spp = CONFIGS[a.config]
    return a


def cpu_baseline(text, args, threads):
    """The oracle in the reference's BvhNode mode (the reference threaded
    renderer's algorithm, step_by_step chunking) on a bounded sample: the full
    frame at k spp, k chosen from a probe so the run takes ~cpu_seconds."""
    import numpy as np
    import oracle
    sc = oracle.Scene(text, seed=args.scene_seed).use_bvh(True, 7)
    w, h = args.width, args.height
    px = (np.arange(0, h, 4)[:, None] * w + np.arange(0, w, 4)[None, :]).ravel().astype(np.uint32)
    t = time.perf_counter()
    sc.render(w, h, 1, args.depth, args.seed, pixels=px, threads=threads)
    rate = len(px) / max(1e-9, time.perf_counter() - t)
    spp = int(max(1, min(args.spp, round(args.cpu_seconds * rate / (w * h)))))
    t = time.perf_counter()
    sc.render(w, h, spp, args.depth, args.seed, threads=threads)
    dt = time.perf_counter() - t
    n = w * h * spp
    return {"value": round(n / dt / 1e6, 6), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": "full %dx%d frame at %d spp, depth %d = %d samples in %.1f s (%d threads); oracle "
                      "restatement with the reference's BvhNode traversal" % (w, h, spp, args.depth, n, dt, threads)}


def algorithmic_flops(pt, r, cam, args):
    """F (FLOP/sample) of the kernel's own policy, from its GPU event counters
    on a strided pixel sample (1/144 of the frame) at 4 spp."""
    import numpy as np
    w, h = args.width, args.height
    px = (np.arange(3, h, 12)[:, None] * w + np.arange(5, w, 12)[None, :]).ravel().astype(np.uint32)
    cnt = pt.count_work(r, cam, pt.ImageParams(w, h), 4, px, seed=args.seed)
    return flops_per_sample(cnt), cnt


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print("warning: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world), file=sys.stderr)
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import __graft_entry__ as ge
    pt = ge.load_package()
    text = scene_text(args.scene)
    scene = pt.Scene.from_json(text, seed=args.scene_seed)
    r = pt.HipRenderer(scene, device=local, depth=args.depth)
    cam = scene.camera()
    W, H, spp = args.width, args.height, args.spp
    stream = torch.cuda.Stream()  # a real stream: the HIP events below time exactly our launches
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream

    frame = torch.zeros(W * H * 3, dtype=torch.float64, device="cuda")
    per = pt.shard_tiles(W, H, 0, world)
    if world > 1:
        shard = torch.zeros(per * 256 * 3, dtype=torch.float64, device="cuda")
        gathered = torch.zeros(world * per * 256 * 3, dtype=torch.float64, device="cuda") if rank == 0 else None
        glist = list(gathered.view(world, -1).unbind(0)) if rank == 0 else None
    torch.cuda.synchronize()

    k_start, k_end = [], []

    def step():
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        if world == 1:
            r.render_device(cam, W, H, spp, args.seed, 0, 1, frame.data_ptr(), sp)
        else:
            r.render_device(cam, W, H, spp, args.seed, rank, world, shard.data_ptr(), sp)
        ev1.record(stream)
        k_start.append(ev0)
        k_end.append(ev1)
        if world > 1:
            dist.gather(shard, glist, dst=0)
            if rank == 0:
                pt.unshard_device(gathered.data_ptr(), W, H, world, frame.data_ptr(), sp)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    k_start.clear()
    k_end.clear()
    pt.kernel_timing(r, True)  # per-kernel HIP events on the launch stream, timed steps only
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kt = pt.kernel_timing(r, False)
    kernel_ms = sum(a.elapsed_time(b) for a, b in zip(k_start, k_end)) / max(1, len(k_start))
    if world > 1:
        t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms_max = t.tolist()
    else:
        kernel_ms_max = kernel_ms

    if rank == 0:
        samples_frame = W * H * spp
        value = samples_frame * args.steps / elapsed / 1e6
        img = frame.view(-1, 3).cpu().numpy()
        sys.path.insert(0, str(ROOT / "oracle"))
        threads = min(16, os.cpu_count() or 1)

        # roofline of the dominant kernel, this rank's launches in the timed steps
        F, counts = algorithmic_flops(pt, r, cam, args)
        my_tiles = pt.shard_tiles(W, H, rank, world)
        samples_rank = samples_frame * my_tiles / (pt.shard_tiles(W, H, 0, 1)) * args.steps
        f_kind = {"march": flops_per_sample(counts, MARCH_EVENTS),
                  "bounce": flops_per_sample(counts, [k for k in FLOP_WEIGHTS if k not in MARCH_EVENTS]),
                  "megakernel": F}
        dom = max(("bounce", "march", "megakernel"), key=lambda k: kt[k][0])
        dom_ms, dom_n = kt[dom]
        achieved = f_kind[dom] * samples_rank / (dom_ms / 1e3) / 1e12
        out_bytes = 24.0 * W * H * my_tiles / pt.shard_tiles(W, H, 0, 1)
        rec = {
            "metric": METRIC, "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: re-authored %s, add_random_spheres from seed %d" % (args.scene, args.scene_seed),
            "config": {"workload": "%s %dx%d %dspp depth %d" % (args.scene, W, H, spp, args.depth),
                       "width": W, "height": H, "spp": spp, "depth": args.depth, "seed": args.seed,
                       "parallelism": "tile-interleaved x%d, RCCL gather" % world if world > 1 else "single GPU"},
            "roofline": {"bound": "valu_f64", "achieved": round(achieved, 4), "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved / FP64_PEAK_TFLOPS, 5), "traffic": None,
                         "kernel": "wf_" + dom if dom != "megakernel" else "render_tiles",
                         "flops_per_sample": round(f_kind[dom], 1), "launches": dom_n,
                         "kernel_ms_avg": round(dom_ms / max(1, dom_n), 4),
                         "kernel_ms_by_kind": {k: round(v[0] / args.steps, 3) for k, v in kt.items()},
                         "flops_per_sample_total": round(F, 1),
                         "events_per_sample": {k: round(v / max(1, counts["samples"]), 3)
                                               for k, v in counts.items() if k != "samples"},
                         "frame_kernels_ms": round(kernel_ms, 3), "frame_kernels_ms_max_rank": round(kernel_ms_max, 3),
                         # two chunks run concurrently (pt_wave.hip), so one kernel's launches overlap the
                         # other kind's: the whole path's rate is the frame's FLOPs over the frame time
                         "path_achieved": round(F * value * 1e6 / 1e12, 4),
                         "path_frac": round(F * value * 1e6 / 1e12 / FP64_PEAK_TFLOPS, 5)},
            "roofline_hbm": {"achieved": round(out_bytes / (kernel_ms / 1e3) / 1e9, 4), "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": out_bytes / (kernel_ms / 1e3) / 1e9 / HBM_PEAK_GBS,
                             "bytes_per_launch": out_bytes, "note": "algorithmic: 24 B/pixel frame write"},
        }
        # roofline.traffic: HBM bytes per launch of the same kernel from the committed PMC passes of this
        # workload (scripts/pmc_traffic.py; bench.py cannot read PMC counters itself)
        tfile = ROOT / "profiles" / "r1" / "pmc_traffic_c2.json"
        if tfile.exists():
            tr = json.loads(tfile.read_text())
            kind = tr.get("kinds", {}).get(dom)
            if tr.get("workload") == rec["config"]["workload"] and kind and world == 1:
                rec["roofline"]["traffic"] = round(kind["traffic"])
                rec["roofline"]["traffic_source"] = "profiles/r1/pmc_traffic_c2.json (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE)"
                rec["roofline"]["traffic_gbs"] = round(kind["traffic"] / (dom_ms / max(1, dom_n) / 1e3) / 1e9, 1)
        if not args.no_parity:
            import oracle
            rng = np.random.default_rng(1234)
            px = rng.choice(W * H, size=args.parity_pixels, replace=False).astype(np.uint32)
            sc = oracle.Scene(text, seed=args.scene_seed).use_bvh(True, 7)
            ref = sc.render(W, H, spp, args.depth, args.seed, pixels=px, threads=threads)
            got = img[px]
            rec["rms_vs_oracle"] = float(np.sqrt(np.mean((got - ref) ** 2)))
            rec["rms_pixels"] = int(len(px))
            rec["exact_pixels_frac"] = float(np.mean(np.all(got == ref, axis=1)))
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(text, args, threads)
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
