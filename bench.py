"""Benchmark: Msamples/s on cornell_box 1920x1080, 256 spp, 8 bounces (BASELINE.json configs[1]).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c1|c2|c3|c4|c5]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
    python bench.py --gpus N --single-process      # N devices behind one pt_renderer_create_multi

A plain `python bench.py --gpus N` (N > 1, no WORLD_SIZE in the environment)
starts `python -m torch.distributed.run --nproc-per-node N ... bench.py ...`
as a child process (this process never touches the GPU) and exits with its
exit code; rank 0 prints the JSON line.  With the nccl backend and fewer than
N visible devices it exits non-zero, naming the device count: one rank per GPU
(the reference's parallelism knob takes effect however the renderer is
started, ThreadPoolRenderer::new(scene, thread_number, depth),
src/renderer/step_by_step.rs:37).

One step = one full frame (all W*H*spp camera samples, every bounce) rendered
from scene data resident in HBM into an HBM frame buffer.  For N > 1 the
frame's 16x16 tiles are dealt round-robin to the ranks (tile k -> rank k % N),
each rank renders its tiles into a compact shard, the shards are gathered to
rank 0 over RCCL (torch.distributed "nccl") and un-interleaved there: the same
frame at every N ("scaling": "strong").  Rank 0 prints one JSON line.

After the timed steps (not part of `value`):
* roofline: one more frame with one chunk stream (wf_slots = 1), so every
  render kernel runs alone and its HIP-event launch durations are its own; the
  dominant kernel's algorithmic FLOPs per launch / its mean launch duration.
  The timed steps run two chunk streams, whose kernels overlap (their summed
  durations exceed the frame time), so the whole path's rate is reported too.
* parity: >= 8192 stratified pixels (a 16-pixel grid plus a full row and a full
  column through the Heart) against the oracle at the full spp;
* cpu_baseline: the oracle in the reference's BvhNode mode, on the host's
  cores (this process's CPU share) and on the reference's 12 threads.
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
FP32_PEAK_TFLOPS = 157.3  # MI355X FP32 vector (MI355X_MICROARCH.md)
BIG_BVH_NODES = 1 << 15   # pt_types.hpp: from this many nodes per layout the bounce's node slab test is f32
REF_THREADS = 12          # the reference GUI's ThreadPoolRenderer::new(scene, 12, 50) (src/bin/main.rs:229-239)

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
# the trace's events: in the bounce kernel, or in wf_walk for the large-tree scenes without marched shapes
WALK_EVENTS = ("test_sphere", "test_rect", "test_cube", "node_slabs")


def f32_node_flops_per_sample(counts):
    """f32 FLOPs per sample of the large-tree bounce's node slabs: six f32 FMAs (12 FLOPs) per node
    test.  The event counters come from the STATS build of the walk, which tests the root; the large-tree walk
    starts inside it, one node test fewer per trace (a trace is a `bounces` event)."""
    return 12.0 * max(0, counts["node_slabs"] - counts["bounces"]) / max(1, counts["samples"])


def kt_src_has_bounce(src):
    return src.get("bounce", (0, 0))[1] > 0


def node_kernel(src):
    """The kernel kind that tests the BVH nodes: wf_walk when it ran, else the bounce kernel."""
    return "walk" if src.get("walk", (0, 0))[1] > 0 else "bounce"


def flops_per_sample(cnt, keys=None):
    keys = FLOP_WEIGHTS if keys is None else keys
    return sum(FLOP_WEIGHTS[k] * cnt[k] for k in keys) / max(1, cnt["samples"])


# BASELINE.json configs: scene, width, height, spp.  c1 is the reference's own
# CPU-runnable case (spheres.json, the GUI's scene), c2 the headline (the
# default); c5's scene is generated (scenes/make_scenes.py synthetic(100000)).
CONFIGS = {
    "c1": ("spheres.json", 256, 256, 16),
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
    ap.add_argument("--slots", type=int, default=None, help="chunk streams in flight (renderer default: 2)")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="a renderer tuning option (pt_renderer_set_option), repeatable")
    ap.add_argument("--single-process", action="store_true",
                    help="N GPUs behind one renderer (pt_renderer_create_multi, peer-copy gather) instead of ranks")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="ranks' process group: nccl (= RCCL, the multi-GPU default) or gloo (rehearsal: shards "
                         "gathered through host memory, ranks may share a GPU)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target length of each CPU-baseline run")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-roofline-leg", action="store_true", help="skip the one-stream roofline frame")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="skip the frame with per-kernel HIP events after the timed steps (profiler runs)")
    ap.add_argument("--parity-pixels", type=int, default=0,
                    help="0: the stratified set (>= 8192 pixels); n: n random pixels")
    a = ap.parse_args()
    if a.config:
        a.scene, a.width, a.height, a.spp = CONFIGS[a.config]
    return a


def launch_plan(args, env):
    """How this invocation runs: "ranks" (it is a rank of a torch.distributed launch: WORLD_SIZE is set),
    "spawn" (--gpus N > 1 with no launcher: start one as a child), "single-process" (N devices behind one
    pt_renderer_create_multi) or "one" (one GPU)."""
    if "WORLD_SIZE" in env:
        return "ranks"
    if args.gpus > 1:
        return "single-process" if args.single_process else "spawn"
    return "one"


def device_topology(infos, backend, comm_size):
    """What the ranks of a multi-rank bench ran on: each rank's LOCAL_RANK, device ordinal, PCI address and UUID
    (gathered to every rank), the backend and the communicator size, and the groups of ranks that shared one
    physical device (the same PCI address and UUID)."""
    by_dev = {}  # one physical device: the same PCI address and the same UUID (either alone could be blank)
    for i in infos:
        by_dev.setdefault((i.get("pci"), i.get("uuid")), []).append(i["rank"])
    shared = sorted(sorted(v) for v in by_dev.values() if len(v) > 1)
    return {"backend": backend, "comm_size": comm_size, "ranks": sorted(infos, key=lambda i: i["rank"]),
            "distinct_devices": len(by_dev), "shared_devices": shared}


def topology_refusal(topo):
    """Under nccl (RCCL) every rank must own its GPU: a bench line whose ranks shared one would not measure N
    GPUs.  None when the topology is acceptable; gloo rehearsals may share the box's GPU."""
    if topo["backend"] == "nccl" and topo["shared_devices"]:
        return ("bench.py: %d ranks over nccl (RCCL) but only %d distinct GPUs: ranks %s share a device"
                % (topo["comm_size"], topo["distinct_devices"], topo["shared_devices"]))
    if topo["comm_size"] != len(topo["ranks"]):
        return "bench.py: communicator size %d but %d ranks reported" % (topo["comm_size"], len(topo["ranks"]))
    return None


def device_identity(torch, ordinal):
    p = torch.cuda.get_device_properties(ordinal)
    return {"device": ordinal, "name": p.name,
            "pci": "%04x:%02x:%02x" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id), "uuid": str(p.uuid)}


def device_shortfall(world, backend, ndev):
    """The error for `world` ranks on `ndev` visible devices, or None: RCCL needs one GPU per rank; gloo ranks may
    share one (a rehearsal of the rank path)."""
    if backend == "nccl" and world > ndev:
        return ("bench.py: %d ranks over nccl (RCCL) need %d GPUs, but %d device%s visible"
                % (world, world, ndev, " is" if ndev == 1 else "s are"))
    if ndev < 1:
        return "bench.py: no GPU visible"
    return None


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args, argv):
    """Runs this bench as N ranks under torch.distributed.run in a child process (no exec: this process has not
    touched the GPU, and the child is a new program) and returns the child's exit code."""
    import subprocess
    import torch
    err = device_shortfall(args.gpus, args.dist_backend, torch.cuda.device_count())  # counting does not init HIP
    if err:
        print(err, file=sys.stderr, flush=True)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(ROOT / "bench.py")] + list(argv)
    print("bench.py: launching %d ranks: %s" % (args.gpus, " ".join(cmd)), file=sys.stderr, flush=True)
    return subprocess.run(cmd).returncode


def finite_or_null(x):
    """The record with every non-finite float as null (strict JSON; a profiler pass without timing frames has no
    per-kernel times, so its roofline fields are NaN)."""
    if isinstance(x, float):
        return x if math.isfinite(x) else None
    if isinstance(x, dict):
        return {k: finite_or_null(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [finite_or_null(v) for v in x]
    return x


def metric_name(args):
    if (args.scene, args.width, args.height, args.spp, args.depth) == ("cornell_box.json", 1920, 1080, 256, 8):
        return METRIC
    return "Msamples/sec %s %dx%dx%dspp depth %d" % (args.scene.replace(".json", ""), args.width, args.height,
                                                    args.spp, args.depth)


def host_cpus():
    """The host's CPUs as this process sees them: the model, nproc, the affinity
    mask, a cgroup CPU quota and OMP_NUM_THREADS; `share` is the smallest, the
    threads the CPU baseline may use (the GPU box grants one GPU's share of a
    machine whose os.cpu_count() shows every CPU)."""
    info = {"nproc": os.cpu_count() or 1}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity"] = info["nproc"]
    try:
        q = Path("/sys/fs/cgroup/cpu.max").read_text().split()
        info["cgroup_cpus"] = None if q[0] == "max" else round(int(q[0]) / int(q[1]), 2)
    except (OSError, ValueError, IndexError):
        info["cgroup_cpus"] = None
    omp = os.environ.get("OMP_NUM_THREADS")
    info["omp_num_threads"] = int(omp) if omp and omp.isdigit() else None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    cands = [info["affinity"]] + [int(v) for v in (info["cgroup_cpus"], info["omp_num_threads"]) if v]
    info["share"] = max(1, min(cands))
    return info


def time_oracle(sc, args, threads):
    """Full frames at k spp, k from a probe so the run takes ~cpu_seconds."""
    import numpy as np
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
    return n / dt / 1e6, spp, n, dt


def cpu_baseline(text, args):
    """The oracle in the reference's BvhNode mode (the reference threaded
    renderer's algorithm, step_by_step chunking, src/renderer/mod.rs:66-125) on
    a bounded sample: the full frame at k spp.  Timed on this process's CPU
    share and on the reference GUI's 12 threads."""
    import oracle
    host = host_cpus()
    sc = oracle.Scene(text, seed=args.scene_seed).use_bvh(True, 7)
    v, spp, n, dt = time_oracle(sc, args, host["share"])
    v12, spp12, n12, dt12 = time_oracle(sc, args, REF_THREADS)
    what = "oracle restatement with the reference's BvhNode traversal"
    return {"value": round(v, 6), "unit": "Msamples/s", "cores": host["share"], "kind": "port",
            "sample": "full %dx%d frame at %d spp, depth %d = %d samples in %.1f s (%d threads); %s"
                      % (args.width, args.height, spp, args.depth, n, dt, host["share"], what),
            "ref_threads": {"value": round(v12, 6), "cores": REF_THREADS,
                            "sample": "full frame at %d spp = %d samples in %.1f s (12 threads, the reference GUI's)"
                                      % (spp12, n12, dt12)},
            "host": host}


def algorithmic_flops(pt, r, cam, args):
    """F (FLOP/sample) of the kernel's own policy, from its GPU event counters
    on a strided pixel sample (1/144 of the frame) at 4 spp."""
    import numpy as np
    w, h = args.width, args.height
    px = (np.arange(3, h, 12)[:, None] * w + np.arange(5, w, 12)[None, :]).ravel().astype(np.uint32)
    cnt = pt.count_work(r, cam, pt.ImageParams(w, h), 4, px, seed=args.seed)
    return flops_per_sample(cnt), cnt


def parity_pixels(args):
    """A 16-pixel grid over the frame plus a full row and a full column through
    the Heart (cornell's heaviest rays: y ~ 757/1080, x ~ 1142/1920 of the
    frame), or n random pixels."""
    import numpy as np
    W, H = args.width, args.height
    if args.parity_pixels:
        rng = np.random.default_rng(1234)
        return rng.choice(W * H, size=min(args.parity_pixels, W * H), replace=False).astype(np.uint32)
    grid = (np.arange(7, H, 16)[:, None] * W + np.arange(7, W, 16)[None, :]).ravel()
    yr, xc = min(H - 1, H * 757 // 1080), min(W - 1, W * 1142 // 1920)
    row = yr * W + np.arange(W)
    col = np.arange(H) * W + xc
    return np.unique(np.concatenate([grid, row, col])).astype(np.uint32)


ROUNDS = ("r6", "r5", "r4", "r3", "r2", "r1")  # profiles/<round>/, newest first


def parse_workload(w):
    """"cornell_box.json 1920x1080 256spp depth 8" -> (scene, width, height, spp, depth), or None."""
    import re
    m = re.fullmatch(r"(\S+) (\d+)x(\d+) (\d+)spp depth (\d+)", w or "")
    return (m.group(1), int(m.group(2)), int(m.group(3)), int(m.group(4)), int(m.group(5))) if m else None


def pmc_lookup(what, scene, depth, width, height, spp, source, root=ROOT):
    """A committed PMC result (profiles/rN/pmc_<what>_*.json, what = flops | traffic) for this scene and depth,
    collected on this build (its source_id == the loaded library's).  FLOPs and HBM bytes per sample depend on
    the scene, the depth and the machine code, not on the frame size or spp: every sample runs the same path
    (trace_pixel_samples, src/renderer/mod.rs:151-155), and the chunked engine's bytes per path-bounce do not
    depend on how many chunks a frame has (measured: C2 and C3 agree within 0.1 %).  So a pass of any resolution
    and spp of the same (scene, depth, build) serves every config: the exact workload first, then the newest
    round.  Returns (path, record, samples_per_frame_of_the_pass, why_not)."""
    found, builds = [], set()
    for rank, rnd in enumerate(ROUNDS):
        d = root / "profiles" / rnd
        if not d.is_dir():
            continue
        for f in sorted(d.glob("pmc_%s_*.json" % what)):
            try:
                rec = json.loads(f.read_text())
            except (OSError, ValueError):
                continue
            wl = parse_workload(rec.get("workload"))
            if not wl or (wl[0], wl[4]) != (scene, depth):
                continue
            builds.add(rec.get("source_id"))
            if rec.get("source_id") != source:
                continue
            exact = (wl[1], wl[2], wl[3]) == (width, height, spp)
            found.append((not exact, rank, f, rec, float(rec.get("samples_per_frame") or wl[1] * wl[2] * wl[3])))
    if not found:
        why = ("no committed pmc_%s file for %s depth %d" % (what, scene, depth) if not builds else
               "pmc_%s files for %s depth %d were collected on build(s) %s, this is %s"
               % (what, scene, depth, ", ".join(sorted(str(b) for b in builds)), source))
        return None, None, None, why
    found.sort(key=lambda c: (c[0], c[1]))
    _, _, f, rec, spf = found[0]
    return f, rec, spf, None


def main():
    args = parse()
    if launch_plan(args, os.environ) == "spawn":
        sys.exit(spawn_ranks(args, sys.argv[1:]))
    if os.environ.get("PT_SEGV_LOG"):  # diagnostics: a host fault's address, registers and mappings to a file
        import ctypes
        ctypes.CDLL(str(ROOT / "tools" / "segv_maps.so")).pt_segv_install(os.environ["PT_SEGV_LOG"].encode())
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    multi = args.single_process and world == 1 and args.gpus > 1
    if world != args.gpus and rank == 0 and not multi:
        print("warning: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (args.gpus, world), file=sys.stderr)
    gloo = world > 1 and args.dist_backend == "gloo"
    err = device_shortfall(world, args.dist_backend, torch.cuda.device_count()) if world > 1 else None
    if err:
        if rank == 0:
            print(err, file=sys.stderr, flush=True)
        sys.exit(2)
    if gloo:  # rehearsal of the multi-rank path on fewer GPUs than ranks
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    topo = None
    if world > 1:  # which physical GPU each rank renders on, as every rank sees it
        mine = dict(device_identity(torch, local), rank=rank, local_rank=int(os.environ.get("LOCAL_RANK", "0")))
        infos = [None] * world
        dist.all_gather_object(infos, mine)
        topo = device_topology(infos, "gloo" if gloo else "nccl", dist.get_world_size())
        why = topology_refusal(topo)
        if why:
            if rank == 0:
                print(why, file=sys.stderr, flush=True)
            sys.exit(3)

    import __graft_entry__ as ge
    pt = ge.load_package()
    text = scene_text(args.scene)
    scene = pt.Scene.from_json(text, seed=args.scene_seed)
    if multi:
        r = pt.HipRenderer(scene, depth=args.depth, devices=list(range(args.gpus)))
    else:
        r = pt.HipRenderer(scene, device=local, depth=args.depth)
    if args.slots:
        r.set_option("wf_slots", args.slots)
    for o in args.option:
        k, v = o.split("=", 1)
        r.set_option(k, int(v))
    slots = r.get_option("wf_slots")
    cam = scene.camera()
    W, H, spp = args.width, args.height, args.spp
    stream = torch.cuda.Stream()  # a real stream: the HIP events below time exactly our launches
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    n_gpus = args.gpus if multi else world

    frame = torch.zeros(W * H * 3, dtype=torch.float64, device="cuda")
    per = pt.shard_tiles(W, H, 0, world)
    if world > 1:
        shard = torch.zeros(per * 256 * 3, dtype=torch.float64, device="cuda")
        gathered = torch.zeros(world * per * 256 * 3, dtype=torch.float64, device="cuda") if rank == 0 else None
        if gloo:  # gloo gathers host tensors
            shard_h = torch.zeros(shard.numel(), dtype=torch.float64)
            gathered_h = torch.zeros(gathered.numel(), dtype=torch.float64) if rank == 0 else None
        g = gathered_h if gloo else gathered
        glist = list(g.view(world, -1).unbind(0)) if rank == 0 else None
    torch.cuda.synchronize()

    k_start, k_end = [], []
    g_start, g_end = [], []  # the gather + unshard of each step (world > 1), on rank 0's clock

    def step():
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        if multi:
            r.render_frame_device(cam, W, H, spp, args.seed, frame.data_ptr(), sp)
        elif world == 1:
            r.render_device(cam, W, H, spp, args.seed, 0, 1, frame.data_ptr(), sp)
        else:
            r.render_device(cam, W, H, spp, args.seed, rank, world, shard.data_ptr(), sp)
        ev1.record(stream)
        k_start.append(ev0)
        k_end.append(ev1)
        if world > 1:
            gv0, gv1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            gv0.record(stream)
            if gloo:
                shard_h.copy_(shard)  # synchronous D2H on the render stream
                dist.gather(shard_h, glist, dst=0)
                if rank == 0:
                    gathered.copy_(gathered_h)
            else:
                dist.gather(shard, glist, dst=0)
            if rank == 0:
                pt.unshard_device(gathered.data_ptr(), W, H, world, frame.data_ptr(), sp, device=local)
            gv1.record(stream)
            g_start.append(gv0)
            g_end.append(gv1)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    pt.march_guard_drops(r)  # clear
    k_start.clear()
    k_end.clear()
    g_start.clear()
    g_end.clear()
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
    guard_drops = pt.march_guard_drops(r)
    kernel_ms = sum(a.elapsed_time(b) for a, b in zip(k_start, k_end)) / max(1, len(k_start))
    gather_ms = sum(a.elapsed_time(b) for a, b in zip(g_start, g_end)) / max(1, len(g_start))
    # parity is checked on the last timed frame (the one behind `value`): copy it out before the frames below
    img = frame.view(-1, 3).cpu().numpy() if rank == 0 else None
    # per-kernel launch durations: one more frame of the same workload with HIP events around every launch, after
    # the timed region (the events' marker packets would add gaps between a small frame's ~50 dependent launches)
    kt = {}
    if not args.no_kernel_timing:
        pt.kernel_timing(r, True)
        step()
        torch.cuda.synchronize()
        kt = pt.kernel_timing(r, False)
    if world > 1:
        t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device="cpu" if gloo else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms_max = t.tolist()
    else:
        kernel_ms_max = kernel_ms

    # roofline leg: one frame with every render kernel alone on the device (one chunk stream)
    kt_iso = None
    if not args.no_roofline_leg:
        r.set_option("wf_slots", 1)
        pt.kernel_timing(r, True)
        if multi:
            r.render_frame_device(cam, W, H, spp, args.seed, frame.data_ptr(), sp)
        else:
            r.render_device(cam, W, H, spp, args.seed, rank, world, (shard if world > 1 else frame).data_ptr(), sp)
        torch.cuda.synchronize()
        kt_iso = pt.kernel_timing(r, False)
        r.set_option("wf_slots", slots)

    if rank == 0:
        samples_frame = W * H * spp
        value = samples_frame * args.steps / elapsed / 1e6
        sys.path.insert(0, str(ROOT / "oracle"))

        # roofline of the dominant kernel (this rank's / the first device's launches)
        F, counts = algorithmic_flops(pt, r, cam, args)
        share = 1.0 if multi else pt.shard_tiles(W, H, rank, world) / pt.shard_tiles(W, H, 0, 1)
        if multi:  # kernel timing covers the first device: its tile share
            share = pt.shard_tiles(W, H, 0, args.gpus) / pt.shard_tiles(W, H, 0, 1)
        samples_share = samples_frame * share
        src = kt_iso if kt_iso is not None else kt  # each one frame
        if not src:  # neither timing frame ran (--no-roofline-leg --no-kernel-timing: profiler passes)
            src = {"bounce": (float("nan"), 1)}
        nfr = 1
        walked = node_kernel(src) == "walk"  # the trace runs in wf_walk (large tree, no marched shape)
        bounce_ev = [k for k in FLOP_WEIGHTS if k not in MARCH_EVENTS and not (walked and k in WALK_EVENTS)]
        f_weights = {"march": flops_per_sample(counts, MARCH_EVENTS),
                     "bounce": flops_per_sample(counts, bounce_ev),
                     "walk": flops_per_sample(counts, WALK_EVENTS) if walked else 0.0,
                     "megakernel": F}
        workload = "%s %dx%d %dspp depth %d" % (args.scene, W, H, spp, args.depth)
        # algorithmic FLOPs per sample: from the f64 instruction counters of a committed PMC pass of this
        # workload (scripts/pmc_flops.py) when there is one, else the event counts times FLOP_WEIGHTS
        src_id = pt.source_id()
        ff, fl, _, f_why = pmc_lookup("flops", args.scene, args.depth, W, H, spp, src_id)
        f_kind = dict(f_weights)
        if fl:
            for k, v in fl["kinds"].items():
                f_kind[k] = v["algorithmic_flops_per_sample"]
            F = f_kind["bounce"] + f_kind["march"] + f_kind.get("walk", 0.0)
        kname = {"bounce": "wf_bounce", "march": "wf_march", "walk": "wf_walk", "megakernel": "render_tiles"}
        dom = max(("bounce", "march", "walk", "megakernel"), key=lambda k: src.get(k, (0, 0))[0])
        dom_ms, dom_n = src[dom]
        achieved = f_kind[dom] * samples_share * nfr / (dom_ms / 1e3) / 1e12
        per_kernel = {}
        for k in ("bounce", "march", "walk", "megakernel"):
            ms_k, n_k = src.get(k, (0.0, 0))
            if n_k:
                a_k = f_kind[k] * samples_share * nfr / (ms_k / 1e3) / 1e12
                per_kernel[kname[k]] = {"achieved": round(a_k, 4), "frac": round(a_k / FP64_PEAK_TFLOPS, 5),
                                        "flops_per_sample": round(f_kind[k], 1),
                                        "flops_per_sample_weights": round(f_weights[k], 1), "launches": n_k // nfr,
                                        "ms_per_frame": round(ms_k / nfr, 3),
                                        "kernel_ms_avg": round(ms_k / n_k, 4)}
        # the large-tree bounce build tests BVH nodes in f32: 6 FMAs per node slab, outside the f64
        # counters; reported beside the f64 roofline, and both shares of the VALU's FLOP rate summed
        f32_kind = {}
        nk = node_kernel(src)
        if r.get_option("bvh_nodes") >= BIG_BVH_NODES and src.get(nk, (0, 0))[1] > 0:
            f32_ps = f32_node_flops_per_sample(counts)
            ms_b, _ = src[nk]
            a32 = f32_ps * samples_share * nfr / (ms_b / 1e3) / 1e12
            f32_kind = {"kernel": kname[nk], "flops_per_sample": round(f32_ps, 1), "achieved": round(a32, 4),
                        "peak": FP32_PEAK_TFLOPS, "frac": round(a32 / FP32_PEAK_TFLOPS, 5),
                        "source": "(node_slabs - bounces) events (pt_count_work) x 12: six f32 FMAs per node, "
                                  "less the root test the large-tree walk skips once per trace"}
            if kname[nk] in per_kernel:
                per_kernel[kname[nk]]["valu_frac_f64_plus_f32"] = round(
                    per_kernel[kname[nk]]["frac"] + a32 / FP32_PEAK_TFLOPS, 5)
        out_bytes = 24.0 * W * H * share
        tuning = {k: v for k, v in r.options().items() if v != pt.OPTION_DEFAULTS.get(k)}
        rec = {
            "metric": metric_name(args), "value": round(value, 3), "unit": "Msamples/s", "n_gpus": n_gpus,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: re-authored %s, add_random_spheres from seed %d" % (args.scene, args.scene_seed),
            "config": {"workload": workload, "config": args.config or ("c2" if metric_name(args) == METRIC else None),
                       "width": W, "height": H, "spp": spp, "depth": args.depth, "seed": args.seed,
                       "parallelism": ("%d devices in one process, peer-copy gather" % args.gpus if multi else
                                       "tile-interleaved x%d, gloo gather through host memory (rehearsal, %d "
                                       "GPU(s))" % (world, torch.cuda.device_count()) if gloo else
                                       "tile-interleaved x%d, RCCL gather" % world if world > 1 else "single GPU"),
                       "wf_slots": slots},
            "roofline": {"bound": "valu_f64", "achieved": round(achieved, 4), "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved / FP64_PEAK_TFLOPS, 5), "traffic": None,
                         "kernel": kname[dom], "flops_per_sample": round(f_kind[dom], 1),
                         "launches": dom_n // nfr, "kernel_ms_avg": round(dom_ms / max(1, dom_n), 4),
                         "measured": ("one extra frame after the timed steps with one chunk stream (wf_slots=1): "
                                      "every launch alone on the device, HIP events on its stream"
                                      if kt_iso is not None else "timed steps (launches of two chunk streams overlap)"),
                         "kernels": per_kernel,
                         "valu_f32": f32_kind or None,
                         "flops_per_sample_total": round(F, 1),
                         "flops_source": ("f64 instruction counters x mean active lanes, %s (%s; scripts/pmc_flops.py); "
                                          "event weights give %.1f FLOP/sample (%.2fx)"
                                          % (ff.relative_to(ROOT), fl["workload"],
                                             f_weights["bounce"] + f_weights["march"] + f_weights["walk"],
                                             (f_weights["bounce"] + f_weights["march"] + f_weights["walk"]) / F)
                                          if fl else
                                          "kernel event counters (pt_count_work) x FLOP_WEIGHTS (%s)" % f_why),
                         "events_per_sample": {k: round(v / max(1, counts["samples"]), 3)
                                               for k, v in counts.items() if k != "samples"},
                         # the timed steps: two chunk streams run concurrently (pt_wave.hip), so one kernel's
                         # launches overlap the other stream's; these sums of launch durations can exceed the
                         # step time, and the whole path's rate is the frame's FLOPs over the frame time
                         "kernel_ms_per_step_summed_over_streams": {k: round(v[0], 3) for k, v in kt.items()} or None,
                         "kernel_ms_note": ("one frame of the timed workload after the timed steps, HIP events "
                                            "around each launch; launch durations summed per kernel kind over %d "
                                            "concurrent chunk streams: they overlap, so a sum may exceed "
                                            "ms_per_step; per-kernel times of launches that run alone are in "
                                            "`kernels`" % slots),
                         "frame_kernels_ms": round(kernel_ms, 3), "frame_kernels_ms_max_rank": round(kernel_ms_max, 3),
                         "path_achieved": round(F * value * 1e6 / 1e12, 4),
                         "path_frac": round(F * value * 1e6 / 1e12 / FP64_PEAK_TFLOPS, 5)},
            "roofline_hbm": {"achieved": round(out_bytes / (kernel_ms / 1e3) / 1e9, 4), "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": out_bytes / (kernel_ms / 1e3) / 1e9 / HBM_PEAK_GBS,
                             "bytes_per_launch": out_bytes, "note": "algorithmic: 24 B/pixel frame write"},
            "march_guard_drops": guard_drops,
            "frame_plan": {"chunks_per_frame": kt["reduce"][1] if kt else None, "chunk_streams": slots,
                           "note": "the timed frames' sample chunks (one wf_reduce each) on this rank / first device"},
        }
        per_rank_tiles = [pt.shard_tiles(W, H, k, n_gpus) for k in range(n_gpus)]
        rec["rank_share"] = {"tiles_total": pt.shard_tiles(W, H, 0, 1), "tiles_per_rank_max": max(per_rank_tiles),
                             "tiles_per_rank_min": min(per_rank_tiles),
                             "samples_per_rank_max": max(per_rank_tiles) * 256 * spp,
                             "deal": "16x16 tiles, logical tile k -> rank k % N, diagonal columns"}
        if world > 1:
            rec["gather"] = {"bytes_per_rank": per * 256 * 3 * 8, "bytes_total": world * per * 256 * 3 * 8,
                             "ms_per_step": round(gather_ms, 3),
                             "what": ("dist.gather of the compact f64 shards to rank 0 (%s) + pt_unshard_device, "
                                      "HIP events on rank 0's stream" % ("gloo, through host memory" if gloo
                                                                         else "RCCL"))}
        if topo is not None:
            rec["topology"] = topo
        if multi:
            rec["topology"] = {"backend": "one process, peer copies", "devices": [
                device_identity(torch, d) for d in range(args.gpus)]}
            pairs, enabled = r.peer_access()
            rec["gather"] = {"bytes_total": args.gpus * pt.shard_tiles(W, H, 0, args.gpus) * 256 * 3 * 8,
                             "peer_pairs": pairs, "peer_access_enabled": enabled,
                             "what": "hipMemcpyPeerAsync of each device's shard to the first device, per band"}
        if tuning:
            rec["tuning"] = tuning
        # roofline.traffic: HBM bytes per launch of the same kernel from the committed PMC passes of this
        # workload (scripts/pmc_traffic.py; bench.py cannot read PMC counters itself)
        tf, tr, t_spf, t_why = pmc_lookup("traffic", args.scene, args.depth, W, H, spp, src_id)
        if not tr:
            rec["roofline"]["traffic_source"] = t_why
        kind = tr.get("kinds", {}).get(dom) if tr else None
        if kind:
            # bytes per sample of the pass (its launches x bytes per launch over its samples), times the samples
            # this rank's (or first device's) launches of the kernel processed, per launch: bytes per sample do
            # not depend on the chunking or the frame size, bytes per launch do
            per_sample = kind["traffic"] * kind["launches"] / (t_spf * tr.get("frames", 1))
            per_launch = per_sample * samples_share * nfr / max(1, dom_n)
            rec["roofline"]["traffic"] = round(per_launch)
            rec["roofline"]["traffic_source"] = ("%s (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, %s)"
                                                 % (tf.relative_to(ROOT), tr["workload"]))
            rec["roofline"]["traffic_gbs"] = round(per_launch / (dom_ms / max(1, dom_n) / 1e3) / 1e9, 1)
            rec["roofline"]["traffic_per_sample"] = round(per_sample, 1)
            if world > 1 or multi:
                rec["roofline"]["traffic_note"] = "per launch of this rank's share (%d of %d tiles)" % (
                    per_rank_tiles[0], pt.shard_tiles(W, H, 0, 1))
        if not args.no_parity:
            import oracle
            px = parity_pixels(args)
            sc = oracle.Scene(text, seed=args.scene_seed).use_bvh(True, 7)
            t = time.perf_counter()
            ref = sc.render(W, H, spp, args.depth, args.seed, pixels=px, threads=host_cpus()["share"])
            got = img[px]
            rec["rms_vs_oracle"] = float(np.sqrt(np.mean((got - ref) ** 2)))
            rec["rms_per_channel"] = [float(x) for x in np.sqrt(np.mean((got - ref) ** 2, axis=0))]
            rec["rms_pixels"] = int(len(px))
            rec["exact_pixels_frac"] = float(np.mean(np.all(got == ref, axis=1)))
            rec["parity_pixels"] = ("stratified: 16-px grid + full row %d + full column %d, %d spp, %.1f s"
                                    % (min(H - 1, H * 757 // 1080), min(W - 1, W * 1142 // 1920), spp,
                                       time.perf_counter() - t) if not args.parity_pixels
                                    else "%d random pixels" % len(px))
            rec["parity_frame"] = ("the last timed step's frame (the one behind `value`: %d chunks on %d chunk "
                                   "streams%s), copied out before the kernel-timing and roofline frames"
                                   % (rec["frame_plan"]["chunks_per_frame"], slots,
                                      ", gathered from %d ranks" % world if world > 1 else ""))
        if world == 1 and not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_baseline(text, args)
        print(json.dumps(finite_or_null(rec)), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
