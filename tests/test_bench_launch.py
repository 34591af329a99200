"""bench.py's launch decision (CPU): a plain `bench.py --gpus N` runs N ranks under torch.distributed.run in a child
process, and refuses nccl with fewer devices than ranks (VERDICT r4 ask 1; the reference's parallelism knob,
ThreadPoolRenderer::new(scene, thread_number, depth), src/renderer/step_by_step.rs:37, takes effect however the
renderer is started)."""
import subprocess
import sys
from pathlib import Path
from types import SimpleNamespace

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def args(gpus=1, single=False, backend="nccl"):
    return SimpleNamespace(gpus=gpus, single_process=single, dist_backend=backend)


def test_launch_plan():
    assert bench.launch_plan(args(1), {}) == "one"
    assert bench.launch_plan(args(8), {}) == "spawn"
    assert bench.launch_plan(args(2, backend="gloo"), {}) == "spawn"
    assert bench.launch_plan(args(8, single=True), {}) == "single-process"
    # a rank of a launch (the driver's torchrun, or the child this bench starts) never spawns again
    assert bench.launch_plan(args(8), {"WORLD_SIZE": "8"}) == "ranks"
    assert bench.launch_plan(args(1), {"WORLD_SIZE": "1"}) == "ranks"


def test_device_shortfall():
    assert bench.device_shortfall(8, "nccl", 8) is None
    assert bench.device_shortfall(4, "nccl", 8) is None
    msg = bench.device_shortfall(2, "nccl", 1)
    assert msg and "need 2 GPUs" in msg and "1 device is visible" in msg
    assert "0 devices are visible" in bench.device_shortfall(2, "nccl", 0)
    assert bench.device_shortfall(8, "gloo", 1) is None  # gloo ranks may share one GPU (rehearsal)
    assert bench.device_shortfall(2, "gloo", 0) == "bench.py: no GPU visible"


def test_plain_multi_gpu_bench_refuses_too_few_devices():
    """On this CPU container no device is visible: a plain --gpus 2 over nccl exits non-zero at once, naming the
    device count, before any rank starts."""
    # (no device visible to the child whatever the host has: it must refuse, not start a real 2-rank bench)
    env = {k: v for k, v in __import__("os").environ.items() if k != "WORLD_SIZE"}
    env.update(HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, cwd=str(ROOT), env=env)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "need 2 GPUs" in r.stderr and "0 devices are visible" in r.stderr
    assert "launching" not in r.stderr


def test_topology_fields_and_refusal():
    """A multi-rank line reports what each rank ran on; under nccl two ranks on one physical GPU are refused
    (the line would not measure N GPUs), under gloo (a rehearsal on fewer GPUs) they are reported, not refused."""
    dev = lambda r, u: {"rank": r, "local_rank": r, "device": r, "pci": "0000:%02x:00" % (0x10 + u), "uuid": "GPU-%d" % u,
                        "name": "AMD Instinct MI355X"}
    ok = bench.device_topology([dev(1, 1), dev(0, 0)], "nccl", 2)
    assert ok["distinct_devices"] == 2 and ok["shared_devices"] == [] and ok["comm_size"] == 2
    assert [i["rank"] for i in ok["ranks"]] == [0, 1] and ok["backend"] == "nccl"
    assert bench.topology_refusal(ok) is None
    same = bench.device_topology([dev(0, 0), dev(1, 0), dev(2, 1)], "nccl", 3)
    assert same["shared_devices"] == [[0, 1]] and same["distinct_devices"] == 2
    msg = bench.topology_refusal(same)
    assert msg and "share a device" in msg and "[[0, 1]]" in msg
    rehearsal = bench.device_topology([dev(0, 0), dev(1, 0)], "gloo", 2)
    assert rehearsal["shared_devices"] == [[0, 1]] and bench.topology_refusal(rehearsal) is None
    assert "communicator size" in bench.topology_refusal(bench.device_topology([dev(0, 0)], "gloo", 2))
    # a blank UUID (a driver that reports none) does not make distinct GPUs one device: the PCI address differs
    blank = [dict(dev(r, r), uuid="") for r in range(8)]
    assert bench.topology_refusal(bench.device_topology(blank, "nccl", 8)) is None


def _gather_identities(rank, world, port, out):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = {"rank": rank, "local_rank": rank, "device": 0, "pci": "0000:%02x:00" % rank, "uuid": "GPU-%d" % rank,
            "name": "x"}
    infos = [None] * world
    dist.all_gather_object(infos, mine)
    topo = bench.device_topology(infos, "nccl", dist.get_world_size())
    out.put((rank, topo["distinct_devices"], topo["comm_size"], bench.topology_refusal(topo)))
    dist.destroy_process_group()


def test_topology_gathered_over_two_ranks():
    """The identities go through the same all_gather_object bench.py uses (gloo, world 2, CPU)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = bench.free_port()
    ps = [ctx.Process(target=_gather_identities, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == [(0, 2, 2, None), (1, 2, 2, None)]


def test_bench_line_is_strict_json():
    """A profiler pass's record (no timing frames: NaN roofline fields) prints as strict JSON, NaN as null."""
    import json
    rec = bench.finite_or_null({"roofline": {"achieved": float("nan"), "frac": float("inf")}, "value": 2042.8,
                                "kernels": [1.5, float("-inf")]})
    text = json.dumps(rec, allow_nan=False)
    assert json.loads(text) == {"roofline": {"achieved": None, "frac": None}, "value": 2042.8, "kernels": [1.5, None]}
