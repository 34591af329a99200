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
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, cwd=str(ROOT),
                       env={k: v for k, v in __import__("os").environ.items() if k != "WORLD_SIZE"})
    assert r.returncode == 2, r.stderr[-2000:]
    assert "need 2 GPUs" in r.stderr and "0 devices are visible" in r.stderr
    assert "launching" not in r.stderr
