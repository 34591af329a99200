"""The multi-rank frame path on the GPU: bench.py under torch.distributed.run
with 2 and 3 ranks sharing the test box's one GPU over the gloo rehearsal
backend.  Every rank renders its diagonal tile deal through the C-ABI
(pt_render_device, rank r of N), the compact shards are gathered to rank 0
and un-interleaved there by pt_unshard_device; rank 0's frame is checked
against the oracle on bench.py's stratified pixel set (the same check as the
single-GPU bench line).  The RCCL gather itself needs one GPU per rank and is
the driver's multi-GPU run."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_ranks_gather_unshard_parity(world):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           str(ROOT / "bench.py"), "--gpus", str(world), "--dist-backend", "gloo",
           "--scene", "cornell_box.json", "--width", "320", "--height", "180", "--spp", "4",
           "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == world
    assert "gloo gather" in rec["config"]["parallelism"]
    assert rec["rms_pixels"] >= 700
    assert rec["exact_pixels_frac"] == 1.0 and rec["rms_vs_oracle"] == 0.0
    # the frame checked is the last timed step's, gathered from every rank (the roofline leg ran after it)
    assert "gathered from %d ranks" % world in rec["parity_frame"]
    assert rec["gather"]["bytes_per_rank"] == rec["rank_share"]["tiles_per_rank_max"] * 256 * 3 * 8
