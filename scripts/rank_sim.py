"""Per-rank render time of the N-GPU tile partition, simulated on one GPU.

For world N, each rank r renders its round-robin tiles (render_device with
rank r of N) into its compact shard; the N-GPU frame time is the slowest
rank's plus the frame-end gather and un-interleave.  Running every rank's
share on the one GPU we have gives the compute part without the other GPUs;
the gather is bounded from the link rate the design assumes (an
MI355X has 7 xGMI links of ~153 GB/s, one to each other GPU of the node):

* lower bound: every rank's shard reaches rank 0 over its own link at once,
  shard bytes / link rate, plus the un-interleave kernel timed here;
* upper bound: the N-1 shards reach rank 0 one after another over one link,
  (N-1) x shard bytes / link rate, plus the un-interleave;
* a local device-to-device copy of the gathered bytes (round 3's model) is
  reported beside them; it is faster than any link, so it is not a bound.

    python scripts/rank_sim.py [--worlds 1,8] [--spp 256] [--reps 2] [--link-gbs 153]

Prints one JSON line per world: max/mean rank ms, the gather bounds, and the
projected strong-scaling efficiency t1 / (N * (max_rank_ms + gather)) for the
compute alone and with each bound.  The driver's SCALE run measures the real one.
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--ranks", default="", help="subset of ranks to time (default: all)")
    ap.add_argument("--link-gbs", type=float, default=153.0, help="xGMI link rate per direction (GB/s)")
    ap.add_argument("--scene", default="cornell_box.json")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="a renderer tuning option (pt_renderer_set_option), repeatable")
    a = ap.parse_args()
    import torch
    import __graft_entry__ as ge
    pt = ge.load_package()
    text = (ROOT / "scenes" / a.scene).read_text()
    scene = pt.Scene.from_json(text, seed=1)
    r = pt.HipRenderer(scene, device=0, depth=8)
    for o in a.option:
        k, v = o.split("=", 1)
        r.set_option(k, int(v))
    cam = scene.camera()
    W, H, spp = a.width, a.height, a.spp
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    buf = torch.zeros(W * H * 3, dtype=torch.float64, device="cuda")
    t1 = None
    for world in [int(x) for x in a.worlds.split(",")]:
        ranks = [int(x) for x in a.ranks.split(",")] if a.ranks else list(range(world))
        ms = []
        for rank in ranks:
            if rank >= world:
                continue
            r.render_device(cam, W, H, spp, 1, rank, world, buf.data_ptr(), sp)  # warm
            torch.cuda.synchronize()
            best = 1e30
            for _ in range(a.reps):
                t = time.perf_counter()
                r.render_device(cam, W, H, spp, 1, rank, world, buf.data_ptr(), sp)
                torch.cuda.synchronize()
                best = min(best, (time.perf_counter() - t) * 1e3)
            ms.append(best)
            print("world %d rank %d: %.1f ms" % (world, rank, best), file=sys.stderr, flush=True)
        mx = max(ms)
        if world == 1:
            t1 = mx
        copy_ms = unshard_ms = 0.0
        shard_bytes = 0
        if world > 1:  # the frame-end gather's local-copy model and the un-interleave, timed separately
            per = pt.shard_tiles(W, H, 0, world)
            shard_bytes = per * 256 * 3 * 8
            g = torch.zeros(world * per * 256 * 3, dtype=torch.float64, device="cuda")
            src = torch.zeros_like(g)
            frame = torch.zeros(W * H * 3, dtype=torch.float64, device="cuda")
            for rep in range(a.reps + 1):
                torch.cuda.synchronize()
                t = time.perf_counter()
                g.copy_(src)
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                pt.unshard_device(g.data_ptr(), W, H, world, frame.data_ptr(), sp)
                torch.cuda.synchronize()
                if rep:
                    copy_ms = min(copy_ms or 1e30, (t2 - t) * 1e3)
                    unshard_ms = min(unshard_ms or 1e30, (time.perf_counter() - t2) * 1e3)
        link = a.link_gbs * 1e9
        lb_ms = (shard_bytes / link * 1e3 + unshard_ms) if world > 1 else 0.0
        ub_ms = ((world - 1) * shard_bytes / link * 1e3 + unshard_ms) if world > 1 else 0.0
        rec = {"world": world, "max_rank_ms": round(mx, 2), "mean_rank_ms": round(sum(ms) / len(ms), 2),
               "shard_bytes": shard_bytes, "unshard_ms": round(unshard_ms, 3),
               "gather_link_lb_ms": round(lb_ms, 3), "gather_link_ub_ms": round(ub_ms, 3),
               "gather_local_copy_ms": round(copy_ms + unshard_ms, 3),
               "msamples_s_range": [round(W * H * spp / (mx + ub_ms) / 1e3, 1), round(W * H * spp / (mx + lb_ms) / 1e3, 1)]}
        if t1:
            rec["projected_eff_compute_only"] = round(t1 / (world * mx), 4)
            rec["projected_eff_range"] = [round(t1 / (world * (mx + ub_ms)), 4), round(t1 / (world * (mx + lb_ms)), 4)]
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
