"""The large-tree bounce build (BVH of >= 2^15 nodes per layout: the f32 node slab
with its folded widening and the axis-aligned sphere leaves) on
scenes far from the origin and at other scales, every pixel against the oracle's
reference BvhNode traversal (src/world/shapes/mod.rs:620-729).  The widening
grows with |o| and the planes' magnitude (bvh_bound), so these are the frames
where a cull that is not conservative would show: a lost hit changes a pixel.
Forced onto the wavefront engine (engine = 2), whose bounce kernel is the only
user of the large-tree build.
"""
import json
import sys
from pathlib import Path

import numpy as np
import pytest

import oracle as O
from conftest import host_threads

pytestmark = pytest.mark.gpu

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "scenes"))


def moved(scene, shift=(0.0, 0.0, 0.0), scale=1.0):
    """Every translation and the camera position scaled by `scale` then shifted; sphere scales by `scale`."""
    doc = json.loads(json.dumps(scene))
    for s in doc["shapes"]:
        t = s["transform"]
        t["translate"] = [v * scale + d for v, d in zip(t["translate"], shift)]
        if "scale" in t:
            t["scale"] = [v * scale for v in t["scale"]]
    cam = doc["camera"]
    cam["position"] = [v * scale + d for v, d in zip(cam["position"], shift)]
    return doc


def render_both(pt, doc, w=128, h=72, spp=2, depth=8, seed=3, **opts):
    import torch
    text = json.dumps(doc)
    ps = pt.Scene.from_json(text, seed=1)
    r = pt.HipRenderer(ps, depth=depth)
    r.set_option("engine", 2)
    for k, v in opts.items():
        r.set_option(k, v)
    assert r.get_option("bvh_nodes") >= 1 << 15, "not the large-tree build"
    frame = torch.zeros(w * h * 3, dtype=torch.float64, device="cuda")
    r.render_device(ps.camera(), w, h, spp, seed, 0, 1, frame.data_ptr())
    torch.cuda.synchronize()
    img = frame.view(-1, 3).cpu().numpy()
    ref = O.Scene(text, seed=1).use_bvh(True, 7).render(w, h, spp, depth, seed, threads=host_threads())
    return img, ref


@pytest.mark.parametrize("shift,scale", [((0.0, 0.0, 0.0), 1.0), ((3.0e4, 0.0, -2.0e4), 1.0),
                                         ((-7.5e5, 40.0, 1.25e5), 1.0), ((0.0, 0.0, 0.0), 1.0e3),
                                         ((12.0, 0.0, -5.0), 0.01)])
def test_large_tree_frames_far_and_scaled(pt, shift, scale):
    import make_scenes
    doc = moved(make_scenes.synthetic(40000), shift, scale)
    img, ref = render_both(pt, doc)
    bad = np.flatnonzero(np.any(img != ref, axis=1))
    assert bad.size == 0, "%d of %d pixels differ (first %s)" % (bad.size, len(img), bad[:8].tolist())
    assert np.count_nonzero(ref) > 0


@pytest.mark.parametrize("waves", [0, 4, 6, 8])
def test_walk_register_budgets(pt, waves):
    """Every register budget of the large-tree walk kernel (wf_walk 4, 6, 8 waves per SIMD, the 6- and 8-wave
    builds with spills; 0: the walk inside the bounce kernel) renders the oracle's pixels (the default 5 is every
    other test of this file)."""
    import make_scenes
    img, ref = render_both(pt, make_scenes.synthetic(40000), w=96, h=54, wf_walk=waves)
    bad = np.flatnonzero(np.any(img != ref, axis=1))
    assert len(bad) == 0, "%d of %d pixels differ" % (len(bad), len(img))
