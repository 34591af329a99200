"""Adversarial rays (tests/adversarial.py) through the host build of the
product's skipping march against the oracle's literal march
(src/world/shapes/ray_marching.rs:20-74): grazing rays, frozen and
zero-crossing coordinates, binade edges, at cornell's 82.5x Heart and at
scale 1, for several step / depth settings.  The same rays run through the
GPU kernels in test_gpu_fullframe.py."""
import numpy as np
import pytest

import adversarial as A
import oracle as O
from test_march_exact import march_lib, run_case  # noqa: F401  (fixture)


@pytest.mark.parametrize("xf", ["cornell", "unit", "scaled"])
def test_adversarial_rays_exact(march_lib, xf):
    tr = {"cornell": A.HEART_XF, "unit": A.UNIT_XF, "scaled": A.SCALED_XF}[xf]
    sc = O.Scene(A.heart_json(tr), random_spheres=False)
    rays = A.world_rays(sc.shape(0).direct, A.object_rays(np.random.default_rng(41)))
    n_hit, _ = run_case(march_lib, sc, rays, 0.01, 4)
    assert n_hit > 100


@pytest.mark.parametrize("step,depth", [(0.05, 4), (0.003, 4), (0.01, 1), (0.01, 0), (0.02, 7), (-0.01, 4)])
def test_adversarial_rays_march_parameters(march_lib, step, depth):
    sc = O.Scene(A.heart_json(A.UNIT_XF, step=step, depth=depth), random_spheres=False)
    rays = A.world_rays(sc.shape(0).direct, A.object_rays(np.random.default_rng(43), n_graze=150))
    run_case(march_lib, sc, rays, step, depth)
