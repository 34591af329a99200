"""Adversarial rays for the exact skipping march (pt_march.hpp), shared by the
host-build test (test_march_adversarial.py) and the GPU test
(test_gpu_fullframe.py).  Each family aims at a place where the closed-form
accumulation or the Bernstein sign proof could differ from the reference's
literal march (src/world/shapes/ray_marching.rs:20-74):

* grazing: rays tangent to the Heart surface, shifted along the normal by
  0, +-1e-12 .. +-1e-3 of the object scale (f stays within a hair of 0 for
  many steps: the proof margin is what decides);
* frozen / zero-crossing: object-space rays with a direction component
  exactly 0 (that coordinate never changes: the c == 0 closed form), rays
  lying in a coordinate plane, and rays through the object origin (every
  coordinate crosses 0 at once: no binade segment is long there);
* binade edges: origins with power-of-two coordinates and directions that
  keep a coordinate on a binade edge for a while;
* scale: the same families at cornell's 82.5x Heart and at scale 1.
"""
import json

import numpy as np

HEART_XF = {"translate": [212.5, 200, 147.5], "rotate": [-95, -18, 0], "scale": [82.5, 82.5, 82.5]}
UNIT_XF = {"translate": [0, 0, 0], "rotate": [0, 0, 0], "scale": [1, 1, 1]}
SCALED_XF = {"translate": [0, 0, 0], "rotate": [0, 0, 0], "scale": [82.5, 82.5, 82.5]}


def heart_json(xf, step=0.01, depth=None):
    sh = {"type": "BruteForsableShape", "name": "Heart", "shape": {"type": "Heart", "sphere_radius": 1.45},
          "step": step, "transform": xf, "material": "Red"}
    if depth is not None:
        sh["depth"] = depth
    return json.dumps({
        "camera": {"position": [278, 278, -800], "direction": [0, 0, 1], "up": [0, 1, 0], "fov": 40,
                   "focal_length": 1},
        "shapes": [sh],
        "materials": {"Red": {"type": "Lambertian", "albedo": {"type": "SolidColor", "color": [0.65, 0.05, 0.05]}}},
        "background": [0, 0, 0]})


def heart_f(p):
    x, y, z = p[..., 0], p[..., 1], p[..., 2]
    a = x * x + 2.25 * y * y + z * z - 1.0
    return a ** 3 - x * x * z ** 3 - 0.1125 * y * y * z ** 3


def heart_grad(p, h=1e-7):
    g = np.zeros_like(p)
    for k in range(3):
        e = np.zeros(3)
        e[k] = h
        g[..., k] = (heart_f(p + e) - heart_f(p - e)) / (2 * h)
    return g


def surface_points(rng, n):
    """Points on f = 0 along random directions from the object origin (f(0) = -1)."""
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    lo = np.zeros(n)
    hi = np.full(n, 1.6)
    for _ in range(80):
        mid = 0.5 * (lo + hi)
        inside = heart_f(u * mid[:, None]) < 0
        lo = np.where(inside, mid, lo)
        hi = np.where(inside, hi, mid)
    return u * lo[:, None]


def object_rays(rng, n_graze=400):
    """(origin, direction) pairs in object space, not normalised."""
    rays = []
    # grazing: tangent at a surface point, shifted along the normal
    p = surface_points(rng, n_graze)
    g = heart_grad(p)
    g /= np.linalg.norm(g, axis=1, keepdims=True)
    t = np.cross(g, rng.normal(size=(n_graze, 3)))
    t /= np.linalg.norm(t, axis=1, keepdims=True)
    shifts = np.array([0.0, 1e-12, -1e-12, 1e-9, -1e-9, 1e-6, -1e-6, 1e-3, -1e-3])
    s = shifts[rng.integers(0, len(shifts), n_graze)]
    o = p + g * s[:, None] - 2.5 * t
    rays += [np.concatenate([o, t], 1)]
    # frozen coordinates and coordinate planes: one or two direction components exactly 0
    m = 240
    o = rng.uniform(-3, 3, size=(m, 3))
    d = rng.normal(size=(m, 3))
    for i in range(m):
        k = i % 3
        d[i, k] = 0.0
        if i % 2 == 0:
            o[i, k] = 0.0  # the frozen coordinate sits exactly at 0
        if i % 5 == 0:
            d[i, (k + 1) % 3] = 0.0
    aim = -o + rng.normal(scale=0.3, size=(m, 3))  # point roughly back at the heart
    for i in range(m):
        for k in range(3):
            if d[i, k] != 0.0:
                d[i, k] = aim[i, k]
    rays += [np.concatenate([o, d], 1)]
    # through the object origin: every coordinate crosses 0 together
    m = 120
    d = rng.normal(size=(m, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = -d * rng.uniform(1.6, 4.0, size=(m, 1))
    rays += [np.concatenate([o, d], 1)]
    # binade edges: power-of-two origins, one direction component tiny
    m = 120
    pw = 2.0 ** rng.integers(-3, 2, size=(m, 3)) * rng.choice([-1.0, 1.0], size=(m, 3))
    d = -pw + rng.normal(scale=0.05, size=(m, 3))
    d[np.arange(m), rng.integers(0, 3, m)] *= 1e-9
    rays += [np.concatenate([pw * 2.0, d], 1)]
    return np.concatenate(rays)


def world_rays(direct, obj):
    """World rays (normalised directions) for object-space rays under `direct` (4x4 row-major)."""
    D = np.asarray(direct, float).reshape(4, 4)
    o = obj[:, :3] @ D[:3, :3].T + D[:3, 3]
    d = obj[:, 3:] @ D[:3, :3].T
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return np.concatenate([o, d], 1)
