"""Generates tests/golden/kat_primitives.json with the independent pure-Python
restatement (pyref.py) — known-answer vectors for single-shape hits
(ray_hit_transformed over Sphere / Rectangle / Cube / Heart), written as
float.hex strings so the comparison is bit-exact.

    python tests/golden/make_golden.py
"""
import json
import math
import random
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
import pyref  # noqa: E402

# Shapes: the cornell_box / spheres.json leaves plus edge cases.
SHAPES = {
    "unit_sphere": {"type": "Sphere", "translate": [0, 0, 0], "rotate": [0, 0, 0], "scale": [1, 1, 1]},
    "inverse_sphere": {"type": "Sphere", "translate": [0, 1, 0], "rotate": [0, 0, 0], "scale": [0.5, 0.5, 0.5],
                       "inverse_normal": True},
    "ground": {"type": "Sphere", "translate": [0, -1000, 0], "rotate": [0, 0, 0], "scale": [1000, 1000, 1000]},
    "cornell_green": {"type": "Rectangle", "x0": 0, "x1": 555, "y0": 0, "y1": 555, "translate": [555, 0, 555],
                      "rotate": [0, 90, 0], "scale": [1, 1, 1]},
    "cornell_floor": {"type": "Rectangle", "x0": 0, "x1": 555, "y0": 0, "y1": 555, "translate": [0, 0, 0],
                      "rotate": [90, 0, 0], "scale": [1, 1, 1]},
    "cornell_back": {"type": "Rectangle", "x0": 0, "x1": 555, "y0": 0, "y1": 555, "translate": [555, 0, 555],
                     "rotate": [0, 0, 90], "scale": [1, 1, 1]},
    "cornell_light": {"type": "Rectangle", "x0": 213, "x1": 343, "y0": 227, "y1": 332, "translate": [0, 554, 0],
                      "rotate": [90, 0, 0], "scale": [1, 1, 1]},
    "cornell_cube1": {"type": "Cube", "translate": [347.5, 165, 377.5], "rotate": [0, 15, 0],
                      "scale": [82.5, 165, 82.5]},
    "cornell_cube2": {"type": "Cube", "translate": [212.5, 82.5, 147.5], "rotate": [0, -18, 0],
                      "scale": [82.5, 82.5, 82.5]},
    "unit_cube": {"type": "Cube", "translate": [0, 0, 0], "rotate": [0, 0, 0], "scale": [1, 1, 1]},
    "heart_unit": {"type": "Heart", "translate": [-4, 1, 0], "rotate": [-90, 25, 0], "scale": [1, 1, 1],
                   "step": 0.01, "depth": 4},
    "cornell_heart": {"type": "Heart", "translate": [212.5, 200, 147.5], "rotate": [-95, -18, 0],
                      "scale": [82.5, 82.5, 82.5], "step": 0.01, "depth": 4},
}


def rays_for(name, sh, rng):
    c = sh["translate"]
    rays = []
    if name == "unit_sphere":  # hand-derivable cases first
        rays += [((0, 0, -5), (0, 0, 1)), ((0, 0, 0), (0, 0, 1)), ((1, 0, -5), (0, 0, 1)), ((2, 0, -5), (0, 0, 1))]
    if name == "unit_cube":
        rays += [((0, 0, -5), (0, 0, 1)), ((0, 0, 0), (1, 0, 0)), ((0.5, 0.5, -3), (0, 0, 1))]
    eye = (278.0, 278.0, -800.0) if name.startswith("cornell") else (0.0, 3.0, -20.0)
    n = 4 if "heart" in name else 12
    spread = 60.0 if name.startswith("cornell") else 1.5
    for _ in range(n):
        target = tuple(c[k] + rng.uniform(-spread, spread) for k in range(3))
        rays.append((eye, pyref.norm(tuple(target[k] - eye[k] for k in range(3)))))
    for _ in range(4 if "heart" in name else 8):  # random directions from a point near the shape
        o = tuple(c[k] + rng.uniform(-3 * spread, 3 * spread) for k in range(3))
        rays.append((o, pyref.norm((rng.gauss(0, 1), rng.gauss(0, 1), rng.gauss(0, 1)))))
    return rays


def hexs(v):
    return [float(x).hex() for x in v]


def main():
    rng = random.Random(20261015)
    out = {"shapes": SHAPES, "cases": []}
    for name, sh in SHAPES.items():
        for o, d in rays_for(name, sh, rng):
            o = tuple(float(x) for x in o)
            d = tuple(float(x) for x in d)
            h = pyref.shape_hit(sh, o, d)
            case = {"shape": name, "o": hexs(o), "d": hexs(d)}
            if h is None:
                case["hit"] = None
            else:
                t, p, n, front = h
                case["hit"] = {"t": float(t).hex(), "point": hexs(p), "normal": hexs(n), "front": bool(front)}
            out["cases"].append(case)
    (HERE / "kat_primitives.json").write_text(json.dumps(out, indent=0) + "\n")
    hits = sum(1 for c in out["cases"] if c["hit"])
    print("wrote %d cases (%d hits)" % (len(out["cases"]), hits))


if __name__ == "__main__":
    main()
