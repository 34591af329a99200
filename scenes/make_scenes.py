"""Writes the benchmark scenes in the reference's JSON schema.

The scenes are re-authored (not copied): the Cornell box is the standard
public 555-unit box (walls, ceiling light, two blocks) as the reference
configures it in scenes/cornell_box.json, plus its ray-marched Heart
(BruteForsableShape); spheres.json is the reference's ground + glass + heart
arrangement.  The schema is SceneJson (src/world/json_models.rs:23-29).

    python scenes/make_scenes.py            # writes cornell_box.json, spheres.json
    python scenes/make_scenes.py --synthetic N   # also synthetic_N.json (config C5)

textured.json and noise.json exercise every texture (CheckerTexture,
UVChecker, NoiseTexture, ImageTexture on textures/grid.ppm; texture.rs).
marched.json exercises every ray-marched ShapeFunction of the reference
(Heart, Sine, Star, DupinCyclide, HuntsSurface, Cushion;
src/world/shapes/ray_marching.rs:121-520) on a ground plane under a light.
"""
import argparse
import json
import random
from pathlib import Path

HERE = Path(__file__).resolve().parent


def tr(t, r=(0, 0, 0), s=(1, 1, 1)):
    return {"translate": list(t), "rotate": list(r), "scale": list(s)}


def solid(c):
    return {"type": "SolidColor", "color": list(c)}


def lambert(c):
    return {"type": "Lambertian", "albedo": solid(c)}


def cornell():
    def wall(t, r, mat, x=(0, 555), y=(0, 555)):
        return {"type": "Rectangle", "x0": x[0], "x1": x[1], "y0": y[0], "y1": y[1],
                "transform": tr(t, r), "material": mat}

    shapes = [
        wall((555, 0, 555), (0, 90, 0), "Green"),
        wall((0, 0, 555), (0, 90, 0), "Red"),
        wall((0, 0, 0), (90, 0, 0), "White"),
        wall((0, 555, 0), (90, 0, 0), "White"),
        wall((555, 0, 555), (0, 0, 90), "White"),
        wall((0, 554, 0), (90, 0, 0), "Light", x=(213, 343), y=(227, 332)),
        {"type": "Cube", "name": "Cube1", "transform": tr((347.5, 165, 377.5), (0, 15, 0), (82.5, 165, 82.5)),
         "material": "White"},
        {"type": "Cube", "name": "Cube2", "transform": tr((212.5, 82.5, 147.5), (0, -18, 0), (82.5, 82.5, 82.5)),
         "material": "White"},
        {"type": "BruteForsableShape", "name": "Heart", "shape": {"type": "Heart", "sphere_radius": 1.45},
         "step": 0.01, "transform": tr((212.5, 200, 147.5), (-95, -18, 0), (82.5, 82.5, 82.5)),
         "material": "Red"},
    ]
    return {
        "camera": {"position": [278, 278, -800], "direction": [0, 0, 1], "up": [0, 1, 0],
                   "fov": 40, "focal_length": 1},
        "shapes": shapes,
        "materials": {
            "Green": lambert((0.12, 0.45, 0.15)),
            "Red": lambert((0.65, 0.05, 0.05)),
            "White": lambert((0.73, 0.73, 0.73)),
            "Light": {"type": "DiffuseLight", "emit": solid((15, 15, 15))},
        },
        "background": [0, 0, 0],
    }


def spheres():
    shapes = [
        {"type": "Sphere", "name": "Ground", "transform": tr((0, -1000, 0), s=(1000, 1000, 1000)),
         "material": "Ground"},
        {"type": "Sphere", "name": "GlassSphere", "transform": tr((0, 1, 0), (-90, 0, 0)), "material": "Glass"},
        {"type": "Sphere", "name": "GlassSphereInside", "transform": tr((0, 1, 0), s=(0.5, 0.5, 0.5)),
         "material": "Glass", "inverse_normal": True},
        {"type": "BruteForsableShape", "name": "Heart2", "shape": {"type": "Heart"}, "step": 0.01,
         "transform": tr((-4, 1, 0), (-90, 25, 0)), "material": "Brown"},
        {"type": "BruteForsableShape", "name": "Heart3", "shape": {"type": "Heart"}, "step": 0.01,
         "transform": tr((4, 2, 0), (-90, -25, 0)), "material": "Mirror"},
    ]
    return {
        "camera": {"position": [-0.6, 7, -69], "direction": [0.6, -7, 69], "up": [0, 1, 0],
                   "fov": 20, "focal_length": 1},
        "shapes": shapes,
        "materials": {
            "Ground": lambert((0.5, 0.5, 0.5)),
            "Glass": {"type": "Dielectric", "index_of_refraction": 1.5},
            "Brown": lambert((0.4, 0.2, 0.1)),
            "Mirror": {"type": "Metal", "albedo": solid((0.7, 0.6, 0.5)), "fuzz": 0},
        },
        "background": [0, 0, 0],
    }


def marched():
    def fn(name, shape, t, r, scale, mat, step=0.01, depth=4):
        return {"type": "BruteForsableShape", "name": name, "shape": shape, "step": step, "depth": depth,
                "transform": tr(t, r, (scale, scale, scale)), "material": mat}

    shapes = [
        {"type": "Sphere", "name": "Ground", "transform": tr((0, -1000, 0), s=(1000, 1000, 1000)),
         "material": "Ground"},
        {"type": "Rectangle", "x0": -3, "x1": 3, "y0": -2, "y1": 2, "transform": tr((0, 9, 2), (90, 0, 0)),
         "material": "Light"},
        fn("Dupin", {"type": "DupinCyclide", "a": 1.11, "b": 0.99, "c": 0.5, "d": 0.1, "sphere_radius": 2.5},
           (-6, 1.6, 0), (0, -100, 0), 1.2, "Copper"),
        fn("Sine", {"type": "Sine", "a": 1.0, "sphere_radius": 1.5}, (-3, 1.6, 0), (20, 30, 0), 1.0, "Chalk"),
        fn("Star", {"type": "Star", "a": -1.0, "sphere_radius": 1.6}, (0, 1.6, 0), (0, 45, 10), 1.0, "Glass"),
        fn("Hunts", {"type": "HuntsSurface", "sphere_radius": 4.0}, (3, 1.6, 0), (-90, 0, 0), 0.35, "Steel"),
        fn("Cushion", {"type": "Cushion", "sphere_radius": 1.5}, (6, 1.6, 0), (-70, 20, 0), 1.1, "Chalk", depth=3),
        fn("Heart", {"type": "Heart"}, (0, 1.2, -3), (-90, 0, 0), 0.8, "Copper", step=0.005),
    ]
    return {
        "camera": {"position": [0, 3.5, -16], "direction": [0, -0.12, 1], "up": [0, 1, 0], "fov": 40,
                   "focal_length": 1},
        "shapes": shapes,
        "materials": {
            "Ground": lambert((0.45, 0.5, 0.45)),
            "Light": {"type": "DiffuseLight", "emit": solid((6, 6, 6))},
            "Copper": {"type": "Metal", "albedo": solid((0.8, 0.5, 0.3)), "fuzz": 0.2},
            "Chalk": lambert((0.8, 0.8, 0.75)),
            "Glass": {"type": "Dielectric", "index_of_refraction": 1.5},
            "Steel": {"type": "Metal", "albedo": solid((0.6, 0.6, 0.65)), "fuzz": 0},
        },
        "background": [0, 0, 0],
    }


def checker(odd, even, mult=(5, 5, 5)):
    return {"type": "CheckerTexture", "scale": 4.0, "odd": solid(odd), "even": solid(even),
            "multipliers": {"x": mult[0], "y": mult[1], "z": mult[2]}}


def uvchecker(odd, even, mult=(40, 40)):
    return {"type": "UVChecker", "scale": 4.0, "odd": solid(odd), "even": solid(even), "multipliers": list(mult)}


def textured():
    """Every texture of src/world/texture.rs on every shape kind that carries
    u, v: the detached_materials.json arrangement (checker Metal ground, UV-
    checker spheres, an image-mapped Metal sphere, a Cushion) plus a noise
    sphere, a textured cube and rectangle, and a checker-textured light."""
    shapes = [
        {"type": "Sphere", "name": "Ground", "transform": tr((0, -1000, 0), s=(1000, 1000, 1000)),
         "material": "Ground"},
        {"type": "Sphere", "name": "Ball", "transform": tr((-2.2, 1, 0), (0, 30, 0)), "material": "UV"},
        {"type": "Sphere", "name": "Earth", "transform": tr((0, 1, 0), (0, 0, 0)), "material": "EarthMap"},
        {"type": "Sphere", "name": "Marble", "transform": tr((2.2, 1, 0)), "material": "Marble"},
        {"type": "Cube", "name": "Box", "transform": tr((-1.1, 0.45, -2.2), (0, 25, 0), (0.45, 0.45, 0.45)),
         "material": "UV"},
        {"type": "Rectangle", "x0": -1, "x1": 1, "y0": 0, "y1": 1.5, "transform": tr((0, 0, 2.5), (0, 180, 0)),
         "material": "Poster"},
        {"type": "Rectangle", "x0": -2, "x1": 2, "y0": -1, "y1": 1, "transform": tr((0, 5, 0), (90, 0, 0)),
         "material": "Sun"},
        {"type": "BruteForsableShape", "name": "Cushion", "shape": {"type": "Cushion", "sphere_radius": 1.5},
         "step": 0.01, "depth": 3, "transform": tr((1.2, 0.5, -2.4), (-70, 20, 0), (0.45, 0.45, 0.45)),
         "material": "UV"},
    ]
    return {
        "camera": {"position": [0, 2.2, -9], "direction": [0, -0.2, 1], "up": [0, 1, 0], "fov": 40,
                   "focal_length": 1},
        "shapes": shapes,
        "materials": {
            "Ground": {"type": "Metal", "albedo": checker((0.1, 0.2, 0.8), (0.9, 0.2, 0.1)), "fuzz": 0.0},
            "UV": {"type": "Lambertian", "albedo": uvchecker((0.1, 0.9, 0.9), (0.9, 0.1, 0.9))},
            "EarthMap": {"type": "Metal", "albedo": {"type": "ImageTexture",
                                                     "image_filename": "./scenes/textures/grid.ppm"}, "fuzz": 1},
            "Poster": {"type": "Lambertian", "albedo": {"type": "ImageTexture",
                                                        "image_filename": "./scenes/textures/grid.ppm"}},
            "Marble": {"type": "Lambertian", "albedo": {"type": "NoiseTexture", "scale": 4.0}},
            "Sun": {"type": "DiffuseLight", "emit": checker((4, 4, 4), (9, 8, 7), (3, 3, 3))},
        },
        "background": [0, 0, 0],
    }


def noise():
    """light_source.json's arrangement: NoiseTexture ground and sphere under a
    rectangle light (no ray-marched shape)."""
    return {
        "camera": {"position": [13, 2, 3], "direction": [-13, -1, -3], "up": [0, 1, 0], "fov": 30,
                   "focal_length": 1},
        "shapes": [
            {"type": "Rectangle", "x0": -1, "x1": 1, "y0": -1, "y1": 1, "transform": tr((0, 5, -2), (45, 0, 0)),
             "material": "Light"},
            {"type": "Sphere", "name": "Sphere1", "transform": tr((0, 2, 0), s=(2, 2, 2)), "material": "Ground"},
            {"type": "Sphere", "name": "Ground", "transform": tr((0, -1000, 0), s=(1000, 1000, 1000)),
             "material": "Ground"},
        ],
        "materials": {
            "Ground": {"type": "Lambertian", "albedo": {"type": "NoiseTexture", "scale": 4.0}},
            "Light": {"type": "DiffuseLight", "emit": solid((4, 4, 4))},
        },
        "background": [0, 0, 0],
    }


def torus():
    """Tori (src/world/shapes/mod.rs:400-494; no reference scene uses one): a
    lying ring, a standing UV-checked ring and a glass one over a ground."""
    def ring(name, t, r, scale, mat, R=1.0, tube=0.3):
        return {"type": "Torus", "name": name, "radius": R, "tube_radius": tube,
                "transform": tr(t, r, (scale, scale, scale)), "material": mat}
    return {
        "camera": {"position": [0, 3, -10], "direction": [0, -0.25, 1], "up": [0, 1, 0], "fov": 35,
                   "focal_length": 1},
        "shapes": [
            {"type": "Sphere", "name": "Ground", "transform": tr((0, -1000, 0), s=(1000, 1000, 1000)),
             "material": "Ground"},
            ring("Flat", (-2.5, 0.3, 0), (90, 0, 0), 1.0, "Copper"),
            ring("Standing", (0, 1.3, 0.5), (0, 30, 0), 1.0, "UV", R=1.0, tube=0.25),
            ring("Glassy", (2.6, 0.6, -0.5), (60, -20, 0), 0.8, "Glass", R=0.9, tube=0.35),
            {"type": "Rectangle", "x0": -3, "x1": 3, "y0": -2, "y1": 2, "transform": tr((0, 7, 0), (90, 0, 0)),
             "material": "Light"},
        ],
        "materials": {
            "Ground": lambert((0.5, 0.55, 0.5)),
            "Copper": {"type": "Metal", "albedo": solid((0.8, 0.5, 0.3)), "fuzz": 0.1},
            "UV": {"type": "Lambertian", "albedo": uvchecker((0.9, 0.9, 0.2), (0.2, 0.3, 0.9), (16, 16))},
            "Glass": {"type": "Dielectric", "index_of_refraction": 1.5},
            "Light": {"type": "DiffuseLight", "emit": solid((5, 5, 5))},
        },
        "background": [0, 0, 0],
    }


def grid_ppm(w=64, h=32):
    """A small RGB test image (binary PPM): a colour ramp with a grid, so that
    every texel of an image-mapped sphere is distinguishable."""
    px = bytearray()
    for y in range(h):
        for x in range(w):
            line = x % 8 == 0 or y % 8 == 0
            px += bytes((255, 255, 255) if line else ((x * 4) % 256, (y * 8) % 256, (x * y) % 256))
    return b"P6\n%d %d\n255\n" % (w, h) + bytes(px)


def synthetic(n, seed=1):
    """C5: n small spheres on a jittered grid (add_random_spheres recipe scaled up,
    json_models.rs:73-133), a Lambertian ground sphere and the spheres.json camera."""
    rng = random.Random(seed)
    side = int(round(n ** 0.5))
    mats = {"Ground": lambert((0.5, 0.5, 0.5))}
    shapes = [{"type": "Sphere", "name": "Ground", "transform": tr((0, -1000, 0), s=(1000, 1000, 1000)),
               "material": "Ground"}]
    half = side // 2
    k = 0
    for a in range(-half, side - half):
        for b in range(-half, side - half):
            if k >= n:
                break
            c = (a * 0.5 + 0.45 * rng.random(), 0.2, b * 0.5 + 0.45 * rng.random())
            roll = rng.random()
            name = "M%d" % k
            if roll < 0.8:
                col = [rng.random() ** 2 for _ in range(3)]
                mats[name] = lambert(col)
            elif roll < 0.95:
                mats[name] = {"type": "Metal", "albedo": solid([0.5 * (1 - rng.random()) for _ in range(3)]),
                              "fuzz": 0.5 * rng.random()}
            else:
                mats[name] = {"type": "Dielectric", "index_of_refraction": 1.5}
            shapes.append({"type": "Sphere", "name": "S%d" % k, "transform": tr(c, s=(0.2, 0.2, 0.2)),
                           "material": name})
            k += 1
    return {
        "camera": {"position": [13, 2, 3], "direction": [-13, -2, -3], "up": [0, 1, 0], "fov": 20,
                   "focal_length": 1},
        "shapes": shapes, "materials": mats, "background": [0, 0, 0],
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--synthetic", type=int, default=0)
    a = ap.parse_args()
    (HERE / "cornell_box.json").write_text(json.dumps(cornell(), indent=1) + "\n")
    (HERE / "spheres.json").write_text(json.dumps(spheres(), indent=1) + "\n")
    (HERE / "marched.json").write_text(json.dumps(marched(), indent=1) + "\n")
    (HERE / "textured.json").write_text(json.dumps(textured(), indent=1) + "\n")
    (HERE / "noise.json").write_text(json.dumps(noise(), indent=1) + "\n")
    (HERE / "torus.json").write_text(json.dumps(torus(), indent=1) + "\n")
    (HERE / "textures").mkdir(exist_ok=True)
    (HERE / "textures" / "grid.ppm").write_bytes(grid_ppm())
    if a.synthetic:
        (HERE / ("synthetic_%d.json" % a.synthetic)).write_text(json.dumps(synthetic(a.synthetic)) + "\n")


if __name__ == "__main__":
    main()
