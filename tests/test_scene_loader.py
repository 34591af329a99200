"""Product scene realization (C++ Scene::from_json) vs the oracle's, and the
loader's error behaviour.  Host code only: runs without a GPU."""
import json

import numpy as np
import pytest

import oracle as O


def product(pt, text, **kw):
    return pt.Scene.from_json(text, **kw)


@pytest.mark.parametrize("name", ["cornell_box.json", "spheres.json"])
@pytest.mark.parametrize("random_spheres", [True, False])
def test_realized_scene_matches_oracle(pt, name, random_spheres):
    from conftest import scene_text
    text = scene_text(name)
    p = product(pt, text, random_spheres=random_spheres, seed=5)
    o = O.Scene(text, random_spheres=random_spheres, seed=5)
    assert p.num_shapes == o.num_shapes
    assert p.num_materials == o.num_materials
    # JSON materials are indexed in file order by both
    for i in range(p.num_shapes):
        a, b = p.shape(i), o.shape(i)
        assert a.type == b.type and a.inverse_normal == b.inverse_normal
        assert list(a.direct) == list(b.direct), i  # bit-exact matrices
        assert list(a.inverse) == list(b.inverse), i
        assert (a.x0, a.y0, a.x1, a.y1, a.step) == (b.x0, b.y0, b.x1, b.y1, b.step)
        ma, mb = p.material(a.material), o.material(b.material)
        assert ma.type == mb.type
        assert list(ma.albedo) == list(mb.albedo) and ma.fuzz == mb.fuzz and ma.ior == mb.ior
        assert list(ma.emit) == list(mb.emit)
    if random_spheres:
        assert p.num_shapes > o.n_json_shapes + 400  # ~480 spheres appended (json_models.rs:44)


def test_random_spheres_depend_on_seed(pt, cornell_text):
    a = product(pt, cornell_text, seed=1)
    b = product(pt, cornell_text, seed=2)
    assert list(a.shape(20).direct) != list(b.shape(20).direct)


def test_camera_matches_oracle(pt, cornell_text):
    p = product(pt, cornell_text).camera()
    o = O.Scene(cornell_text).camera()
    for f in ("position", "direction", "up", "right"):
        assert list(getattr(p, f)) == list(getattr(o, f))
    assert p.fov == o.fov and p.focal_length == o.focal_length
    # cornell: dir (0,0,1), up (0,1,0) -> right (-1,0,0)  
    assert list(p.right) == [-1.0, 0.0, 0.0]


def test_camera_new(pt):
    c = pt.Camera.new([0, 0, 0], [0, 0, -1], [0, 1, 0], 1.0, np.pi / 2)
    assert list(c.right) == [1.0, 0.0, 0.0]


def base_scene():
    return {"camera": {"position": [0, 0, 0], "direction": [0, 0, 1], "up": [0, 1, 0], "fov": 40,
                       "focal_length": 1},
            "shapes": [{"type": "Sphere", "name": "S", "material": "M",
                        "transform": {"translate": [0, 0, 5], "rotate": [0, 0, 0], "scale": [1, 1, 1]}}],
            "materials": {"M": {"type": "Lambertian", "albedo": {"type": "SolidColor", "color": [1, 0, 0]}}},
            "background": [0, 0, 0]}


def expect(pt, js, code, random_spheres=False):
    with pytest.raises(pt.PtError) as e:
        pt.Scene.from_json(js if isinstance(js, str) else json.dumps(js), random_spheres=random_spheres)
    assert e.value.code == code, str(e.value)
    return str(e.value)


def test_errors(pt):
    expect(pt, "{not json", pt.PT_ERR_PARSE)
    js = base_scene()
    js["shapes"][0]["material"] = "Nope"  # reference panics on the HashMap index (shapes/mod.rs:760)
    assert "Nope" in expect(pt, js, pt.PT_ERR_INVALID)
    js = base_scene()
    del js["background"]  # SceneJson::background is required
    assert "background" in expect(pt, js, pt.PT_ERR_PARSE)
    js = base_scene()
    js["shapes"][0]["transform"]["skew"] = [1, 2, 3]  # custom visitor rejects unknown keys
    expect(pt, js, pt.PT_ERR_PARSE)
    js = base_scene()
    js["shapes"][0]["type"] = "Torus"
    js["shapes"][0].update(radius=1)  # tube_radius is required
    assert "tube_radius" in expect(pt, js, pt.PT_ERR_PARSE)
    js = base_scene()
    js["materials"]["M"]["albedo"] = {"type": "NoiseTexture"}  # `scale` is required
    assert "scale" in expect(pt, js, pt.PT_ERR_PARSE)
    js = base_scene()
    js["materials"]["M"]["albedo"] = {"type": "ImageTexture", "image_filename": "/nonexistent/earthmap.jpg"}
    assert "earthmap.jpg" in expect(pt, js, pt.PT_ERR_UNSUPPORTED)  # no loader: PPM only
    js = base_scene()
    js["shapes"][0]["type"] = "Banana"
    expect(pt, js, pt.PT_ERR_PARSE)
    js = base_scene()
    js["shapes"] = []  # BvhNode::new panics on an empty list
    expect(pt, js, pt.PT_ERR_INVALID)
    js["shapes"] = []
    pt.Scene.from_json(json.dumps(js), random_spheres=True)  # empty.json loads: random spheres added


def test_schema_variants(pt):
    js = base_scene()
    js["shapes"][0]["transform"] = {"translate": {"x": 0, "y": 0, "z": 5}, "rotate": [0, 0, 0],
                                    "scale": {"x": 1, "y": 1, "z": 1}}
    js["shapes"][0]["unknown_key"] = 7  # serde ignores unknown struct keys
    js["shapes"].append({"type": "BruteForsableShape", "material": "M", "shape": {"type": "Heart"}, "step": 0.01,
                         "transform": {"translate": [0, 0, 9], "rotate": [0, 0, 0], "scale": [1, 1, 1]}})
    sc = pt.Scene.from_json(json.dumps(js), random_spheres=False)
    assert sc.num_shapes == 2
    assert sc.shape(1).depth == 4  # default_depth (ray_marching.rs:528-530)
    o = O.Scene(json.dumps(js), random_spheres=False)
    assert list(sc.shape(0).direct) == list(o.shape(0).direct)
