"""Writes tests/golden/reference_scenes.json: what Scene::from_json
(src/world/mod.rs:46-49, src/world/json_models.rs:23-48) makes of each file of
the reference's own scene set (/root/reference/scenes/*.json), through the
product loader (pt.Scene.from_json, random spheres on, seed 1).

Per file: its sha256, the outcome (ok, or the error the loader reports), the
shape / material counts and a digest of every realized shape (type, material,
flags, both 4x4 matrices, parameters) and material (float.hex).  The scene
files themselves are not copied.  tests/test_reference_scenes.py checks the
loader and the oracle against the files when the checkout is present, and the
re-authored scenes/ against the digests when it is not.

    python tests/golden/make_reference_scenes.py [/root/reference/scenes]
"""
import hashlib
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

# detached_materials.json names a JPEG (ImageTexture); the reference decodes it with image::open, here the
# host's loader hands the pixels over (pt_scene_opts.load_image): a fixed 2x2 image stands in for the decode
STAND_IN_IMAGE = (2, 2, bytes([255, 0, 0, 255, 0, 255, 0, 255, 0, 0, 255, 255, 255, 255, 255, 255]))
SEED = 1


def realized_digest(sc):
    """sha256 over the realized shapes of a product or oracle scene, each with the material it resolves to
    (so unused materials and the materials' file order do not enter), as float.hex text."""
    h = hashlib.sha256()
    for i in range(sc.num_shapes):
        s = sc.shape(i)
        m = sc.material(s.material)
        fields = [s.type, s.inverse_normal] + [float(v).hex() for v in s.direct] + \
                 [float(v).hex() for v in s.inverse] + [float(v).hex() for v in (s.x0, s.y0, s.x1, s.y1, s.step)]
        fields += [m.type] + [float(v).hex() for v in list(m.albedo) + [m.fuzz, m.ior] + list(m.emit)]
        h.update(repr(fields).encode())
    return h.hexdigest()


def outcome(pt, text, images=None):
    try:
        sc = pt.Scene.from_json(text, seed=SEED, images=images)
    except pt.PtError as e:
        return {"outcome": "error", "error": str(e)}
    return {"outcome": "ok", "shapes": sc.num_shapes, "materials": sc.num_materials, "digest": realized_digest(sc)}


def main():
    src = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/scenes")
    import __graft_entry__ as ge
    pt = ge.load_package()
    out = {"seed": SEED, "random_spheres": True, "stand_in_image": list(STAND_IN_IMAGE[:2]), "scenes": {}}
    for f in sorted(src.glob("*.json")):
        text = f.read_text()
        rec = {"sha256": hashlib.sha256(f.read_bytes()).hexdigest()}
        rec.update(outcome(pt, text))
        if "image_filename" in text:
            files = sorted(set(_image_files(json.loads(text))))
            rec["with_loader"] = outcome(pt, text, images={n: STAND_IN_IMAGE for n in files})
            rec["with_loader"]["images"] = files
        out["scenes"][f.name] = rec
    dst = Path(__file__).resolve().parent / "reference_scenes.json"
    dst.write_text(json.dumps(out, indent=1, sort_keys=True) + "\n")
    print("wrote", dst)


def _image_files(node):
    if isinstance(node, dict):
        if node.get("type") == "ImageTexture":
            yield node["image_filename"]
        for v in node.values():
            yield from _image_files(v)
    elif isinstance(node, list):
        for v in node:
            yield from _image_files(v)


if __name__ == "__main__":
    main()
