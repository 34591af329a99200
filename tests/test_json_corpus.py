"""Malformed-input corpus for Scene::from_json (the C-ABI's JSON reader,
pt_json.hpp, and the scene realization, pt_scene.cpp).  The reference parses
with serde_json and returns its error (src/world/mod.rs:46-49); the library
must return a status and a message for every malformed file and never crash,
read out of bounds or overflow its stack.  scripts/san.sh runs this file (with
the rest of the CPU suite) on the ASan + UBSan build, where any invalid memory
access aborts the run.

The corpus is generated deterministically from the repo's own scenes:
truncations at many offsets, single-byte substitutions and deletions, deep
nesting, numbers out of range, broken escapes and invalid UTF-8, and type
confusions in every schema field.  Host code only: runs without a GPU.
"""
import json

import numpy as np
import pytest

from conftest import ROOT

SCENES = ["cornell_box.json", "spheres.json", "textured.json", "marched.json", "torus.json", "noise.json"]
BYTES_OF_NOTE = b'{}[]",:-+.eE0123456789\\ntfu\x00\x7f\xff'


def load(pt, raw):
    """PT_OK or a PtError with a message; anything else (a crash, another exception) fails the test."""
    try:
        sc = pt.Scene.from_json(raw, seed=1)
    except pt.PtError as e:
        assert str(e), "an error without a message"
        return False
    assert sc.num_shapes >= 0
    return True


def texts():
    return {n: (ROOT / "scenes" / n).read_bytes() for n in SCENES}


@pytest.mark.parametrize("name", SCENES)
def test_truncations(pt, name):
    raw = texts()[name].rstrip()
    cuts = sorted(set(np.linspace(0, len(raw) - 1, 160).astype(int).tolist()))  # all short of the closing brace
    ok = sum(load(pt, raw[:c]) for c in cuts)
    assert ok == 0  # a scene cut short is never valid JSON
    assert load(pt, raw)


@pytest.mark.parametrize("name", SCENES)
def test_byte_substitutions_and_deletions(pt, name):
    raw = texts()[name]
    rng = np.random.default_rng(hash(name) % 2**32)
    for _ in range(150):
        i = int(rng.integers(len(raw)))
        b = BYTES_OF_NOTE[int(rng.integers(len(BYTES_OF_NOTE)))]
        load(pt, raw[:i] + bytes([b]) + raw[i + 1:])
        load(pt, raw[:i] + raw[i + 1:])
        load(pt, raw[:i] + raw[i:i + 17] + raw[i:])


def test_nesting_depth_is_bounded(pt):
    """serde_json stops at 128 levels ("recursion limit exceeded"); so does the
    reader, so a hostile file cannot exhaust the caller's stack."""
    for opener in (b"[", b'{"a":'):
        with pytest.raises(pt.PtError, match="recursion limit"):
            pt.Scene.from_json(opener * 200000, seed=1)
    deep_ok = b"[" * 127 + b"1" + b"]" * 127
    with pytest.raises(pt.PtError, match="SceneJson"):
        pt.Scene.from_json(deep_ok, seed=1)  # parses, then fails the schema (not a scene object)


def test_numbers_strings_and_encodings(pt):
    base = json.loads(texts()["cornell_box.json"])
    base["camera"]["fov"] = 12345.678  # a sentinel the number cases replace
    text = json.dumps(base)
    cases = []
    for v in ["1e400", "-1e400", "1e-400", "-0.0", "4.9e-324", "1" * 400, "0." + "0" * 400 + "1", "01", "1.",
              "-", ".5", "1e", "+1", "NaN", "Infinity", "0x10", "1_000"]:
        cases.append(text.replace("12345.678", v).encode())
    for s in ['"\\u12"', '"\\ud800"', '"\\udc00"', '"\\ud800\\u0041"', '"\\x41"', '"\\', '"abc', '"\t"',
              '"\\u0000"', '"\\ud83d\\ude00"']:
        cases.append(b'{"camera": ' + s.encode() + b"}")
    cases += [b"", b" ", b"\xef\xbb\xbf{}", b"\xff\xfe{", b'{"\xc3":1}', b"{\x00}", b"nul", b"tru", b"[1,]",
              b'{"a":1,}', b'{"a" 1}', b"{1:2}", b"[" + b"1," * 100000 + b"1]"]
    for raw in cases:
        load(pt, raw)
    with pytest.raises(pt.PtError, match="number out of range"):  # serde_json's overflow error
        pt.Scene.from_json(text.replace("12345.678", "1e400"), seed=1)
    sc = pt.Scene.from_json(text.replace("12345.678", "1e-400"), seed=1)  # an underflow is zero, as in serde
    assert sc.camera().fov == 0.0


MISSING = object()


def _mutations(node, path=()):
    """Every schema field replaced by values of the wrong type / shape, or left out."""
    wrong = [None, True, "s", 1, -1, 1.5e308, [], [1], [1, 2], [1, 2, 3, 4], {}, {"x": 1}, MISSING]
    if isinstance(node, dict):
        for k, v in node.items():
            for w in wrong:
                yield path + (k,), w
            yield from _mutations(v, path + (k,))
    elif isinstance(node, list):
        for i, v in enumerate(node[:3]):
            yield from _mutations(v, path + (i,))


def _replace(doc, path, value):
    doc = json.loads(json.dumps(doc))
    cur = doc
    for p in path[:-1]:
        cur = cur[p]
    if value is MISSING:
        del cur[path[-1]]
    else:
        cur[path[-1]] = value
    return doc


@pytest.mark.parametrize("name", ["cornell_box.json", "textured.json", "marched.json"])
def test_schema_type_confusions(pt, name):
    """Wrong types, wrong array lengths and missing keys in every field: an
    error status (or a scene, where serde would accept the value too), never a
    crash.  Shapes and materials lists are cut to their first entries."""
    doc = json.loads(texts()[name])
    doc["shapes"] = doc["shapes"][:3]
    n = 0
    for path, w in _mutations(doc):
        load(pt, json.dumps(_replace(doc, path, w)).encode())
        n += 1
    assert n > 300
