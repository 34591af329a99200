"""Image output of the display-encoded frame (no GPU): pt_write_png writes what
image::save_buffer(.., ColorType::Rgba8) saves in the reference's GUI
(src/bin/main.rs:71-82) — a PNG any reader decodes to the same RGBA bytes —
and pt_write_ppm a binary PPM."""
import struct
import zlib

import numpy as np
import pytest


def read_png(path):
    data = path.read_bytes()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, chunks = 8, []
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        typ = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(typ + body) & 0xFFFFFFFF, typ
        chunks.append((typ, body))
        pos += 12 + n
    assert chunks[0][0] == b"IHDR" and chunks[-1][0] == b"IEND"
    w, h, depth, ctype, comp, filt, inter = struct.unpack(">IIBBBBB", chunks[0][1])
    assert (depth, ctype, comp, filt, inter) == (8, 6, 0, 0, 0)
    raw = zlib.decompress(b"".join(b for t, b in chunks if t == b"IDAT"))
    rows = np.frombuffer(raw, np.uint8).reshape(h, 1 + w * 4)
    assert np.all(rows[:, 0] == 0)  # filter None
    return w, h, rows[:, 1:].reshape(h * w, 4)


@pytest.mark.parametrize("w,h", [(1, 1), (7, 3), (300, 250)])  # 300x250: several stored deflate blocks
def test_png_round_trip(pt, tmp_path, w, h):
    rng = np.random.default_rng(w * h)
    rgba = rng.integers(0, 256, size=(w * h, 4), dtype=np.uint8)
    pt.write_png(tmp_path / "a.png", rgba, w, h)
    gw, gh, px = read_png(tmp_path / "a.png")
    assert (gw, gh) == (w, h)
    assert np.array_equal(px, rgba)


def test_ppm(pt, tmp_path):
    w, h = 5, 4
    rgba = np.arange(w * h * 4, dtype=np.uint8).reshape(-1, 4)
    pt.write_ppm(tmp_path / "a.ppm", rgba, w, h)
    data = (tmp_path / "a.ppm").read_bytes()
    head = b"P6\n5 4\n255\n"
    assert data[:len(head)] == head
    assert np.array_equal(np.frombuffer(data[len(head):], np.uint8).reshape(-1, 3), rgba[:, :3])


def test_encode_then_png_of_an_oracle_frame(pt, tmp_path, cornell_text):
    import oracle as O
    img = O.Scene(cornell_text, seed=1).render(24, 16, 2, 8, 1, threads=2)
    rgba = pt.encode_rgba8(img)
    pt.write_png(tmp_path / "rendered.png", rgba, 24, 16)
    _, _, px = read_png(tmp_path / "rendered.png")
    assert np.array_equal(px, rgba)


def test_bad_arguments(pt, tmp_path):
    with pytest.raises(ValueError):
        pt.write_png(tmp_path / "x.png", np.zeros(3, np.uint8), 1, 1)
    with pytest.raises(pt.PtError):
        pt.write_png(tmp_path / "no_such_dir" / "x.png", np.zeros(4, np.uint8), 1, 1)
