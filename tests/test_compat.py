"""gpu/rt compatibility mode -- host-side tests.

The reference's gpu/rt (gpu/rt.cpp, gpu/raytracer.cu, gpu/light.cu,
gpu/colors.cu) renders at 3x width and height, one ray per high-resolution
pixel, in saturating uint8 colours with at most 11 bounces, box-downscales
3x3 and writes an RGBA PNG.  No gpu/rt output can be produced here (CUDA is
absent and the reference ships no PNG), so this mode is PARITY UNPINNED: the
oracle (oracle_render_gpu) restates the gpu/ sources; these tests pin its
colour algebra by hand-computed known answers, and the PNG writer by a
decoder written here.  GPU-vs-oracle parity: tests/test_gpu.py.
"""
import gzip
import os
import struct
import zlib

import numpy as np

from conftest import GOLDEN

import oracle as orc
import rtgpu


def decode_png(path):
    """Minimal PNG decoder (8-bit RGBA, filter 0 or any of the 5 filters)."""
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, ihdr = 8, b"", None
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        typ = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert zlib.crc32(typ + body) & 0xFFFFFFFF == crc, typ
        if typ == b"IHDR":
            ihdr = struct.unpack(">IIBBBBB", body)
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
        if typ == b"IEND":
            break
    w, h, depth, ctype, comp, filt, inter = ihdr
    assert (depth, ctype, comp, filt, inter) == (8, 6, 0, 0, 0)
    raw = zlib.decompress(idat)
    stride = 4 * w
    out = np.zeros((h, stride), np.uint8)
    prev = np.zeros(stride, np.int32)
    for y in range(h):
        f = raw[y * (stride + 1)]
        line = np.frombuffer(raw, np.uint8, stride, y * (stride + 1) + 1).astype(np.int32)
        assert f == 0, "writer uses filter 0"
        out[y] = line
        prev = line
    return out.reshape(h, w, 4)


def _scene(tmp_path, name, w, h):
    p = tmp_path / f"{name}.svati"
    p.write_bytes(gzip.open(os.path.join(GOLDEN, "scenes", name + ".svati.gz")).read())
    s = rtgpu.Scene.load_svati(str(p))
    s.set_size(w, h)
    return s


def test_png_roundtrip(tmp_path, built):
    rng = np.random.default_rng(7)
    img = rng.integers(0, 256, size=(37, 53, 4), dtype=np.uint8)
    p = tmp_path / "x.png"
    rtgpu.write_png(str(p), img)
    assert np.array_equal(decode_png(str(p)), img)


def _init8(x):
    """gpu/colors.cu:3-20 in float32: x*255, clamp, truncate."""
    y = np.float32(x) * np.float32(255)
    y = min(max(y, np.float32(0)), np.float32(255))
    return int(y)


def _mults8(a, b):
    return _init8((np.float32(a) / np.float32(255)) * (np.float32(b) / np.float32(255)))


def _mul8(a, coef):
    return _init8(np.float32(a) / np.float32(255) * np.float32(coef))


def test_oracle_gpu_mode_ambient_known_answer(tmp_path, built):
    """triangle-ambient (one a_light 0.65, Ka 0.8 0 0): a fully covered
    output pixel is the downscale of nine identical high-resolution pixels
    mul8(mults8(init8(.65), init8(.8)), 1) -- computed here by hand."""
    s = _scene(tmp_path, "triangle-ambient", 32, 32)
    img, cnt = orc.render_gpu(s.ptr, 32, 32, threads=4)
    c = _mul8(_mults8(_init8(0.65), _init8(0.8)), 1.0)
    full = _init8(np.float32(9 * c) / (np.float32(255) * np.float32(3) * np.float32(3)))
    assert (img[..., 3] == 255).all()
    assert (img[..., 1:3] == 0).all()
    assert full in set(np.unique(img[..., 0]).tolist())
    assert 0 in set(np.unique(img[..., 0]).tolist())  # background
    # at most one query per high-resolution pixel (Nr 0: no bounce), no shadows
    assert cnt["closest"] == 9 * 32 * 32 and cnt["shadow"] == 0


def test_oracle_gpu_mode_bounce_cap(tmp_path, built):
    """Two facing perfect mirrors: gpu/raytracer.cu:113-120 stops after 11
    closest-hit queries (MAX_BOUNCE = 10, post-decrement)."""
    # camera rays start on the film, L = 68 behind the eye (cpu/raytracer.c:
    # 82-86), and travel +z: one mirror in front of the eye, one behind the
    # film, both wide enough for the (slowly diverging) bounces
    sv = tmp_path / "mir.svati"
    tri = ("v -{a} -{a} {z}\nv {a} -{a} {z}\nv 0 {a} {z}\nvn 0 0 1\nvn 0 0 1\nvn 0 0 1\n")
    sv.write_text("camera 4 4 0 0 -1 1 0 0 0 -1 0 10\na_light 1 1 1\n\n"
                  "object 3\nKa 0.01 0.01 0.01\nNr 1\n" + tri.format(a=5000, z=1) + "\n"
                  "object 3\nKa 0.01 0.01 0.01\nNr 1\n" + tri.format(a=5000, z=-100))
    s = rtgpu.Scene.load_svati(str(sv))
    _, cnt = orc.render_gpu(s.ptr, 4, 4, threads=2)
    assert cnt["closest"] == 11 * 9 * 16
