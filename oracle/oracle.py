"""oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes access to oracle/_build/liboracle.so, the plain-C restatement of the
reference cpu/rt (oracle/rt_oracle.c).  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this; the product never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")


class Counts(C.Structure):
    _fields_ = [("closest", C.c_ulonglong), ("shadow", C.c_ulonglong),
                ("max_depth", C.c_ulonglong)]


class ColorS(C.Structure):
    _fields_ = [("r", C.c_float), ("g", C.c_float), ("b", C.c_float)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE, "oracle"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.oracle_load_svati.argtypes = [C.c_char_p, C.POINTER(C.c_void_p)]
        L.oracle_load_svati.restype = C.c_int
        L.oracle_free_scene.argtypes = [C.c_void_p]
        L.oracle_free_scene.restype = None
        L.oracle_render.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p,
                                    C.POINTER(Counts)]
        L.oracle_render.restype = C.c_int
        L.oracle_render_gpu.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p,
                                        C.POINTER(Counts)]
        L.oracle_render_gpu.restype = C.c_int
        L.oracle_camera_tri_accepts.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.oracle_camera_tri_accepts.restype = None
        L.oracle_camera_tri_accepts_gpu.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.oracle_camera_tri_accepts_gpu.restype = None
        L.oracle_init_color.argtypes = [C.c_float, C.c_float, C.c_float]
        L.oracle_init_color.restype = ColorS
        L.oracle_color_add.argtypes = [ColorS, ColorS]
        L.oracle_color_add.restype = ColorS
        L.oracle_color_mul.argtypes = [ColorS, C.c_float]
        L.oracle_color_mul.restype = ColorS
        L.oracle_color_mul2.argtypes = [ColorS, ColorS]
        L.oracle_color_mul2.restype = ColorS
        _lib = L
    return _lib


class OracleScene:
    """A scene loaded by the oracle's own restated parser."""

    def __init__(self, path):
        p = C.c_void_p()
        rc = lib().oracle_load_svati(os.fsencode(path), C.byref(p))
        if rc != 0:
            raise RuntimeError(f"oracle_load_svati({path}) = {rc}")
        self.ptr = p

    def set_size(self, width, height):
        # struct or_scene: objects*, size_t, lights*, size_t, camera{int w, int h, ...}
        cam = C.cast(self.ptr.value + 32, C.POINTER(C.c_int))
        cam[0] = width
        cam[1] = height

    def __del__(self):
        if getattr(self, "ptr", None) and _lib is not None:
            _lib.oracle_free_scene(self.ptr)
            self.ptr = None


class DiagQuery(C.Structure):
    """struct or_diag_query (oracle/diag.c)."""
    _fields_ = [("kind", C.c_int), ("depth", C.c_int), ("sample", C.c_int), ("result", C.c_int),
                ("o", C.c_float * 3), ("d", C.c_float * 3), ("obj", C.c_int), ("tri", C.c_int),
                ("dist", C.c_float), ("naccept", C.c_int), ("u", C.c_double), ("v", C.c_double),
                ("cosn", C.c_double), ("need", C.c_double), ("S", C.c_double),
                ("inplane", C.c_double), ("shape", C.c_double), ("kbary", C.c_double)]

    KINDS = ("camera", "reflection", "shadow_dir", "shadow_point")

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["o"] = list(self.o)
        d["d"] = list(self.d)
        d["kind"] = self.KINDS[self.kind]
        return d


_diag = None


def diag_pixel(scene_ptr, row, col, max_queries=512):
    """Every query of one pixel's oracle path with its deciding triangle and
    that triangle's conditioning (oracle/diag.c).  Returns (queries, rgb)."""
    global _diag
    if _diag is None:
        path = os.path.join(HERE, "_build", "liboracle_diag.so")
        if not os.path.exists(path):
            build()
        _diag = C.CDLL(path)
        _diag.oracle_diag_pixel.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                            C.c_void_p]
        _diag.oracle_diag_pixel.restype = C.c_int
    buf = (DiagQuery * max_queries)()
    rgb = np.zeros(3, np.float32)
    ptr = scene_ptr.ptr if isinstance(scene_ptr, OracleScene) else scene_ptr
    if not isinstance(ptr, C.c_void_p):
        ptr = C.cast(ptr, C.c_void_p)
    n = _diag.oracle_diag_pixel(ptr, int(row), int(col), buf, max_queries,
                                rgb.ctypes.data_as(C.c_void_p))
    return [buf[i].as_dict() for i in range(min(n, max_queries))], rgb


def render(scene_ptr, width, height, pixels=None, threads=0):
    """Render with the oracle.  scene_ptr: an oracle scene or a product rt_scene*
    (same C layout).  pixels: None (whole frame, PPM order) or an (N, 2) int
    array of (row, col).  Returns (float32 array (N,3) or (H,W,3), counts dict)."""
    if pixels is None:
        n = width * height
        pix_ptr = None
    else:
        pixels = np.ascontiguousarray(pixels, dtype=np.int32)
        n = len(pixels)
        pix_ptr = pixels.ctypes.data_as(C.c_void_p)
    out = np.zeros((n, 3), np.float32)
    cnt = Counts()
    ptr = scene_ptr.ptr if isinstance(scene_ptr, OracleScene) else scene_ptr
    if not isinstance(ptr, C.c_void_p):
        ptr = C.cast(ptr, C.c_void_p)
    rc = lib().oracle_render(ptr, pix_ptr, n, threads, out.ctypes.data_as(C.c_void_p),
                             C.byref(cnt))
    if rc != 0:
        raise RuntimeError(f"oracle_render = {rc}")
    counts = {"closest": cnt.closest, "shadow": cnt.shadow, "max_depth": cnt.max_depth}
    if pixels is None:
        out = out.reshape(height, width, 3)
    return out, counts


def camera_tri_accepts(scene_ptr, tris, rects, gpu=False):
    """cpu/rt's camera samples of pixel rectangles against one triangle each
    (oracle_camera_tri_accepts).  tris: (n, 6, 3) float32 (vertices, normals
    as rt_scene holds them); rects: (n, 4) (row0, col0, rows, cols).  Returns
    (n, 2): samples accepted, samples passing the a, u, v tests.  gpu: gpu/rt's
    rays, one per pixel of the 3x frame (rects in its pixels)."""
    tris = np.ascontiguousarray(tris, dtype=np.float32)
    rects = np.ascontiguousarray(rects, dtype=np.int32)
    assert tris.shape[1:] == (6, 3) and rects.shape == (len(tris), 4)
    out = np.zeros((len(tris), 2), np.uint64)
    ptr = scene_ptr.ptr if isinstance(scene_ptr, OracleScene) else scene_ptr
    if not isinstance(ptr, C.c_void_p):
        ptr = C.cast(ptr, C.c_void_p)
    fn = lib().oracle_camera_tri_accepts_gpu if gpu else lib().oracle_camera_tri_accepts
    fn(ptr, tris.ctypes.data, rects.ctypes.data, len(tris), out.ctypes.data)
    return out


def render_gpu(scene_ptr, width, height, pixels=None, threads=0):
    """gpu/rt compatibility mode with the oracle (oracle_render_gpu).
    pixels: None (whole W x H image, gpu/rt's PNG row order) or an (N, 2)
    (row, col) array.  Returns (uint8 (N, 4) or (H, W, 4), counts)."""
    if pixels is None:
        n = width * height
        pix_ptr = None
    else:
        pixels = np.ascontiguousarray(pixels, dtype=np.int32)
        n = len(pixels)
        pix_ptr = pixels.ctypes.data_as(C.c_void_p)
    out = np.zeros((n, 4), np.uint8)
    cnt = Counts()
    ptr = scene_ptr.ptr if isinstance(scene_ptr, OracleScene) else scene_ptr
    if not isinstance(ptr, C.c_void_p):
        ptr = C.cast(ptr, C.c_void_p)
    rc = lib().oracle_render_gpu(ptr, pix_ptr, n, threads, out.ctypes.data_as(C.c_void_p),
                                 C.byref(cnt))
    if rc != 0:
        raise RuntimeError(f"oracle_render_gpu = {rc}")
    counts = {"closest": cnt.closest, "shadow": cnt.shadow, "max_depth": cnt.max_depth}
    if pixels is None:
        out = out.reshape(height, width, 4)
    return out, counts
