"""rtgpu -- Python view of the C ABI in include/rt_scene.h and include/rt_hip.h.

A thin ctypes binding used by bench.py and the tests; the product is the
shared library lib/librtgpu.so (host C + gfx950 HIP kernels).  There is no
Python or CPU fallback: if the library or a gfx950 device is missing every
render call raises RtError.

Mirrors the reference interface for the path: `raytrace(input, output)`
(cpu/headers/raytracer.h:4) is `raytrace()`, the scene model of
cpu/headers/scene.h:7-55 is `Scene` (same C layout), the per-render query
counters are those of SURVEY.md §8d.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(HERE, "lib")
LIB_PATH = os.environ.get("RTGPU_LIB") or os.path.join(LIB_DIR, "librtgpu.so")

RT_ACCEL_FLAT = 0
RT_ACCEL_OCTREE = 1
RT_ACCEL_OCTREE_GPU = 2
ACCEL = {"flat": RT_ACCEL_FLAT, "octree": RT_ACCEL_OCTREE, "octree_gpu": RT_ACCEL_OCTREE_GPU}


class RtError(RuntimeError):
    def __init__(self, code, what):
        super().__init__(f"{what}: rt error {code}")
        self.code = code


# ---- C layouts (include/rt_scene.h, identical to cpu/headers/scene.h) ----
class Vec3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class Triangle(C.Structure):
    _fields_ = [("vertex", Vec3 * 3), ("normal", Vec3 * 3)]


class Object(C.Structure):
    _fields_ = [("triangles", C.POINTER(Triangle)), ("triangle_count", C.c_uint),
                ("ka", Vec3), ("kd", Vec3), ("ks", Vec3),
                ("ns", C.c_float), ("ni", C.c_float), ("nr", C.c_float), ("d", C.c_float)]


class Light(C.Structure):
    _fields_ = [("type", C.c_int), ("r", C.c_float), ("g", C.c_float), ("b", C.c_float),
                ("v", Vec3)]


class Camera(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("position", Vec3), ("u", Vec3),
                ("v", Vec3), ("fov", C.c_float)]


class SceneStruct(C.Structure):
    _fields_ = [("objects", C.POINTER(Object)), ("object_count", C.c_size_t),
                ("lights", C.POINTER(Light)), ("light_count", C.c_size_t),
                ("camera", Camera)]


class ProbeResult(C.Structure):
    _fields_ = [("queries", C.c_ulonglong), ("hits", C.c_ulonglong),
                ("node_visits", C.c_ulonglong), ("tri_tests", C.c_ulonglong),
                ("max_stack", C.c_ulonglong), ("mismatches", C.c_ulonglong),
                ("shadow_queries", C.c_ulonglong), ("shadow_hits", C.c_ulonglong),
                ("shadow_node_visits", C.c_ulonglong), ("shadow_tri_tests", C.c_ulonglong)]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


class Frame(C.Structure):
    _fields_ = [("u", Vec3), ("v", Vec3), ("C", Vec3), ("position", Vec3),
                ("width", C.c_int), ("height", C.c_int)]


class Stats(C.Structure):
    _fields_ = [("closest", C.c_ulonglong), ("shadow", C.c_ulonglong), ("camera", C.c_ulonglong),
                ("node_visits", C.c_ulonglong), ("tri_tests", C.c_ulonglong),
                ("depth_overflow", C.c_ulonglong), ("zero_normal", C.c_ulonglong),
                ("pixels", C.c_ulonglong), ("hits", C.c_ulonglong),
                ("cand_prims", C.c_ulonglong), ("cand_entries", C.c_ulonglong),
                ("cand_global", C.c_ulonglong),
                ("closest_node_lanes", C.c_ulonglong), ("closest_tri_lanes", C.c_ulonglong),
                ("shadow_node_lanes", C.c_ulonglong), ("shadow_tri_lanes", C.c_ulonglong),
                ("cycles_camera", C.c_ulonglong), ("cycles_cand", C.c_ulonglong),
                ("cycles_secondary", C.c_ulonglong), ("cycles_shadow", C.c_ulonglong),
                ("cycles_shadow_directional", C.c_ulonglong), ("stack_spills", C.c_ulonglong),
                ("shadow_zero_risk", C.c_ulonglong), ("hit_records", C.c_ulonglong),
                ("shadow_node_visits", C.c_ulonglong), ("shadow_tri_tests", C.c_ulonglong),
                ("shadow_unproven", C.c_ulonglong), ("shadow_deferred", C.c_ulonglong),
                ("closest_unproven", C.c_ulonglong)]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


class AccelInfo(C.Structure):
    _fields_ = [("triangles", C.c_ulonglong), ("tri_refs", C.c_ulonglong),
                ("nodes", C.c_ulonglong), ("leaves", C.c_ulonglong), ("max_depth", C.c_ulonglong),
                ("tri_record_bytes", C.c_ulonglong), ("node_record_bytes", C.c_ulonglong),
                ("device_bytes", C.c_ulonglong), ("build_seconds", C.c_double),
                ("max_leaf", C.c_ulonglong), ("shadow_global", C.c_ulonglong),
                ("shadow_mu_max", C.c_double), ("lightbuf_entries", C.c_ulonglong),
                ("lightbuf_global", C.c_ulonglong), ("lightbuf_seconds", C.c_double),
                ("lightbuf_never", C.c_ulonglong), ("lightbuf_band", C.c_ulonglong),
                ("lightbuf_failed", C.c_ulonglong), ("lightbuf_fail_reason", C.c_char * 96),
                ("trace_grid", C.c_int), ("shade_grid", C.c_int),
                ("scene_center", C.c_float * 3), ("scene_radius", C.c_float)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["lightbuf_fail_reason"] = d["lightbuf_fail_reason"].decode(errors="replace")
        d["scene_center"] = list(d["scene_center"])
        return d


# (name, restype, argtypes) for every entry point of include/*.h
_PROTOS = [
    ("rt_strerror", C.c_char_p, [C.c_int]),
    ("rt_last_error", C.c_char_p, []),
    ("rt_scene_load_svati", C.c_int, [C.c_char_p, C.POINTER(C.POINTER(SceneStruct))]),
    ("rt_scene_load_obj", C.c_int, [C.c_char_p, C.POINTER(C.POINTER(SceneStruct))]),
    ("rt_scene_append_obj", C.c_int, [C.POINTER(SceneStruct), C.c_char_p]),
    ("rt_scene_write_svati", C.c_int, [C.POINTER(SceneStruct), C.c_char_p]),
    ("rt_scene_write_obj", C.c_int, [C.POINTER(SceneStruct), C.c_char_p]),
    ("rt_scene_synthetic", C.c_int, [C.c_uint, C.c_uint, C.c_uint, C.c_ulonglong, C.c_int,
                                     C.c_int, C.POINTER(C.POINTER(SceneStruct))]),
    ("rt_scene_synthetic_uv", C.c_int, [C.c_uint, C.c_uint, C.c_uint, C.c_uint, C.c_ulonglong,
                                        C.c_int, C.c_int, C.POINTER(C.POINTER(SceneStruct))]),
    ("rt_scene_triangle_count", C.c_size_t, [C.POINTER(SceneStruct)]),
    ("rt_scene_free", None, [C.POINTER(SceneStruct)]),
    ("rt_ppm_write", C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_void_p]),
    ("rt_png_write_rgba", C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_void_p]),
    ("rt_frame_from_camera", C.c_int, [C.POINTER(Camera), C.POINTER(Frame)]),
    ("rt_accel_build_info", C.c_int, [C.POINTER(SceneStruct), C.c_int, C.POINTER(AccelInfo)]),
    ("rt_accel_validate", C.c_int, [C.POINTER(SceneStruct), C.c_int]),
    ("rt_accel_probe", C.c_int, [C.POINTER(SceneStruct), C.c_int, C.c_int, C.c_int,
                                 C.POINTER(ProbeResult)]),
    ("rt_hip_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("rt_hip_create", C.c_int, [C.c_int, C.POINTER(SceneStruct), C.c_int, C.POINTER(C.c_void_p)]),
    ("rt_hip_accel_info", C.c_int, [C.c_void_p, C.POINTER(AccelInfo)]),
    ("rt_hip_accel_validate", C.c_int, [C.c_void_p]),
    ("rt_hip_destroy", None, [C.c_void_p]),
    ("rt_hip_tiles_per_rank", C.c_int, [C.c_int, C.c_int, C.c_int]),
    ("rt_hip_tile_buffer_floats", C.c_size_t, [C.c_int, C.c_int, C.c_int]),
    ("rt_tile_map_check", C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_ulonglong)]),
    ("rt_hip_render", C.c_int, [C.c_void_p, C.POINTER(Frame), C.c_int, C.c_int, C.c_void_p,
                                C.c_void_p]),
    ("rt_hip_stats", C.c_int, [C.c_void_p, C.POINTER(Stats)]),
    ("rt_hip_frame_check", C.c_int, [C.c_void_p, C.POINTER(C.c_uint), C.POINTER(C.c_uint),
                                     C.POINTER(C.c_ulonglong)]),
    ("rt_hip_set_count_work", C.c_int, [C.c_void_p, C.c_int]),
    ("rt_hip_set_cull_slack", C.c_int, [C.c_void_p, C.c_float]),
    ("rt_hip_set_camera_slack", C.c_int, [C.c_void_p, C.c_float]),
    ("rt_hip_cand_verify", C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    ("rt_hip_cand_verify_compat", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ("rt_hip_cand_tile_entries", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    ("rt_hip_set_cand_item_cap", C.c_int, [C.c_void_p, C.c_uint]),
    ("rt_hip_verify_shadows", C.c_int, [C.c_void_p, C.c_uint, C.POINTER(C.c_ulonglong)]),
    ("rt_hip_verify_shadows_from", C.c_int, [C.c_void_p, C.c_uint, C.c_uint, C.POINTER(C.c_ulonglong)]),
    ("rt_hip_set_exact_camera", C.c_int, [C.c_void_p, C.c_int]),
    ("rt_hip_set_policy", C.c_int, [C.c_void_p, C.c_int]),
    ("rt_hip_set_exact_shadows", C.c_int, [C.c_void_p, C.c_int]),
    ("rt_hip_set_exact_reflections", C.c_int, [C.c_void_p, C.c_int]),
    ("rt_hip_set_light_buffers", C.c_int, [C.c_void_p, C.c_int]),
    ("rt_hip_set_lightbuf_entry_cap", C.c_int, [C.c_void_p, C.c_ulonglong]),
    ("rt_lightbuf_survey", C.c_int, [C.c_void_p, C.c_uint, C.c_int, C.c_uint, C.c_void_p]),
    ("rt_hip_probe_shadows", C.c_int, [C.c_void_p, C.c_uint, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]),
    ("rt_hip_probe_closest", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p,
                                       C.c_void_p]),
    ("rt_hip_tile_cycles", C.c_int, [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_size_t]),
    ("rt_hip_tile_phase_cycles", C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_ulonglong),
                                           C.c_size_t]),
    ("rt_hip_set_timing", C.c_int, [C.c_void_p, C.c_int]),
    ("rt_hip_frame_times", C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_float),
                                     C.POINTER(C.c_float)]),
    ("rt_hip_frame_kernel_times", C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_float),
                                            C.POINTER(C.c_float), C.POINTER(C.c_float)]),
    ("rt_hip_set_camera_bound_scale", C.c_int, [C.c_void_p, C.c_double]),
    ("rt_hip_set_camera_refine", C.c_int, [C.c_void_p, C.c_int]),
    ("rt_cand_refine_sample", C.c_int, [C.POINTER(SceneStruct), C.c_float, C.c_double, C.c_uint, C.c_int,
                                        C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]),
    ("rt_cand_survey", C.c_int, [C.POINTER(SceneStruct), C.c_float, C.c_double, C.c_int, C.c_int,
                                 C.POINTER(C.c_ulonglong)]),
    ("rt_hip_assemble", C.c_int, [C.c_void_p, C.POINTER(Frame), C.c_void_p, C.c_int, C.c_void_p,
                                  C.c_void_p]),
    ("rt_hip_cand_produce", C.c_int, [C.c_void_p, C.POINTER(Frame), C.c_int, C.c_int, C.POINTER(C.c_uint),
                                      C.POINTER(C.c_uint), C.c_void_p]),
    ("rt_hip_cand_exchange_local", C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.POINTER(Frame)]),
    ("rt_hip_cand_send_buffer", C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
    ("rt_hip_cand_consume", C.c_int, [C.c_void_p, C.POINTER(Frame), C.c_int, C.c_int, C.c_void_p, C.c_size_t,
                                      C.c_uint, C.c_void_p]),
    ("rt_hip_render_image", C.c_int, [C.c_void_p, C.POINTER(Frame), C.c_void_p,
                                      C.POINTER(Stats)]),
    ("rt_hip_malloc", C.c_int, [C.c_int, C.c_size_t, C.POINTER(C.c_void_p)]),
    ("rt_hip_free", C.c_int, [C.c_void_p]),
    ("rt_hip_memcpy_d2h", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    ("rt_hip_memcpy_h2d", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    ("rt_hip_memcpy_d2d", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    ("rt_raytrace", C.c_int, [C.c_char_p, C.c_char_p]),
    ("rt_hip_render_compat", C.c_int, [C.c_void_p, C.POINTER(Camera), C.c_void_p,
                                       C.POINTER(Stats)]),
    ("rt_raytrace_gpu", C.c_int, [C.c_char_p, C.c_char_p, C.c_int]),
    ("rt_raytrace_multi", C.c_int, [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.POINTER(Stats),
                                    C.POINTER(C.c_double)]),
    ("rt_raytrace_multi_dev", C.c_int, [C.c_char_p, C.c_char_p, C.c_int, C.POINTER(C.c_int), C.c_int,
                                        C.POINTER(Stats), C.POINTER(C.c_double)]),
]

_lib = None


def build():
    """Compile lib/librtgpu.so and lib/rt for gfx950 (make -C raytracing-gpu_amd)."""
    subprocess.run(["make", "-s", "-j8", "-C", HERE], check=True)


def lib():
    """The loaded product library; raises if it was never built (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RtError(-6, f"{LIB_PATH} missing: run raytracing-gpu_amd/rtgpu.build() "
                              "(make -C raytracing-gpu_amd)")
        L = C.CDLL(LIB_PATH)
        for name, res, args in _PROTOS:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _check(rc, what):
    if rc != 0:
        L = lib()
        raise RtError(rc, f"{what}: {L.rt_strerror(rc).decode()} ({L.rt_last_error().decode()})")


class Scene:
    """Owns an rt_scene* (layout of cpu/headers/scene.h)."""

    def __init__(self, ptr):
        self.ptr = ptr

    @classmethod
    def load_svati(cls, path):
        p = C.POINTER(SceneStruct)()
        _check(lib().rt_scene_load_svati(os.fsencode(path), C.byref(p)), f"load {path}")
        return cls(p)

    @classmethod
    def load_obj(cls, path):
        p = C.POINTER(SceneStruct)()
        _check(lib().rt_scene_load_obj(os.fsencode(path), C.byref(p)), f"load {path}")
        return cls(p)

    @classmethod
    def synthetic(cls, gx=32, gy=32, tris_per_sphere=9766, seed=0x5EED, width=3840, height=2160):
        p = C.POINTER(SceneStruct)()
        _check(lib().rt_scene_synthetic(gx, gy, tris_per_sphere, seed, width, height, C.byref(p)),
               "synthetic scene")
        return cls(p)

    @classmethod
    def synthetic_uv(cls, gx, gy, stacks, slices, seed=0x5EED, width=3840, height=2160):
        """Explicit tessellation (round 1's C5 was 258 stacks x 19 slices)."""
        p = C.POINTER(SceneStruct)()
        _check(lib().rt_scene_synthetic_uv(gx, gy, stacks, slices, seed, width, height,
                                           C.byref(p)), "synthetic scene")
        return cls(p)

    @property
    def s(self):
        return self.ptr.contents

    @property
    def camera(self):
        return self.s.camera

    def set_size(self, width, height):
        """Same effect as rewriting the camera line's width/height."""
        self.s.camera.width = width
        self.s.camera.height = height

    @property
    def triangle_count(self):
        return int(lib().rt_scene_triangle_count(self.ptr))

    def write_svati(self, path):
        _check(lib().rt_scene_write_svati(self.ptr, os.fsencode(path)), f"write {path}")

    def write_obj(self, path):
        _check(lib().rt_scene_write_obj(self.ptr, os.fsencode(path)), f"write {path}")

    def triangles_array(self):
        """All triangles as a (T, 6, 3) float32 array (vertices then normals)."""
        return scene_triangles(self.ptr)

    def materials_array(self):
        return scene_materials(self.ptr)

    def lightbuf_survey(self, light, exact=False, stride=1):
        """Host-only count of light `light`'s buffer (rt_lightbuf_survey)."""
        out = (C.c_ulonglong * 12)()
        _check(lib().rt_lightbuf_survey(self.ptr, int(light), 1 if exact else 0, int(stride), out),
               "lightbuf_survey")
        keys = ("entries", "never", "global", "band", "big", "surveyed", "band_entries", "max_count",
                "max_prim", "entries_gt1024", "entries_65_1024", "prims_gt64")
        return dict(zip(keys, (int(x) for x in out)))

    def frame(self):
        f = Frame()
        cam = Camera()
        C.pointer(cam)[0] = self.s.camera
        _check(lib().rt_frame_from_camera(C.byref(cam), C.byref(f)), "frame")
        return f

    def close(self):
        if self.ptr:
            lib().rt_scene_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _as_scene_ptr(ptr):
    if isinstance(ptr, C.c_void_p):
        return C.cast(ptr, C.POINTER(SceneStruct))
    return ptr


def scene_triangles(ptr):
    """Triangles of any scene with the cpu/headers/scene.h layout (product or
    oracle), as a (T, 6, 3) float32 array: 3 vertices then 3 normals."""
    s = _as_scene_ptr(ptr).contents
    out = []
    for i in range(s.object_count):
        o = s.objects[i]
        n = o.triangle_count
        if n:
            buf = (C.c_float * (18 * n)).from_address(C.addressof(o.triangles.contents))
            out.append(np.frombuffer(buf, dtype=np.float32).reshape(n, 6, 3).copy())
    return np.concatenate(out) if out else np.zeros((0, 6, 3), np.float32)


def scene_materials(ptr):
    """(objects, 13) float32: ka kd ks ns ni nr d per object."""
    s = _as_scene_ptr(ptr).contents
    rows = []
    for i in range(s.object_count):
        o = s.objects[i]
        rows.append([o.ka.x, o.ka.y, o.ka.z, o.kd.x, o.kd.y, o.kd.z, o.ks.x, o.ks.y, o.ks.z,
                     o.ns, o.ni, o.nr, o.d])
    return np.array(rows, np.float32).reshape(-1, 13)


def accel_build_info(scene, accel="octree"):
    i = AccelInfo()
    a = ACCEL[accel] if isinstance(accel, str) else accel
    _check(lib().rt_accel_build_info(scene.ptr, a, C.byref(i)), "accel_build_info")
    return i.as_dict()


def accel_validate(scene, accel="octree"):
    a = ACCEL[accel] if isinstance(accel, str) else accel
    _check(lib().rt_accel_validate(scene.ptr, a), "accel_validate")


def accel_probe(scene, accel="octree", stride=97, check=True):
    r = ProbeResult()
    a = ACCEL[accel] if isinstance(accel, str) else accel
    _check(lib().rt_accel_probe(scene.ptr, a, stride, 1 if check else 0, C.byref(r)), "probe")
    return r.as_dict()


def cand_survey(scene, eps_ulps=64.0, bound_scale=1.0, threads=8, leaves=False):
    """Host-only: {safe, footprint, global, entries} of the camera candidate
    lists of the scene's frame (csrc/rt_cand.hip classify + raster)."""
    out = (C.c_ulonglong * 88)()
    _check(lib().rt_cand_survey(scene.ptr, eps_ulps, bound_scale, threads, 1 if leaves else 0, out),
           "cand_survey")
    r = dict(zip(("safe", "footprint", "global", "entries"), (int(x) for x in out[:4])))
    # the entries the device lists hold with the per-tile refinement (big
    # footprints refined, csrc/rt_cand.hip tile_keep); the big footprints'
    # entries before and after it
    r["refined"] = int(out[68])
    r["big_entries"], r["big_kept"] = int(out[69]), int(out[70])
    # the float fast path (quick_class) and what the f64 classification makes
    # of the prims it lists
    r["quick"] = dict(zip(("listed", "listed_safe_leaf", "listed_safe_other", "listed_no_tiles",
                           "listed_global", "safe", "away", "listed_safe_reach", "listed_safe_steep",
                           "safe_violations"), (int(x) for x in out[71:81])))
    r["hist"] = [(1 << k, int(out[4 + k]), int(out[20 + k])) for k in range(16) if out[4 + k]]
    # footprint prims by how far their T_D box reaches beyond the triangle, in
    # units of the walk's slack: (lower edge 2^(k-8), prims, entries)
    r["growth_hist"] = [(2.0 ** (k - 8) if k else 0.0, int(out[36 + k]), int(out[52 + k]))
                        for k in range(16) if out[36 + k]]
    return r


def cand_refine_sample(scene, stride=1, cap=1 << 20, eps_ulps=64.0, bound_scale=1.0, compat=False):
    """Host-only: every stride-th entry of the refined candidate footprints
    as rows (prim, tile x, tile y, kept) -- csrc/rt_cand.hip tile_keep -- and
    the number sampled (compat: the gpu/rt mode's 3x frame)."""
    import numpy as np
    out = np.zeros((cap, 4), np.uint32)
    n, total = C.c_size_t(0), C.c_size_t(0)
    _check(lib().rt_cand_refine_sample(scene.ptr, eps_ulps, bound_scale, stride, 1 if compat else 0,
                                       out.ctypes.data, cap, C.byref(n), C.byref(total)), "cand_refine_sample")
    return out[:n.value], total.value


def device_count():
    n = C.c_int(0)
    rc = lib().rt_hip_device_count(C.byref(n))
    return n.value if rc == 0 else 0


def tiles_per_rank(width, height, nranks):
    return int(lib().rt_hip_tiles_per_rank(width, height, nranks))


def tile_buffer_floats(width, height, nranks):
    return int(lib().rt_hip_tile_buffer_floats(width, height, nranks))


class Context:
    """One device image of a scene (rt_hip_create); renders through the C ABI."""

    RT_EINEXACT = -11

    def __init__(self, scene: Scene, accel="octree", device=0):
        self.device = device
        self.accel = ACCEL[accel] if isinstance(accel, str) else accel
        self.inexact = False  # a parity-breaking tuning knob was set (A/B runs)
        h = C.c_void_p()
        _check(lib().rt_hip_create(device, scene.ptr, self.accel, C.byref(h)), "rt_hip_create")
        self.h = h

    def _check_render(self, rc, what):
        """RT_EINEXACT is expected after a parity-breaking knob was set."""
        if rc == self.RT_EINEXACT and self.inexact:
            return
        _check(rc, what)

    def info(self):
        i = AccelInfo()
        _check(lib().rt_hip_accel_info(self.h, C.byref(i)), "accel_info")
        return i.as_dict()

    def validate(self):
        """Invariants of the device scene image (rt_hip_accel_validate)."""
        _check(lib().rt_hip_accel_validate(self.h), "accel_validate")

    def set_count_work(self, on=True):
        _check(lib().rt_hip_set_count_work(self.h, 1 if on else 0), "count_work")

    def set_exact_camera(self, on=True):
        _check(lib().rt_hip_set_exact_camera(self.h, 1 if on else 0), "exact_camera")
        if not on:
            self.inexact = True

    def set_timing(self, on=True):
        """HIP events around the candidate lists and the render kernel of
        every render (rt_hip_set_timing); read them with frame_times()."""
        _check(lib().rt_hip_set_timing(self.h, 1 if on else 0), "timing")

    def frame_times(self, n=1):
        """[(lists_ms, render_kernel_ms)] of the last n timed renders, oldest first."""
        a, b = (C.c_float * n)(), (C.c_float * n)()
        _check(lib().rt_hip_frame_times(self.h, n, a, b), "frame_times")
        return list(zip(a, b))

    def kernel_times(self, n=1):
        """[(trace_ms, shade_ms, fold_ms)] of the last n timed renders, oldest first."""
        a, b, c = (C.c_float * n)(), (C.c_float * n)(), (C.c_float * n)()
        _check(lib().rt_hip_frame_kernel_times(self.h, n, a, b, c), "frame_kernel_times")
        return list(zip(a, b, c))

    def tile_cycles(self, n):
        """Per-tile shader clocks of the last instrumented render (numpy uint64)."""
        out = np.zeros(n, dtype=np.uint64)
        _check(lib().rt_hip_tile_cycles(self.h, out.ctypes.data_as(C.POINTER(C.c_ulonglong)), n),
               "tile_cycles")
        return out

    def tile_phase_cycles(self, phase, n):
        """Per-item phase clocks (rt_hip_tile_phase_cycles; numpy uint64)."""
        out = np.zeros(n, dtype=np.uint64)
        _check(lib().rt_hip_tile_phase_cycles(self.h, phase,
                                              out.ctypes.data_as(C.POINTER(C.c_ulonglong)), n),
               "tile_phase_cycles")
        return out

    def set_light_buffers(self, on=True):
        """Light buffers for the default shadow queries (rt_hip_set_light_buffers)."""
        _check(lib().rt_hip_set_light_buffers(self.h, 1 if on else 0), "light_buffers")

    def set_lightbuf_entry_cap(self, cap):
        """Test hook: light-buffer builds of more than `cap` entries fail (0: no cap);
        the buffers are rebuilt now (rt_hip_set_lightbuf_entry_cap)."""
        _check(lib().rt_hip_set_lightbuf_entry_cap(self.h, int(cap)), "lightbuf_entry_cap")

    def probe_shadows(self, light, origins, brute=False):
        """Shadow rays of light `light` from (n, 3) origins: shadowed flags
        through the light buffer, or brute force (rt_hip_probe_shadows)."""
        o = np.ascontiguousarray(origins, dtype=np.float32).reshape(-1, 3)
        out = np.zeros(len(o), np.uint8)
        _check(lib().rt_hip_probe_shadows(self.h, int(light), o.ctypes.data_as(C.c_void_p), len(o),
                                          1 if brute else 0, out.ctypes.data_as(C.c_void_p)),
               "probe_shadows")
        return out.astype(bool)

    def probe_closest(self, origins, dirs, brute=False):
        """Closest hits of (n, 3) rays queried as reflection rays (the per-lane
        octree walk) or by brute force (rt_hip_probe_closest): (prim, dist)
        arrays, prim = 0xffffffff for no hit."""
        o = np.ascontiguousarray(origins, dtype=np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(dirs, dtype=np.float32).reshape(-1, 3)
        assert len(o) == len(d)
        prim = np.zeros(len(o), np.uint32)
        dist = np.zeros(len(o), np.float32)
        _check(lib().rt_hip_probe_closest(self.h, o.ctypes.data_as(C.c_void_p), d.ctypes.data_as(C.c_void_p),
                                          len(o), 1 if brute else 0, prim.ctypes.data_as(C.c_void_p),
                                          dist.ctypes.data_as(C.c_void_p)), "probe_closest")
        return prim, dist

    def set_exact_shadows(self, on=True):
        """Shadow rays exact by proof (rt_hip_set_exact_shadows; default on):
        proven light buffers, the proven walk where a light's queries walk.
        Off: slack-grown buffers, measured against brute force, not proven."""
        _check(lib().rt_hip_set_exact_shadows(self.h, 1 if on else 0), "exact_shadows")

    def set_exact_reflections(self, on=True):
        """Reflection rays exact by proof (rt_hip_set_exact_reflections):
        the reflection walk grows every node's box by the float test's error
        region for the ray (csrc/rt_reflect.hip); the closest-hit probe uses
        the same walk.  Off (the default): the culling slack, tested."""
        _check(lib().rt_hip_set_exact_reflections(self.h, 1 if on else 0), "exact_reflections")

    def set_policy(self, policy):
        """Octree traversal policy (rt_hip_set_policy): 0 default, 1 per-lane,
        2 staged packet, 3 default + staged directional shadows."""
        _check(lib().rt_hip_set_policy(self.h, int(policy)), "policy")

    def set_camera_refine(self, on=True):
        """Per-tile refinement of the big candidate footprints (default on)."""
        _check(lib().rt_hip_set_camera_refine(self.h, 1 if on else 0), "camera_refine")

    def set_camera_bound_scale(self, scale):
        _check(lib().rt_hip_set_camera_bound_scale(self.h, float(scale)), "bound_scale")
        if scale < 1.0:
            self.inexact = True

    def set_cull_slack(self, ulps):
        _check(lib().rt_hip_set_cull_slack(self.h, float(ulps)), "cull_slack")
        if ulps < 64.0:
            self.inexact = True

    def cand_verify(self, frame, rank=0, nranks=1):
        """Host re-derivation of the last render's candidate lists:
        {listed, entries, fp_mismatch, tile_mismatch, global}."""
        out = (C.c_ulonglong * 7)()
        _check(lib().rt_hip_cand_verify(self.h, C.byref(frame), rank, nranks, out), "cand_verify")
        return dict(zip(("listed", "entries", "fp_mismatch", "tile_mismatch", "global",
                         "filter_violation", "filtered"), (int(x) for x in out)))

    def cand_verify_compat(self, camera):
        """cand_verify for the last rt_hip_render_compat of `camera`."""
        out = (C.c_ulonglong * 7)()
        _check(lib().rt_hip_cand_verify_compat(self.h, C.byref(camera), out), "cand_verify_compat")
        return dict(zip(("listed", "entries", "fp_mismatch", "tile_mismatch", "global",
                         "filter_violation", "filtered"), (int(x) for x in out)))

    def verify_shadows(self, stride=1, first=0):
        """Shadow outcomes of the last render's hit records (every stride-th
        per region, from the first-th): the walk vs brute force
        (rt_hip_verify_shadows_from)."""
        out = (C.c_ulonglong * 4)()
        _check(lib().rt_hip_verify_shadows_from(self.h, stride, first, out), "verify_shadows")
        return dict(zip(("records", "queries", "records_differ", "walk_lit_brute_shadowed"),
                        (int(x) for x in out)))

    def cand_tile_entries(self, ntiles):
        """Candidate-list entries per rank-local tile of the last render."""
        out = np.zeros(ntiles, np.uint32)
        _check(lib().rt_hip_cand_tile_entries(self.h, out.ctypes.data_as(C.c_void_p), ntiles),
               "cand_tile_entries")
        return out

    def set_cand_item_cap(self, cap):
        """Test hook: cap the big footprints' emission work items (0: one
        wave per footprint, the fallback path)."""
        _check(lib().rt_hip_set_cand_item_cap(self.h, int(cap)), "cand_item_cap")

    def set_camera_slack(self, ulps):
        _check(lib().rt_hip_set_camera_slack(self.h, float(ulps)), "camera_slack")

    def render(self, frame, rank, nranks, d_tiles, stream=None):
        _check(lib().rt_hip_render(self.h, C.byref(frame), rank, nranks, C.c_void_p(d_tiles),
                                   C.c_void_p(stream) if stream else None), "rt_hip_render")

    def stats(self):
        st = Stats()
        self._check_render(lib().rt_hip_stats(self.h, C.byref(st)), "rt_hip_stats")
        return st.as_dict()

    # rt_hip_frame_check flag bits (csrc/rt_kernels.h RT_FRAME_*)
    FRAME_FLAGS = {1: "hit records past the buffer (RT_EHITBUF)", 2: "bounce limit / stack overflow (RT_EDEPTH)",
                   4: "zero interpolated normal (RT_EZERONORMAL)", 8: "undecided exact shadow queries (RT_EINEXACT)",
                   16: "asynchronous list build overflow (RT_EHITBUF)"}

    def frame_check(self):
        """(flags, frames, closest, shadow): the per-frame completeness checks
        of every render since the last call, ORed (0 = every frame complete,
        FRAME_FLAGS names the bits), the renders checked and their summed
        closest-hit / shadow queries (rt_hip_frame_check); all reset."""
        fl, n, q = C.c_uint(), C.c_uint(), (C.c_ulonglong * 2)()
        _check(lib().rt_hip_frame_check(self.h, C.byref(fl), C.byref(n), q), "rt_hip_frame_check")
        return int(fl.value), int(n.value), int(q[0]), int(q[1])

    def cand_produce(self, frame, rank, nranks, stream=None):
        """Triangle-parallel lists, step 1 (rt_hip_cand_produce): this rank's
        slice of the prims over the whole frame, routed by destination rank.
        Returns (counts per destination rank, this slice's global prims)."""
        counts = (C.c_uint * nranks)()
        ng = C.c_uint()
        _check(lib().rt_hip_cand_produce(self.h, C.byref(frame), rank, nranks, counts, C.byref(ng),
                                         C.c_void_p(stream) if stream else None), "rt_hip_cand_produce")
        return [int(x) for x in counts], int(ng.value)

    def cand_send_buffer(self):
        """(device pointer, entries) of the last produce's routed entries
        (3 x uint32 each, destination-rank order)."""
        ptr, n = C.c_void_p(), C.c_size_t()
        _check(lib().rt_hip_cand_send_buffer(self.h, C.byref(ptr), C.byref(n)), "rt_hip_cand_send_buffer")
        return ptr.value or 0, int(n.value)

    def cand_consume(self, frame, rank, nranks, d_entries, n, nglobal, stream=None):
        """Step 4: this rank's lists from the n received entries; the next
        render of (frame, rank, nranks) uses them (rt_hip_cand_consume)."""
        _check(lib().rt_hip_cand_consume(self.h, C.byref(frame), rank, nranks, C.c_void_p(d_entries), n, nglobal,
                                         C.c_void_p(stream) if stream else None), "rt_hip_cand_consume")

    def assemble(self, frame, d_gathered, nranks, d_rgb, stream=None):
        _check(lib().rt_hip_assemble(self.h, C.byref(frame), C.c_void_p(d_gathered), nranks,
                                     C.c_void_p(d_rgb), C.c_void_p(stream) if stream else None),
               "rt_hip_assemble")

    def render_image(self, frame):
        """Whole frame on this device -> (H, W, 3) float32 in PPM order, stats."""
        img = np.empty((frame.height, frame.width, 3), np.float32)
        st = Stats()
        self._check_render(lib().rt_hip_render_image(self.h, C.byref(frame),
                                                     img.ctypes.data_as(C.c_void_p), C.byref(st)),
                           "rt_hip_render_image")
        return img, st.as_dict()

    def render_compat(self, camera):
        """gpu/rt compatibility mode (rt_hip_render_compat) -> (H, W, 4)
        uint8 RGBA in gpu/rt's PNG row order, stats."""
        img = np.empty((camera.height, camera.width, 4), np.uint8)
        st = Stats()
        cam = Camera()
        C.pointer(cam)[0] = camera
        self._check_render(lib().rt_hip_render_compat(self.h, C.byref(cam), img.ctypes.data_as(C.c_void_p),
                                                      C.byref(st)), "rt_hip_render_compat")
        return img, st.as_dict()

    def close(self):
        if self.h:
            lib().rt_hip_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def cand_exchange_local(contexts, frame):
    """Triangle-parallel lists of an len(contexts)-rank frame in this process
    (rt_hip_cand_exchange_local): contexts[r] produces rank r's slice, the
    blocks move by device memcpy, every rank consumes its own; each context's
    next render(frame, r, n) uses them.  The exchange rt_raytrace_multi makes
    over RCCL from 4 GPUs up, drivable with every context on one GPU."""
    arr = (C.c_void_p * len(contexts))(*[c.h for c in contexts])
    _check(lib().rt_hip_cand_exchange_local(arr, len(contexts), C.byref(frame)), "rt_hip_cand_exchange_local")


def exchange_cand_entries(dist, send, counts, nglobal):
    """Step 3 of the triangle-parallel lists (include/rt_hip.h
    rt_hip_cand_produce): the all-to-all of the routed entries over
    torch.distributed (RCCL for device tensors, gloo for host tensors).
    send: (sum(counts), 3) int32 tensor in destination-rank order; counts:
    entries for each rank; nglobal: this rank's global prims.  Returns (the
    (n, 3) int32 entries this rank receives, in source-rank order, and the
    producers' global prims summed).  Two collectives: the (count, globals)
    pairs, then the entries."""
    import torch
    w = len(counts)
    meta = torch.tensor([[int(c), int(nglobal)] for c in counts], dtype=torch.int64,
                        device=send.device).reshape(-1)
    rmeta = torch.empty_like(meta)
    dist.all_to_all_single(rmeta, meta)
    rm = rmeta.view(w, 2).tolist()
    rc = [int(a) for a, _ in rm]
    recv = torch.empty((sum(rc), 3), dtype=torch.int32, device=send.device)
    dist.all_to_all_single(recv, send[: sum(counts)], output_split_sizes=rc,
                           input_split_sizes=[int(c) for c in counts])
    return recv, sum(int(b) for _, b in rm)


def write_ppm(path, rgb):
    rgb = np.ascontiguousarray(rgb, dtype=np.float32)
    h, w, _ = rgb.shape
    _check(lib().rt_ppm_write(os.fsencode(path), w, h, rgb.ctypes.data_as(C.c_void_p)), "ppm")


def write_png(path, rgba):
    """8-bit RGBA PNG (rt_png_write_rgba); rgba = (H, W, 4) uint8."""
    rgba = np.ascontiguousarray(rgba, dtype=np.uint8)
    h, w, _ = rgba.shape
    _check(lib().rt_png_write_rgba(os.fsencode(path), w, h, rgba.ctypes.data_as(C.c_void_p)), "png")


def raytrace_gpu(input_path, output_path, accel=None):
    """Drop-in for gpu/rt's main (gpu/rt.cpp:56-97): PNG in compatibility mode."""
    a = -1 if accel is None else (ACCEL[accel] if isinstance(accel, str) else accel)
    _check(lib().rt_raytrace_gpu(os.fsencode(input_path), os.fsencode(output_path), a),
           "rt_raytrace_gpu")


def raytrace_devices(input_path, output_path, devices, accel=None):
    """rt_raytrace_multi_dev: rank g on device devices[g] (a device shared by
    several ranks: memcpy transport in place of RCCL); (stats, render_ms)."""
    st = Stats()
    ms = C.c_double(0)
    a = -1 if accel is None else (ACCEL[accel] if isinstance(accel, str) else accel)
    devs = (C.c_int * len(devices))(*devices)
    _check(lib().rt_raytrace_multi_dev(os.fsencode(input_path), os.fsencode(output_path), len(devices), devs, a,
                                       C.byref(st), C.byref(ms)), "rt_raytrace_multi_dev")
    return st.as_dict(), ms.value


def raytrace(input_path, output_path, gpus=1, accel=None):
    """Drop-in for raytrace() (cpu/raytracer.c:79-136); returns (stats, render_ms)."""
    st = Stats()
    ms = C.c_double(0)
    a = -1 if accel is None else (ACCEL[accel] if isinstance(accel, str) else accel)
    _check(lib().rt_raytrace_multi(os.fsencode(input_path), os.fsencode(output_path), gpus, a,
                                   C.byref(st), C.byref(ms)), "rt_raytrace")
    return st.as_dict(), ms.value


# ---- tile map (host mirror of csrc/rt_tiles.h) ----
def block_side(nranks):
    """Tiles per block side: 4 when the frame is split, 1 (plain scanline
    tiles) for one rank.  Block (bx, by) belongs to rank (bx + by) % nranks;
    a rank's buffer holds its blocks in scanline order."""
    return 4 if nranks > 1 else 1


def _blocks(width, height, nranks):
    tb = block_side(nranks)
    tx, ty = (width + 7) // 8, (height + 7) // 8
    return tb, -(-tx // tb), -(-ty // tb)


def _rank_block_grid(width, height, nranks):
    """(blocks_y, blocks_x) arrays: each block's rank and rank-local index."""
    tb, bx, by = _blocks(width, height, nranks)
    x = np.arange(bx)[None, :]
    y = np.arange(by)[:, None]
    rank = (x + y) % nranks
    local = np.zeros((by, bx), np.int64)
    for r in range(nranks):
        m = (rank == r).ravel()
        local.ravel()[m] = np.arange(int(m.sum()))
    return rank, local


def rank_tile_count(width, height, rank, nranks):
    """Tiles (whole blocks, edge padding included) rank `rank` renders."""
    tb = block_side(nranks)
    rk, _ = _rank_block_grid(width, height, nranks)
    return int((rk == rank).sum()) * tb * tb


def tiles_per_rank_host(width, height, nranks):
    """The most tiles any rank holds (the tile buffers' stride)."""
    return max(rank_tile_count(width, height, r, nranks) for r in range(nranks))


def tile_xy(t, rank, nranks, width, height):
    """(tx, ty) of rank-local tiles t (numpy arrays) of rank `rank`."""
    tb = block_side(nranks)
    rk, _ = _rank_block_grid(width, height, nranks)
    ys, xs = np.nonzero(rk == rank)  # scanline order = the rank's block order
    t = np.asarray(t)
    j, k = t // (tb * tb), t % (tb * tb)
    return xs[j] * tb + k % tb, ys[j] * tb + k // tb


def tile_local(tx, ty, nranks, width, height):
    """(rank, local index) of tiles (tx, ty) (numpy arrays)."""
    tb = block_side(nranks)
    rk, loc = _rank_block_grid(width, height, nranks)
    tx, ty = np.asarray(tx), np.asarray(ty)
    bx, by = tx // tb, ty // tb
    return rk[by, bx], loc[by, bx] * (tb * tb) + (ty % tb) * tb + tx % tb


def tile_pixels(width, height, rank, nranks):
    """(tiles, 64, 2) PPM (row, col) of the rank's tile-buffer slots, -1 where
    the slot is padding (past the frame's edge)."""
    n = rank_tile_count(width, height, rank, nranks)
    tx, ty = tile_xy(np.arange(n), rank, nranks, width, height)
    lane = np.arange(64)
    r = ty[:, None] * 8 + (lane // 8)[None, :]
    c = tx[:, None] * 8 + (lane % 8)[None, :]
    bad = (r >= height) | (c >= width)
    return np.stack([np.where(bad, -1, r), np.where(bad, -1, c)], axis=2)


def assemble_tiles_numpy(gathered, width, height, nranks):
    """Host mirror of the assemble kernel's index map (for CPU tests of the
    tiling / gather layout): gathered = nranks x tiles_per_rank x 64 x 3."""
    tpr = tiles_per_rank_host(width, height, nranks)
    g = np.asarray(gathered, np.float32).reshape(nranks, tpr, 64, 3)
    rows, cols = np.mgrid[0:height, 0:width]
    rk, loc = tile_local(cols // 8, rows // 8, nranks, width, height)
    lane = (rows % 8) * 8 + (cols % 8)
    return g[rk, loc, lane]


def tiles_from_image_numpy(img, rank, nranks):
    """Host mirror of what rank `rank` renders: its tile buffer
    (tiles_per_rank x 64 x 3, zero-padded) cut from a full (H, W, 3) image."""
    img = np.asarray(img, np.float32)
    height, width, _ = img.shape
    tpr = tiles_per_rank_host(width, height, nranks)
    out = np.zeros((tpr, 64, 3), np.float32)
    pix = tile_pixels(width, height, rank, nranks)
    ok = pix[..., 0] >= 0
    out[: len(pix)][ok] = img[pix[..., 0][ok], pix[..., 1][ok]]
    return out
