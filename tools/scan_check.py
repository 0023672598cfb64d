import sys, ctypes as C, numpy as np
sys.path.insert(0, 'raytracing-gpu_amd')
import rtgpu
L = rtgpu.lib()
L.rt_cand_scan.restype = C.c_int
L.rt_cand_scan.argtypes = [C.c_void_p, C.c_void_p, C.c_uint, C.c_void_p, C.POINTER(C.c_size_t), C.c_void_p]
rng = np.random.default_rng(1)
bad = 0
tmp = C.c_void_p()
assert L.rt_hip_malloc(0, 1 << 20, C.byref(tmp)) == 0
for n in [0, 1, 5, 63, 64, 65, 127, 1000, 1023, 1024, 1025, 4096, 5000, 9216, 9233, 16200, 16384, 20000, 32767]:
    x = rng.integers(0, 1000, n + 1).astype(np.uint32)
    di, do = C.c_void_p(), C.c_void_p()
    assert L.rt_hip_malloc(0, 4 * (n + 1), C.byref(di)) == 0
    assert L.rt_hip_malloc(0, 4 * (n + 1), C.byref(do)) == 0
    assert L.rt_hip_memcpy_h2d(di, x.ctypes.data_as(C.c_void_p), 4 * (n + 1)) == 0
    tb = C.c_size_t(1 << 20)
    e = L.rt_cand_scan(di, do, n, tmp, C.byref(tb), None)
    y = np.empty(n + 1, np.uint32)
    assert L.rt_hip_memcpy_d2h(y.ctypes.data_as(C.c_void_p), do, 4 * (n + 1)) == 0
    ref = np.concatenate([[0], np.cumsum(x[:-1], dtype=np.uint64)]).astype(np.uint32)
    ok = np.array_equal(y, ref)
    if not ok:
        bad += 1
        k = np.flatnonzero(y != ref)
        print("n", n, "err", e, "first bad", k[:5], y[k[:3]], ref[k[:3]])
    L.rt_hip_free(di); L.rt_hip_free(do)
print("bad", bad)
