"""Host C side of the product, no GPU: loaders, printer, writers, octree build,
and the C-ABI library's exported surface."""
import ctypes as C
import hashlib
import os
import re

import numpy as np
import pytest

from conftest import REPO, case_id, golden_image, load_manifest_static

SCENES = sorted(f[:-9] for f in os.listdir(os.path.join(REPO, "tests", "golden", "scenes"))
                if f.endswith(".svati.gz"))
CASES = load_manifest_static()


def _header_functions():
    names = set()
    for h in ("rt_scene.h", "rt_hip.h", "rt_hip_test.h"):
        src = open(os.path.join(REPO, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(rt_\w+)\s*\(", src, re.M):
            names.add(m.group(1))
    return sorted(names)


def test_public_header_is_the_drop_in_boundary():
    """include/rt_hip.h declares the drop-in ABI (context,
    render, stats, assemble, multi-rank lists, rt_raytrace*, device memory
    helpers, exactness modes); probes, surveys, verification and A/B knobs
    live in include/rt_hip_test.h only."""
    def decls(h):
        src = re.sub(r"/\*.*?\*/", "", open(os.path.join(REPO, "include", h)).read(), flags=re.S)
        return {m.group(1) for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(rt_\w+)\s*\(", src, re.M)}
    pub, tst = decls("rt_hip.h"), decls("rt_hip_test.h")
    assert not pub & tst
    for hook in ("rt_hip_probe_closest", "rt_hip_set_policy", "rt_cand_survey", "rt_hip_cand_verify",
                 "rt_hip_set_cull_slack", "rt_hip_frame_times", "rt_accel_probe"):
        assert hook in tst and hook not in pub, hook
    for entry in ("rt_hip_create", "rt_hip_render", "rt_hip_stats", "rt_hip_destroy", "rt_raytrace",
                  "rt_raytrace_multi", "rt_hip_assemble", "rt_hip_cand_produce", "rt_hip_cand_consume"):
        assert entry in pub, entry


def test_library_exports_every_header_symbol(built):
    import rtgpu
    L = C.CDLL(rtgpu.LIB_PATH)
    names = _header_functions()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    bound = {p[0] for p in rtgpu._PROTOS}
    assert set(names) <= bound, set(names) - bound


@pytest.mark.parametrize("scene", SCENES)
def test_svati_loader_matches_reference_parser(scene, built, scene_dir):
    """Product loader == oracle's restatement of cpu/parser.c + parse_obj.c + stack.c."""
    import oracle as orc
    import rtgpu
    path = os.path.join(scene_dir, scene + ".svati")
    prod = rtgpu.Scene.load_svati(path)
    ref = orc.OracleScene(path)
    a = prod.triangles_array()
    b = rtgpu.scene_triangles(ref.ptr)
    assert a.shape == b.shape
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert np.array_equal(prod.materials_array().view(np.uint32),
                          rtgpu.scene_materials(ref.ptr).view(np.uint32))
    rs = C.cast(ref.ptr, C.POINTER(rtgpu.SceneStruct)).contents
    ps = prod.s
    assert rs.light_count == ps.light_count
    for i in range(ps.light_count):
        la, lb = ps.lights[i], rs.lights[i]
        assert (la.type, la.r, la.g, la.b, la.v.x, la.v.y, la.v.z) == \
               (lb.type, lb.r, lb.g, lb.b, lb.v.x, lb.v.y, lb.v.z)
    assert bytes(ps.camera) == bytes(rs.camera)


def test_lifo_triangle_order(built, tmp_path):
    """cpu/parse_obj.c:29-40,83-88: triangle t, corner k = v line N-1-3t-k."""
    import rtgpu
    p = tmp_path / "order.svati"
    lines = ["camera 8 8 0 0 -4 1 0 0 0 -1 0 70", "object 6"]
    lines += [f"v {i} {10 + i} {20 + i}" for i in range(6)]
    lines += [f"vn {i} 1 0" for i in range(6)]
    p.write_text("\n".join(lines) + "\n")
    tris = rtgpu.Scene.load_svati(str(p)).triangles_array()
    for t in range(2):
        for k in range(3):
            assert tris[t, k, 0] == 6 - 1 - 3 * t - k
            assert tris[t, 3 + k, 0] == 6 - 1 - 3 * t - k


def test_comment_swallows_next_line_like_reference(built, tmp_path):
    """'#' reads ' %[^\\n]' (cpu/parser.c:108-109): a bare '#' eats the next line."""
    import rtgpu
    p = tmp_path / "c.svati"
    p.write_text("camera 8 8 0 0 -4 1 0 0 0 -1 0 70\n#\na_light 1 1 1\n# note\nd_light 1 1 1 0 -1 0\n")
    s = rtgpu.Scene.load_svati(str(p))
    assert s.s.light_count == 1 and s.s.lights[0].type == 1


def test_parse_errors(built, tmp_path):
    import rtgpu
    p = tmp_path / "bad.svati"
    p.write_text("camera 8 8 0 0 -4 1 0 0 0 -1 0 70\nbogus 1 2 3\n")
    with pytest.raises(rtgpu.RtError) as e:
        rtgpu.Scene.load_svati(str(p))
    assert e.value.code == -3
    with pytest.raises(rtgpu.RtError) as e:
        rtgpu.Scene.load_svati(str(tmp_path / "missing.svati"))
    assert e.value.code == -2


def test_parse_error_texts_and_strict_vertex_count(built, tmp_path):
    """Error texts as the reference prints them (cpu/parser.c:111 "Error during
    the parsing %s", cpu/parse_obj.c:80 "Error during parsing %s"), and the
    deliberate strictness on objects whose v/vn lines do not match the
    declared count (the reference's behaviour there is undefined: it pops a
    NULL stack head, cpu/stack.c:36-39, or leaves triangles unallocated,
    cpu/parse_obj.c:83-89) -- rejected with a parse error, never rendered."""
    import rtgpu
    cam = "camera 8 8 0 0 -4 1 0 0 0 -1 0 70\n"
    cases = [
        (cam + "bogus 1 2 3\n", "Error during the parsing bogus"),
        (cam + "object 3\nKa 1 1 1\nfoo 1\n", "Error during parsing foo"),
        (cam + "object 6\nv 0 0 0\nv 1 0 0\nv 0 1 0\nvn 0 0 1\nvn 0 0 1\nvn 0 0 1\n",
         "object declares 6 vertices"),
        (cam + "object 3\nv 0 0 0\nv 1 0 0\nv 0 1 0\nvn 0 0 1\n", "object declares 3 vertices"),
    ]
    for k, (text, msg) in enumerate(cases):
        p = tmp_path / f"bad{k}.svati"
        p.write_text(text)
        with pytest.raises(rtgpu.RtError) as e:
            rtgpu.Scene.load_svati(str(p))
        assert e.value.code == -3 and msg in str(e.value), (k, str(e.value))


@pytest.mark.parametrize("case", CASES, ids=[case_id(c) for c in CASES])
def test_ppm_writer_byte_identical(case, built, tmp_path):
    """cpu/printer.c:3-18 + cpu/raytracer.c:128-134 from the golden framebuffer."""
    import rtgpu
    out = tmp_path / "o.ppm"
    rtgpu.write_ppm(str(out), golden_image(case))
    assert hashlib.md5(out.read_bytes()).hexdigest() == case["ppm_md5"]


def test_svati_and_obj_writers_round_trip(built, tmp_path):
    import oracle as orc
    import rtgpu
    s = rtgpu.Scene.synthetic(3, 2, 96, seed=0x5EED, width=64, height=36)
    tris = s.triangles_array()
    assert tris.shape[0] == s.triangle_count == 6 * s.triangles_array().shape[0] // 6
    sv = tmp_path / "syn.svati"
    s.write_svati(str(sv))
    back = rtgpu.Scene.load_svati(str(sv))
    assert np.array_equal(back.triangles_array().view(np.uint32), tris.view(np.uint32))
    ref = orc.OracleScene(str(sv))  # the reference grammar reads it back identically
    assert np.array_equal(rtgpu.scene_triangles(ref.ptr).view(np.uint32), tris.view(np.uint32))
    ob = tmp_path / "syn.obj"
    s.write_obj(str(ob))
    o = rtgpu.Scene.load_obj(str(ob))
    assert np.array_equal(o.triangles_array().view(np.uint32), tris.view(np.uint32))
    assert np.array_equal(o.materials_array().view(np.uint32),
                          s.materials_array().view(np.uint32))
    # objfile directive: camera + lights from .svati, geometry from .obj
    sv2 = tmp_path / "withobj.svati"
    sv2.write_text("camera 64 36 0 4 -20 1 0 0 0 -1 0 70\na_light 0.2 0.2 0.2\nobjfile syn.obj\n")
    w = rtgpu.Scene.load_svati(str(sv2))
    assert np.array_equal(w.triangles_array().view(np.uint32), tris.view(np.uint32))


def test_obj_loader_faces(built, tmp_path):
    import rtgpu
    p = tmp_path / "q.obj"
    p.write_text("v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nvn 0 0 1\n"
                 "o quad\nf 1//1 2//1 3//1 4//1\no tri\nf -4 -3 -2\n")
    s = rtgpu.Scene.load_obj(str(p))
    assert s.s.object_count == 2
    t = s.triangles_array()
    assert t.shape[0] == 3
    assert t[1, 1].tolist() == [1, 1, 0] and t[1, 2].tolist() == [0, 1, 0]
    assert t[2, 3].tolist() == [0, 0, 1]  # geometric normal for faces without vn


def test_synthetic_is_deterministic(built):
    import rtgpu
    a = rtgpu.Scene.synthetic(4, 4, 200, seed=1, width=32, height=32).triangles_array()
    b = rtgpu.Scene.synthetic(4, 4, 200, seed=1, width=32, height=32).triangles_array()
    c = rtgpu.Scene.synthetic(4, 4, 200, seed=2, width=32, height=32).triangles_array()
    assert np.array_equal(a, b) and not np.array_equal(a, c)


@pytest.mark.parametrize("scene", ["cube", "spheres", "island_smooth", "car-on-road", "dark-night"])
def test_octree_invariants(scene, built, scene_dir):
    import rtgpu
    s = rtgpu.Scene.load_svati(os.path.join(scene_dir, scene + ".svati"))
    rtgpu.accel_validate(s, "octree")
    rtgpu.accel_validate(s, "flat")
    info = rtgpu.accel_build_info(s, "octree")
    assert info["triangles"] == s.triangle_count
    assert info["tri_refs"] >= info["triangles"]


def test_octree_invariants_synthetic(built):
    import rtgpu
    s = rtgpu.Scene.synthetic(8, 8, 2000, seed=0x5EED, width=64, height=36)
    rtgpu.accel_validate(s, "octree")
    info = rtgpu.accel_build_info(s, "octree")
    assert info["leaves"] > 100


def test_render_fails_loudly_without_gpu(built, scene_dir):
    """No CPU fallback in the product path."""
    import rtgpu
    if rtgpu.device_count() > 0:
        pytest.skip("a GPU is present")
    s = rtgpu.Scene.load_svati(os.path.join(scene_dir, "cube.svati"))
    with pytest.raises(rtgpu.RtError) as e:
        rtgpu.Context(s, "flat")
    assert e.value.code == -6


@pytest.mark.parametrize("W,H", [(481, 270), (480, 271), (1, 1), (3841, 2161)])
def test_odd_frame_sizes_rejected(built, scene_dir, W, H):
    """cpu/rt writes pixel (i + W/2, j + H/2) (cpu/raytracer.c:89-91) but prints
    slot j*W + i for i in [1, W], j in [1, H] (:128-134): for odd W or H the two
    disagree and cpu/rt prints uninitialised memory, so the size is refused
    (RT_EINVAL) rather than rendered as something the reference never made."""
    import rtgpu
    s = rtgpu.Scene.load_svati(os.path.join(scene_dir, "cube.svati"))
    s.set_size(W, H)
    with pytest.raises(rtgpu.RtError) as e:
        s.frame()
    assert e.value.code == -1 and "even" in str(e.value)
    s.set_size(W + (W & 1), H + (H & 1))
    s.frame()  # the even neighbour is fine


@pytest.mark.parametrize("scene,W,H,stride", [("island_smooth", 960, 540, 31),
                                              ("car-on-road", 960, 540, 61),
                                              ("spheres", 480, 270, 37),
                                              ("susans_smooth", 960, 540, 61)])
def test_octree_culling_matches_brute_force_camera_rays(built, scene_dir, scene, W, H, stride):
    """Host model of the device walk (host/accel_probe.c): every sampled camera
    ray's closest-hit winner through the octree equals brute force."""
    import rtgpu
    s = rtgpu.Scene.load_svati(os.path.join(scene_dir, scene + ".svati"))
    s.set_size(W, H)
    r = rtgpu.accel_probe(s, "octree", stride, True)
    assert r["queries"] > 1000 and r["mismatches"] == 0, r


def test_octree_probe_synthetic(built):
    import rtgpu
    s = rtgpu.Scene.synthetic(2, 2, 1000, seed=0x5EED, width=640, height=360)
    r = rtgpu.accel_probe(s, "octree", 53, True)
    assert r["mismatches"] == 0 and r["hits"] > 100, r


def _threads(n):
    """RT_HOST_THREADS is read by the library on every call (lex_prescan.c)."""
    if n is None:
        os.environ.pop("RT_HOST_THREADS", None)
    else:
        os.environ["RT_HOST_THREADS"] = str(n)


def _load(kind, path, threads):
    import rtgpu
    _threads(threads)
    try:
        s = rtgpu.Scene.load_svati(path) if kind == "svati" else rtgpu.Scene.load_obj(path)
        return s.triangles_array(), s.materials_array()
    except rtgpu.RtError as e:
        return ("error", e.code)
    finally:
        _threads(None)


@pytest.mark.parametrize("kind", ["svati", "obj"])
def test_parallel_loader_equals_serial(built, tmp_path, kind):
    """§8f item 1: the multi-threaded v/vn pre-parse (host/lex_prescan.c,
    files >= 4 MB) gives bit-identical scenes to the serial scanner."""
    import rtgpu
    s = rtgpu.Scene.synthetic(4, 4, 3000, seed=0x5EED, width=64, height=36)
    p = str(tmp_path / ("syn." + kind))
    (s.write_svati if kind == "svati" else s.write_obj)(p)
    assert os.path.getsize(p) > (4 << 20)
    a, ma = _load(kind, p, 1)
    b, mb = _load(kind, p, 8)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert np.array_equal(ma.view(np.uint32), mb.view(np.uint32))
    if kind == "svati":
        assert np.array_equal(a.view(np.uint32), s.triangles_array().view(np.uint32))


def test_parallel_loader_irregular_svati(built, tmp_path):
    """Grammar corner cases around pre-parsed lines: a `v` line swallowed by a
    `#` comment (cpu/parser.c:108-109 skips blanks incl. newlines, then a
    line), numbers continued on the next line, a `v` token in mid-line,
    blank-indented lines.  Serial and parallel parses must agree exactly."""
    body = ["camera 64 36 0 4 -20 1 0 0 0 -1 0 70", "a_light 0.2 0.2 0.2",
            "d_light 1 1 1 1 -1 1"]
    rng = np.random.default_rng(7)
    n_obj = 40
    for o in range(n_obj):
        nv = 3 * 600
        body.append(f"object {nv}")
        body.append("Kd 0.5 0.4 0.3")
        vs = rng.normal(size=(nv, 3)).astype(np.float32).tolist()
        for i, v in enumerate(vs):
            line = f"v {v[0]!r} {v[1]!r} {v[2]!r}"
            if i % 97 == 5:
                line = f"v {v[0]!r}\n{v[1]!r} {v[2]!r}"      # continued
            elif i % 89 == 3:
                line = f"   \tv {v[0]!r} {v[1]!r} {v[2]!r}"  # indented
            elif i % 83 == 7:
                line = f"Ns 3 v {v[0]!r} {v[1]!r} {v[2]!r}"  # mid-line token
            body.append(line)
        for i, v in enumerate(vs):
            body.append(f"vn {v[2]!r} {v[0]!r} {v[1]!r}")
        body.append("#\nv 9 9 9")  # a whole v line eaten by the comment
        body.append("# comment")
    p = tmp_path / "odd.svati"
    p.write_text("\n".join(body) + "\n")
    assert os.path.getsize(p) > (4 << 20)
    a = _load("svati", str(p), 1)
    b = _load("svati", str(p), 8)
    assert not isinstance(a[0], str), a
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))


def _ppm_expected(W, H, img):
    f = img.reshape(-1).astype(np.float32)
    ok = (f > np.float32(-2147483904.0)) & (f < np.float32(2147483648.0))
    ints = np.where(ok, np.trunc(np.where(ok, f, 0)).astype(np.int64), -2147483648)
    return (f"P3\n{W} {H}\n255\n" + "".join(f"{v} " for v in ints.tolist())).encode()


def test_ppm_writer_parallel_chunks(built, tmp_path):
    """§8f item 3: multi-chunk, multi-threaded P3 formatting == the
    `"%d %d %d "` loop of cpu/printer.c:12-18 with (int) truncation."""
    import rtgpu
    W, H = 1000, 330  # 5 chunks of 2^16 px, the last ragged
    rng = np.random.default_rng(3)
    img = rng.uniform(-20, 300, size=(H, W, 3)).astype(np.float32)
    img.reshape(-1)[::9973] = np.nan
    img.reshape(-1)[5::7919] = np.inf
    img.reshape(-1)[7::7717] = -3e9
    want = _ppm_expected(W, H, img)
    for th in (1, 3, 8):
        _threads(th)
        try:
            out = tmp_path / f"o{th}.ppm"
            rtgpu.write_ppm(str(out), img)
        finally:
            _threads(None)
        assert out.read_bytes() == want, th


@pytest.mark.parametrize("kind", ["svati", "obj"])
def test_scene_writers_parallel_identical(built, tmp_path, kind):
    """§8f item 1: the scene writers format chunks of lines on the host
    threads (host/par_write.c) and write them in order: the bytes do not
    depend on the thread count, and every `v`/`vn` line is the "%.9g"
    formatting of the scene's floats in the writer's documented order."""
    import rtgpu
    s = rtgpu.Scene.synthetic(3, 3, 3000, seed=0x5EED, width=64, height=36)
    outs = []
    for th in (1, 3, 8):
        _threads(th)
        try:
            p = tmp_path / f"w{th}.{kind}"
            (s.write_svati if kind == "svati" else s.write_obj)(str(p))
            outs.append(p.read_bytes())
        finally:
            _threads(None)
    assert outs[0] == outs[1] == outs[2]
    tri = s.triangles_array()  # (T, 6, 3): 3 vertices then 3 normals, file/object order
    lines = outs[0].decode().split("\n")
    vlines = [ln for ln in lines if ln.startswith("v ")]
    assert len(vlines) == 3 * len(tri)
    # obj: object by object, triangle t corner k in order; svati: each
    # object's corners in reverse (the reference parser pops from the end)
    first = vlines[0].split()[1:]
    if kind == "obj":
        want = tri[0, 0]
    else:
        n0 = sum(1 for ln in lines[:lines.index(vlines[0])] if ln.startswith("object"))
        assert n0 == 1
        nv0 = int(next(ln for ln in lines if ln.startswith("object")).split()[1])
        want = tri[nv0 // 3 - 1, 2]
    assert first == ["%.9g" % float(x) for x in want]


def test_scene_lifecycle_asan(tmp_path, scene_dir):
    """The host C side (loaders, writers, flattening, both octree builds, the
    traversal model) builds, edits and frees scenes cleanly under the CPU
    AddressSanitizer + UBSan build (tests/native/asan_scene.c): no double
    free, overflow or leak.  (Round 2's 'double free or corruption (out)'
    came from an experiment script that advanced the objects pointer of a
    library-owned scene; tools/noground.py now empties the object in place.)"""
    import shutil
    import subprocess
    if not shutil.which("gcc"):
        pytest.skip("gcc missing")
    host = os.path.join(REPO, "raytracing-gpu_amd", "host")
    srcs = [os.path.join(host, f) for f in (
        "rt_error.c", "lex_prescan.c", "par_write.c", "scene_svati.c", "scene_obj.c",
        "vecmath.c", "ppm.c", "synth.c", "accel.c", "accel_probe.c")]
    exe = str(tmp_path / "asan_scene")
    cmd = ["gcc", "-std=c11", "-O1", "-g", "-ffp-contract=off", "-fsanitize=address,undefined",
           "-fno-omit-frame-pointer", "-I" + os.path.join(REPO, "include"), "-I" + host,
           os.path.join(REPO, "tests", "native", "asan_scene.c")] + srcs + \
          ["-lm", "-lpthread", "-o", exe]
    subprocess.run(cmd, check=True)
    scenes = []
    for name in ("cube", "car-on-road", "island_smooth", "spheres", "susans_smooth"):
        scenes.append(os.path.join(scene_dir, name + ".svati"))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", RT_HOST_THREADS="4")
    r = subprocess.run([exe, str(tmp_path)] + scenes, capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "asan scene lifecycle ok" in r.stdout


def test_lightbuf_survey_host(built):
    """Host survey of the light buffers (no device): slack-grown and proven
    footprints of a small synthetic scene, both lights; the proven ones list
    every triangle somewhere (none is edge-on enough to be never accepted
    here) and are deterministic."""
    import rtgpu
    s = rtgpu.Scene.synthetic(2, 2, 9776, seed=0x5EED, width=96, height=54)
    for li in (1, 2):
        a = s.lightbuf_survey(li, False, 1)
        b = s.lightbuf_survey(li, True, 1)
        assert a["surveyed"] == b["surveyed"] == s.triangle_count
        assert a["entries"] >= a["surveyed"] - a["global"]
        assert b["entries"] >= b["surveyed"] - b["global"] - b["never"]
        assert b == s.lightbuf_survey(li, True, 1)
