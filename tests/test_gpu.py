"""GPU parity tests (MI355X).  Every render goes through the C ABI of
lib/librtgpu.so; the checker is the reference's own output (tests/golden/,
bit-exact) or the oracle restatement (oracle/, pinned to those goldens).

Tolerance: north_star allows +-1 ULP per float channel; these tests demand
bit-exact equality (0 ULP) and report the ULP histogram when it fails.
"""
import hashlib
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import (REPO, case_id, golden_image, load_manifest_static, load_own_manifest,
                      own_golden_image, own_scene_path)

pytestmark = pytest.mark.gpu
CASES = load_manifest_static()
OWN_CASES = load_own_manifest()


def ulp_diff(a, b):
    ai = a.view(np.int32).astype(np.int64)
    bi = b.view(np.int32).astype(np.int64)
    ai = np.where(ai < 0, -(ai & 0x7FFFFFFF), ai)
    bi = np.where(bi < 0, -(bi & 0x7FFFFFFF), bi)
    return np.abs(ai - bi)


def assert_bitexact(img, ref, what):
    d = ulp_diff(np.ascontiguousarray(img), np.ascontiguousarray(ref))
    if d.max() != 0:
        bad = np.argwhere(d.reshape(-1, 3).max(axis=1) > 0)[:5].ravel()
        pytest.fail(f"{what}: {int((d > 0).sum())} channels differ, max {int(d.max())} ulp, "
                    f"first bad flat pixels {bad.tolist()}")


@pytest.fixture(scope="module")
def gpu(built):
    import rtgpu
    if rtgpu.device_count() == 0:
        pytest.fail("gpu tests need a gfx950 device")
    return rtgpu


@pytest.mark.parametrize("accel", ["flat", "octree", "octree_gpu"])
@pytest.mark.parametrize("case", CASES, ids=[case_id(c) for c in CASES])
def test_golden_bitexact(case, accel, gpu, scene_dir):
    s = gpu.Scene.load_svati(os.path.join(scene_dir, case["scene"] + ".svati"))
    s.set_size(case["width"], case["height"])
    ctx = gpu.Context(s, accel)
    img, st = ctx.render_image(s.frame())
    assert_bitexact(img, golden_image(case), f"{case_id(case)}/{accel}")
    assert st["closest"] == case["closest"]
    assert st["shadow"] == case["shadow"]
    assert st["depth_overflow"] == 0 and st["zero_normal"] == 0


@pytest.mark.parametrize("accel", ["flat", "octree", "octree_gpu"])
@pytest.mark.parametrize("case", OWN_CASES, ids=[case_id(c) for c in OWN_CASES])
def test_deep_reflections_bitexact(case, accel, gpu, tmp_path):
    """Paths as deep as cpu/rt's recursion makes them (cpu/raytracer.c:19-34):
    two facing Nr 0.9 mirrors, 44 closest-hit queries per camera ray, against
    the reference's own output -- round 2 stopped at 32 with RT_EDEPTH."""
    s = gpu.Scene.load_svati(own_scene_path(case, tmp_path))
    img, st = gpu.Context(s, accel).render_image(s.frame())
    assert_bitexact(img, own_golden_image(case), f"{case_id(case)}/{accel}")
    assert st["closest"] == case["closest"] and st["shadow"] == case["shadow"]
    assert st["depth_overflow"] == 0 and st["hit_records"] == st["closest"]


@pytest.mark.parametrize("accel", ["octree", "octree_gpu"])
@pytest.mark.parametrize("case", CASES + OWN_CASES, ids=[case_id(c) for c in CASES + OWN_CASES])
def test_golden_exact_reflections(case, accel, gpu, scene_dir, tmp_path):
    """The exact reflection mode (rt_hip_set_exact_reflections: the proven
    reflection walk, csrc/rt_reflect.hip) renders every golden case -- the
    reference's 20 scenes and the 44-bounce mirrors -- bit-exact, with the
    reference's query counts."""
    own = case in OWN_CASES
    path = own_scene_path(case, tmp_path) if own else os.path.join(scene_dir, case["scene"] + ".svati")
    s = gpu.Scene.load_svati(path)
    if not own:
        s.set_size(case["width"], case["height"])
    ctx = gpu.Context(s, accel)
    ctx.set_exact_reflections(True)
    img, st = ctx.render_image(s.frame())
    assert_bitexact(img, own_golden_image(case) if own else golden_image(case), f"{case_id(case)}/{accel}/exact-refl")
    assert (st["closest"], st["shadow"]) == (case["closest"], case["shadow"])
    assert st["depth_overflow"] == 0 and st["closest_unproven"] == 0


@pytest.mark.parametrize("scene,W,H", [("car-on-road", 1920, 1080), ("spheres", 960, 540)])
def test_exact_reflections_whole_frame(gpu, scene_dir, scene, W, H):
    """Whole frames with the exact reflection walk == brute force over every
    triangle (both octrees), same query counts."""
    s = gpu.Scene.load_svati(os.path.join(scene_dir, scene + ".svati"))
    s.set_size(W, H)
    f = s.frame()
    img_f, st_f = gpu.Context(s, "flat").render_image(f)
    for accel in ("octree", "octree_gpu"):
        ctx = gpu.Context(s, accel)
        ctx.set_exact_reflections(True)
        img, st = ctx.render_image(f)
        assert_bitexact(img, img_f, f"{scene} {accel} exact reflections vs flat")
        assert (st["closest"], st["shadow"]) == (st_f["closest"], st_f["shadow"])


def test_exact_reflections_synthetic_frame(gpu):
    """A 352k-triangle sphere field (1/8 of the spheres Nr 0.3, as C5) at
    960x540 with the exact reflection walk == brute force, device octree."""
    s = gpu.Scene.synthetic(6, 6, 9776, seed=0x5EED, width=960, height=540)
    f = s.frame()
    img_f, st_f = gpu.Context(s, "flat").render_image(f)
    ctx = gpu.Context(s, "octree_gpu")
    ctx.set_exact_reflections(True)
    img, st = ctx.render_image(f)
    assert_bitexact(img, img_f, "synthetic 960x540 exact reflections vs flat")
    assert (st["closest"], st["shadow"]) == (st_f["closest"], st_f["shadow"])


def test_exact_reflections_need_default_policy(gpu, scene_dir):
    s = gpu.Scene.load_svati(os.path.join(scene_dir, "cube.svati"))
    s.set_size(32, 32)
    ctx = gpu.Context(s, "octree")
    ctx.set_exact_reflections(True)
    ctx.set_policy(1)
    with pytest.raises(gpu.RtError) as e:
        ctx.render_image(s.frame())
    assert e.value.code == -1  # RT_EINVAL


def test_endless_mirror_reports_depth(gpu, tmp_path):
    """Nr 1.0 mirrors facing each other: cpu/rt's recursion never ends (its
    stack overflows); the render stops each path at RT_MAX_BOUNCES and fails
    loudly with RT_EDEPTH instead of writing a silently truncated image."""
    text = open(own_scene_path(OWN_CASES[0], tmp_path)).read().replace("Nr 0.9", "Nr 1.0")
    sv = tmp_path / "endless.svati"
    sv.write_text(text.replace("camera 32 18", "camera 8 4"))
    s = gpu.Scene.load_svati(str(sv))
    with pytest.raises(gpu.RtError) as e:
        gpu.Context(s, "octree").render_image(s.frame())
    assert e.value.code == -7


def test_c4_car_on_road_4k_eight_rank_split(gpu, scene_dir):
    """Config C4 at its real size: car-on-road at 3840x2160 rendered as the
    8-rank split (every rank's tiles, one rank at a time on this GPU), gathered
    rank-major and assembled, equals the brute-force whole frame bit for bit,
    with the same query counts; sampled pixels equal the oracle."""
    import ctypes as C
    s = gpu.Scene.load_svati(os.path.join(scene_dir, "car-on-road.svati"))
    W, H, n = 3840, 2160, 8
    s.set_size(W, H)
    f = s.frame()
    img_f, st_f = gpu.Context(s, "flat").render_image(f)
    ctx = gpu.Context(s, "octree")
    per = gpu.tile_buffer_floats(W, H, n)
    L = gpu.lib()
    dg, drgb = C.c_void_p(), C.c_void_p()
    assert L.rt_hip_malloc(0, per * n * 4, C.byref(dg)) == 0
    assert L.rt_hip_malloc(0, W * H * 12, C.byref(drgb)) == 0
    tot = {"closest": 0, "shadow": 0}
    for r in range(n):
        ctx.render(f, r, n, dg.value + r * per * 4)
        st = ctx.stats()
        tot["closest"] += st["closest"]
        tot["shadow"] += st["shadow"]
    ctx.assemble(f, dg.value, n, drgb.value)
    img = np.empty((H, W, 3), np.float32)
    ctx.stats()  # sync
    assert L.rt_hip_memcpy_d2h(img.ctypes.data_as(C.c_void_p), drgb, img.nbytes) == 0
    L.rt_hip_free(dg)
    L.rt_hip_free(drgb)
    assert_bitexact(img, img_f, "C4 8-rank split vs brute force")
    assert (tot["closest"], tot["shadow"]) == (st_f["closest"], st_f["shadow"])
    pix, vals = _oracle_sample(s, W, H, 32, 4)
    assert_bitexact(img[pix[:, 0], pix[:, 1]], vals, "C4 vs oracle sample")


def test_cli_ppm_md5(gpu, scene_dir, tmp_path, manifest):
    """`rt file.svati out.ppm` writes the reference's exact bytes (config C1)."""
    case = next(c for c in manifest if c["scene"] == "cube" and c["width"] == 256)
    src = os.path.join(scene_dir, "cube.svati")
    sv = tmp_path / "cube256.svati"
    txt = open(src).read().replace("camera 512 512", "camera 256 256")
    sv.write_text(txt)
    out = tmp_path / "o.ppm"
    exe = os.path.join(REPO, "raytracing-gpu_amd", "lib", "rt")
    subprocess.run([exe, str(sv), str(out)], check=True)
    assert hashlib.md5(out.read_bytes()).hexdigest() == case["ppm_md5"]
    p = subprocess.run([exe, str(sv)], capture_output=True, text=True)
    assert p.returncode == 1 and "usage:" in p.stderr


def _with_camera_size(src, dst, width, height):
    """Copy of a .svati scene with its camera line's resolution replaced."""
    lines = open(src).read().split("\n")
    for i, ln in enumerate(lines):
        f = ln.split()
        if f and f[0] == "camera":
            lines[i] = " ".join(["camera", str(width), str(height)] + f[3:])
    dst.write_text("\n".join(lines))


def test_raytrace_multi_one_gpu_md5(gpu, scene_dir, tmp_path, manifest):
    """The drop-in entry rt_raytrace_multi (file in, P3 file out, its own
    device setup, gather and assemble) with ngpus=1 writes the reference's
    exact bytes for every golden case (rt_raytrace is its ngpus=1 form)."""
    for case in manifest:
        sv = tmp_path / f"{case['scene']}_{case['width']}.svati"
        _with_camera_size(os.path.join(scene_dir, case["scene"] + ".svati"), sv, case["width"],
                          case["height"])
        out = tmp_path / "o.ppm"
        st, _ = gpu.raytrace(str(sv), str(out), gpus=1)
        assert hashlib.md5(out.read_bytes()).hexdigest() == case["ppm_md5"], case_id(case)
        assert st["closest"] == case["closest"] and st["shadow"] == case["shadow"], case_id(case)


@pytest.mark.parametrize("nranks", [3, 4, 8])
def test_raytrace_multi_ranks_on_one_gpu(gpu, scene_dir, tmp_path, manifest, nranks):
    """the drop-in N-GPU entry itself on one GPU --
    rt_raytrace_multi_dev with every rank on device 0 runs the same frame as
    rt_raytrace_multi (per-rank octrees and renders, from 4 ranks the
    triangle-parallel candidate lists and their exchange, the gather and the
    assemble) with device memcpys in place of RCCL, and writes the
    reference's exact bytes."""
    for case in manifest:
        if case["scene"] not in ("island_smooth", "spheres", "car-on-road"):
            continue
        sv = tmp_path / f"{case['scene']}_{case['width']}.svati"
        _with_camera_size(os.path.join(scene_dir, case["scene"] + ".svati"), sv, case["width"],
                          case["height"])
        out = tmp_path / "o.ppm"
        st, _ = gpu.raytrace_devices(str(sv), str(out), [0] * nranks)
        assert hashlib.md5(out.read_bytes()).hexdigest() == case["ppm_md5"], (case_id(case), nranks)
        assert st["closest"] == case["closest"] and st["shadow"] == case["shadow"], case_id(case)


@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_tile_partition_gather_assemble(gpu, scene_dir, nranks, manifest):
    """Rank-sharded renders + rank-major gather + assemble == the single image."""
    import ctypes as C
    case = next(c for c in manifest if c["scene"] == "island_smooth" and c["width"] == 192)
    s = gpu.Scene.load_svati(os.path.join(scene_dir, "island_smooth.svati"))
    s.set_size(case["width"], case["height"])
    f = s.frame()
    ctx = gpu.Context(s, "octree")
    per = gpu.tile_buffer_floats(f.width, f.height, nranks)
    L = gpu.lib()
    dg = C.c_void_p()
    drgb = C.c_void_p()
    assert L.rt_hip_malloc(0, per * nranks * 4, C.byref(dg)) == 0
    assert L.rt_hip_malloc(0, f.width * f.height * 12, C.byref(drgb)) == 0
    tot = {"closest": 0, "shadow": 0}
    for r in range(nranks):
        ctx.render(f, r, nranks, dg.value + r * per * 4)
        st = ctx.stats()
        tot["closest"] += st["closest"]
        tot["shadow"] += st["shadow"]
    ctx.assemble(f, dg.value, nranks, drgb.value)
    img = np.empty((f.height, f.width, 3), np.float32)
    ctx.stats()  # sync
    assert L.rt_hip_memcpy_d2h(img.ctypes.data_as(C.c_void_p), drgb, img.nbytes) == 0
    L.rt_hip_free(dg)
    L.rt_hip_free(drgb)
    assert_bitexact(img, golden_image(case), f"{nranks} ranks")
    assert tot["closest"] == case["closest"] and tot["shadow"] == case["shadow"]


def _oracle_sample(scene, W, H, n, seed):
    import oracle as orc
    rng = np.random.default_rng(seed)
    pix = np.stack([rng.integers(0, H, n), rng.integers(0, W, n)], axis=1).astype(np.int32)
    vals, cnt = orc.render(scene.ptr, W, H, pixels=pix, threads=0)
    return pix, vals


@pytest.mark.parametrize("scene,W,H", [("island_smooth", 1920, 1080), ("spheres", 1920, 1080),
                                       ("car-on-road", 960, 540), ("susans_smooth", 960, 540)])
def test_large_flat_equals_octree_and_oracle_sample(gpu, scene_dir, scene, W, H):
    """Full-size configs: octree == brute force over the whole frame (a
    size-independent property), plus oracle parity on sampled pixels."""
    s = gpu.Scene.load_svati(os.path.join(scene_dir, scene + ".svati"))
    s.set_size(W, H)
    f = s.frame()
    img_o, st_o = gpu.Context(s, "octree").render_image(f)
    img_f, st_f = gpu.Context(s, "flat").render_image(f)
    assert_bitexact(img_o, img_f, f"{scene} octree vs flat")
    assert st_o["closest"] == st_f["closest"] and st_o["shadow"] == st_f["shadow"]
    img_g, st_g = gpu.Context(s, "octree_gpu").render_image(f)
    assert_bitexact(img_g, img_f, f"{scene} device-built octree vs flat")
    assert st_g["closest"] == st_f["closest"] and st_g["shadow"] == st_f["shadow"]
    pix, vals = _oracle_sample(s, W, H, 64, 11)
    assert_bitexact(img_o[pix[:, 0], pix[:, 1]], vals, f"{scene} vs oracle sample")


def test_synthetic_octree_vs_oracle(gpu):
    s = gpu.Scene.synthetic(4, 4, 400, seed=0x5EED, width=96, height=54)
    import oracle as orc
    img, st = gpu.Context(s, "octree").render_image(s.frame())
    ref, cnt = orc.render(s.ptr, 96, 54, threads=0)
    assert_bitexact(img, ref, "synthetic small")
    assert st["closest"] == cnt["closest"] and st["shadow"] == cnt["shadow"]


@pytest.mark.parametrize("scene", ["cube", "spheres", "island_smooth", "car-on-road",
                                   "dark-night", "susans_smooth"])
def test_device_octree_invariants(gpu, scene_dir, scene):
    """Device build (csrc/rt_build.hip): every triangle in a leaf, leaf boxes
    overlap their triangles, node boxes contain their children."""
    s = gpu.Scene.load_svati(os.path.join(scene_dir, scene + ".svati"))
    ctx = gpu.Context(s, "octree_gpu")
    ctx.validate()
    info = ctx.info()
    assert info["triangles"] == s.triangle_count and info["tri_refs"] >= info["triangles"]
    assert info["nodes"] >= 1


def test_device_octree_synthetic_and_deterministic(gpu):
    s = gpu.Scene.synthetic(8, 8, 2000, seed=0x5EED, width=320, height=180)
    a = gpu.Context(s, "octree_gpu")
    a.validate()
    ia = a.info()
    ib = gpu.Context(s, "octree_gpu").info()
    assert (ia["nodes"], ia["tri_refs"], ia["leaves"]) == (ib["nodes"], ib["tri_refs"], ib["leaves"])
    f = s.frame()
    img_g, st_g = a.render_image(f)
    img_f, st_f = gpu.Context(s, "flat").render_image(f)
    assert_bitexact(img_g, img_f, "device-built octree vs brute force")
    assert (st_g["closest"], st_g["shadow"]) == (st_f["closest"], st_f["shadow"])


def _tiles_of_rank(ctx, f, rank, nranks):
    """The rank's rendered tiles (its tile buffer minus the padding slots)."""
    import ctypes as C
    L = gpu_lib()
    per = gpu_mod().tile_buffer_floats(f.width, f.height, nranks)
    d = C.c_void_p()
    assert L.rt_hip_malloc(0, per * 4, C.byref(d)) == 0
    ctx.render(f, rank, nranks, d.value)
    st = ctx.stats()
    out = np.empty(per, np.float32)
    assert L.rt_hip_memcpy_d2h(out.ctypes.data_as(C.c_void_p), d, out.nbytes) == 0
    L.rt_hip_free(d)
    return out.reshape(-1, 64, 3)[: gpu_mod().rank_tile_count(f.width, f.height, rank, nranks)], st


def gpu_mod():
    import rtgpu
    return rtgpu


def gpu_lib():
    return gpu_mod().lib()


def test_synthetic_c5_exact_on_sampled_tiles(gpu):
    """C5 itself (10M triangles, 4K), the headline workload: the device-built
    octree with exact camera rays (csrc/rt_cand.hip) equals brute force --
    cpu/rt's own collide/collide_dist over every triangle (cpu/hit.c:72-109)
    -- bit for bit on every pixel of 1/256 of the frame's tiles (every 256th
    8x8 tile, 32,400 pixels), and the oracle on sampled pixels.  No
    allowance: before the candidate lists about 3e-5 of these pixels had a
    grazing camera ray whose float winner the walk culled."""
    s = gpu.Scene.synthetic(32, 32, 9776, seed=0x5EED, width=3840, height=2160)
    f = s.frame()
    ctx = gpu.Context(s, "octree_gpu")
    img, st = ctx.render_image(f)
    assert st["pixels"] == 3840 * 2160 and st["depth_overflow"] == 0 and st["zero_normal"] == 0
    assert st["cand_entries"] > 0
    flat = gpu.Context(s, "flat")
    for rank in (0, 131):
        tf, stf = _tiles_of_rank(flat, f, rank, 256)
        ref = gpu.tiles_from_image_numpy(img, rank, 256)
        assert_bitexact(ref[: len(tf)], tf, f"C5 tiles of rank {rank}/256 vs brute force")
    pix, vals = _oracle_sample(s, 3840, 2160, 8, 5)
    assert_bitexact(img[pix[:, 0], pix[:, 1]], vals, "C5 sample vs oracle")


# Traversal policies of the octree walk (rt_hip_set_policy, one kernel each;
# csrc/rt_render.hip): default (staged packet closest hit for coherent
# queries, per-lane otherwise), all per-lane, all staged packet, default +
# staged directional-light shadows.  The default runs in every other test.
TRAV = [0, 1, 2, 3]
TRAV_SCENES = ["cube", "car-on-road", "dark-night", "island_smooth", "spheres", "susans_smooth",
               "lighthouse", "point-light"]


@pytest.mark.parametrize("trav", TRAV)
def test_traversal_policies_bitexact(gpu, scene_dir, manifest, trav):
    """Every traversal policy reproduces the reference goldens bit for bit."""
    for case in manifest:
        if case["scene"] not in TRAV_SCENES or case["width"] != 96:
            continue
        s = gpu.Scene.load_svati(os.path.join(scene_dir, case["scene"] + ".svati"))
        s.set_size(case["width"], case["height"])
        ctx = gpu.Context(s, "octree")
        ctx.set_policy(trav)
        img, st = ctx.render_image(s.frame())
        assert_bitexact(img, golden_image(case), f"{case_id(case)} trav {trav}")
        assert st["closest"] == case["closest"] and st["shadow"] == case["shadow"]


@pytest.mark.parametrize("trav", TRAV)
def test_traversal_policies_full_frame(gpu, scene_dir, trav):
    """Whole 1080p frame of the densest reference scene: octree walk == brute force."""
    s = gpu.Scene.load_svati(os.path.join(scene_dir, "car-on-road.svati"))
    s.set_size(1920, 1080)
    f = s.frame()
    img_f, _ = gpu.Context(s, "flat").render_image(f)
    ctx = gpu.Context(s, "octree")
    ctx.set_policy(trav)
    img_o, _ = ctx.render_image(f)
    assert_bitexact(img_o, img_f, f"car-on-road 1080p trav {trav}")


@pytest.mark.parametrize("accel", ["octree", "octree_gpu"])
def test_synthetic_full_frame_exact(gpu, accel):
    """Million-triangle synthetic scene, whole frame, octree vs brute force:
    bit-exact (cpu/rt's float Moller-Trumbore accepts some triangles that
    grazing camera rays miss by world units -- DESIGN.md §2; the camera
    candidate lists keep those decisions), and the oracle on sampled pixels
    (including, on the previous build, every pixel that differed)."""
    import oracle as orc
    s = gpu.Scene.synthetic(6, 6, 9776, seed=0x5EED, width=960, height=540)
    f = s.frame()
    img_f, st_f = gpu.Context(s, "flat").render_image(f)
    img_o, st_o = gpu.Context(s, accel).render_image(f)
    assert_bitexact(img_o, img_f, f"synthetic 960x540 {accel} vs brute force")
    assert (st_o["closest"], st_o["shadow"]) == (st_f["closest"], st_f["shadow"])
    pix, vals = _oracle_sample(s, 960, 540, 24, 3)
    assert_bitexact(img_f[pix[:, 0], pix[:, 1]], vals, "synthetic brute force vs oracle")


@pytest.mark.parametrize("accel,policy,exact,lbuf", [("octree_gpu", 0, False, True),
                                                     ("octree", 0, False, True),
                                                     ("octree_gpu", 0, False, False),
                                                     ("octree_gpu", 3, False, True),
                                                     ("octree_gpu", 0, True, True),
                                                     ("octree", 2, True, True)])
def test_shadow_queries_match_brute_force(gpu, accel, policy, exact, lbuf):
    """Every shadow query of a frame (the shade kernel's per-record outcome of
    cpu/light.c:24-31 for each light) through the light buffers (default) or
    the octree walk equals brute force over all triangles (cpu/hit.c:93-109)
    on the same hit records -- shadow rays leave surfaces at grazing angles
    near the terminators, where the float Moller-Trumbore test is least
    conditioned."""
    s = gpu.Scene.synthetic(6, 6, 9776, seed=0x5EED, width=960, height=540)
    ctx = gpu.Context(s, accel)
    if lbuf and not exact and policy == 0:
        assert ctx.info()["lightbuf_entries"] > 0
    ctx.set_light_buffers(lbuf)
    ctx.set_policy(policy)
    ctx.set_exact_shadows(exact)  # the default is on
    if exact:  # proven light buffers, or (staged policies) the proven walk
        assert ctx.info()["shadow_mu_max"] >= 1.0
        if lbuf:
            assert ctx.info()["lightbuf_entries"] > 0
    img, _ = ctx.render_image(s.frame())
    v = ctx.verify_shadows(1)
    assert v["records"] > 100000 and v["queries"] == 2 * v["records"], v
    assert v["records_differ"] == 0 and v["walk_lit_brute_shadowed"] == 0, v


@pytest.mark.parametrize("exact_shadows", [False, True])
def test_no_camera_lists_with_light_buffers(gpu, exact_shadows):
    """exact_camera off (an A/B knob) leaves the render without candidate
    lists; the shadow queries still index the prim-order records (light
    buffers, the exact mode's global list).  Round 3 first ran this with a
    null record pointer -- it must render, and agree with the lists' image
    wherever camera rays are not grazing (here: everywhere)."""
    s = gpu.Scene.synthetic(3, 3, 9776, seed=0x5EED, width=320, height=180)
    f = s.frame()
    ctx = gpu.Context(s, "octree_gpu")
    ctx.set_exact_shadows(exact_shadows)
    img, _ = ctx.render_image(f)
    ctx.set_exact_camera(False)
    img_nc, _ = ctx.render_image(f)
    assert_bitexact(img_nc, img, "without camera candidate lists")


@pytest.mark.parametrize("height,exact", [(0.02, False), (0.5, False), (0.02, True), (0.5, True),
                                          (0.0, True)])
def test_light_buffer_point_light_near_surface(gpu, height, exact):
    """A point light just above a sphere: triangles around it span wide
    angles of the light's cube map (or go to its global list); every shadow
    query still equals brute force, and the image equals the walk's."""
    s = gpu.Scene.synthetic(4, 4, 9776, seed=0x5EED, width=480, height=270)
    tri = s.triangles_array()
    top = tri[2 + 5 * 9776: 2 + 6 * 9776, :3].reshape(-1, 3)  # sphere 5's vertices
    k = int(np.argmax(top[:, 1]))
    L = s.s.lights[2]
    assert int(L.type) == 2
    L.v.x, L.v.y, L.v.z = float(top[k, 0]), float(top[k, 1]) + height, float(top[k, 2])
    f = s.frame()
    ctx = gpu.Context(s, "octree_gpu")
    ctx.set_exact_shadows(exact)  # proven footprints (a light on the sphere: its tangent plane)
    img, _ = ctx.render_image(f)
    v = ctx.verify_shadows(1)
    assert v["records"] > 10000 and v["records_differ"] == 0 and v["walk_lit_brute_shadowed"] == 0, v
    if exact:  # brute force is the reference for the proven mode
        img_w, _ = gpu.Context(s, "flat").render_image(f)
    else:
        ctx.set_light_buffers(False)
        img_w, _ = ctx.render_image(f)
    assert_bitexact(img, img_w, f"light buffers (exact={exact}) vs {'flat' if exact else 'walk'}, "
                                f"light {height} above a sphere")


def test_exact_camera_rank_split(gpu):
    """Candidate lists are built per rank (only the rank's tiles): a 3-way
    split of the synthetic frame, each rank's tiles == brute force."""
    s = gpu.Scene.synthetic(6, 6, 9776, seed=0x5EED, width=960, height=540)
    f = s.frame()
    img_f, _ = gpu.Context(s, "flat").render_image(f)
    ctx = gpu.Context(s, "octree_gpu")
    for rank in range(3):
        t, st = _tiles_of_rank(ctx, f, rank, 3)
        ref = gpu.tiles_from_image_numpy(img_f, rank, 3)
        assert_bitexact(t, ref[: len(t)], f"rank {rank}/3")


@pytest.mark.parametrize("accel,nranks,ranks,item_cap", [("octree_gpu", 1, (0,), None), ("octree", 1, (0,), None),
                                                        ("octree_gpu", 3, (0, 1, 2), None),
                                                        ("octree_gpu", 7, (0, 6), None),
                                                        ("octree_gpu", 1, (0,), 0),
                                                        ("octree_gpu", 3, (0, 2), 5)])
def test_candidate_lists_match_host(gpu, accel, nranks, ranks, item_cap):
    """The device-built camera candidate lists (csrc/rt_cand.hip: float fast
    path, f64 classification, small/big footprint split, emission, radix
    sort, per-tile offsets) equal the host re-derivation from the same
    classify/raster code: every listed prim's footprint bit for bit, every
    tile's list as a multiset -- including the big footprints (hundreds of
    tiles), emitted entry-parallel in chunks (big_item_kernel) or, when the
    work items overflow their cap (item_cap 0, or 5: overflow part-way), one
    wave per footprint (big_kernel); 7 ranks exercise the rank filter's
    per-row path (240 tile columns are not a multiple of 7)."""
    s = gpu.Scene.synthetic(8, 6, 9776, seed=0x5EED, width=1920, height=1080)
    f = s.frame()
    ctx = gpu.Context(s, accel)
    if item_cap is not None:
        ctx.set_cand_item_cap(item_cap)
    for rank in ranks:
        _tiles_of_rank(ctx, f, rank, nranks)
        v = ctx.cand_verify(f, rank, nranks)
        assert v["listed"] > 0 and v["entries"] > 0, v
        assert v["fp_mismatch"] == 0 and v["tile_mismatch"] == 0, str(v)
        assert v["filter_violation"] == 0 and v["filtered"] > 0, str(v)


def test_candidate_lists_match_host_c5(gpu):
    """The headline scene itself (C5: 10,010,626 triangles at 3840x2160):
    every float fast-path verdict (Q_SAFE / Q_LIST / rank-filtered) checked
    against the f64 classify() over all 10M triangles, every listed
    footprint bit for bit and every tile's list as a multiset -- for the
    whole frame (N = 1) and for ranks 0 and 3 of an 8-way split.  This pins
    the exactness of the shipped camera-ray lists on the shipped tree
    (/root/reference/cpu/hit.c:4-44,72-91)."""
    s = gpu.Scene.synthetic(32, 32, 9776, seed=0x5EED, width=3840, height=2160)
    assert s.triangle_count == 10010626
    f = s.frame()
    ctx = gpu.Context(s, "octree_gpu")
    for nranks, rank in ((1, 0), (8, 0), (8, 3)):
        _tiles_of_rank(ctx, f, rank, nranks)
        v = ctx.cand_verify(f, rank, nranks)
        assert v["listed"] > 0 and v["entries"] > 0, v
        assert v["fp_mismatch"] == 0 and v["tile_mismatch"] == 0, (nranks, rank, v)
        assert v["filter_violation"] == 0, (nranks, rank, v)


def _produce_all(ctx, f, nranks):
    """Every rank's triangle-parallel produce, on one context in turn: per
    producer (host copy of its routed entries (n, 3) uint32, counts, globals)."""
    import ctypes as C
    L = gpu_lib()
    parts = []
    for r in range(nranks):
        counts, ng = ctx.cand_produce(f, r, nranks)
        ptr, n = ctx.cand_send_buffer()
        assert n == sum(counts)
        host = np.empty((max(n, 1), 3), np.uint32)
        if n:
            assert L.rt_hip_memcpy_d2h(host.ctypes.data_as(C.c_void_p), C.c_void_p(ptr), n * 12) == 0
        parts.append((host[:n], counts, ng))
    return parts


def _consume_rank(ctx, f, d, nranks, parts):
    """What rank d receives in the all-to-all (its block from every producer,
    in source order), uploaded and consumed."""
    import ctypes as C
    L = gpu_lib()
    blocks = []
    for host, counts, _ in parts:
        o = sum(counts[:d])
        blocks.append(host[o:o + counts[d]])
    recv = np.ascontiguousarray(np.concatenate(blocks) if blocks else np.empty((0, 3), np.uint32))
    g = sum(p[2] for p in parts)
    dptr = C.c_void_p()
    assert L.rt_hip_malloc(0, max(recv.nbytes, 16), C.byref(dptr)) == 0
    if recv.size:
        assert L.rt_hip_memcpy_h2d(dptr, recv.ctypes.data_as(C.c_void_p), recv.nbytes) == 0
    ctx.cand_consume(f, d, nranks, dptr.value, len(recv), g)
    return dptr, len(recv), g


@pytest.mark.parametrize("nranks,accel", [(3, "octree_gpu"), (8, "octree_gpu"), (2, "octree")])
def test_triangle_parallel_lists_match_per_rank(gpu, nranks, accel):
    """Triangle-parallel candidate lists (rt_hip_cand_produce -> all-to-all ->
    rt_hip_cand_consume; the exchange emulated on the host): every producer
    builds the whole frame's entries of its slice of the triangles, routed to
    the tiles' ranks; each rank's consumed lists give the same per-tile entry
    counts as its own per-rank build, and its render the same tile bits and
    query counts (the winner's key is order-independent)."""
    s = gpu.Scene.synthetic(6, 6, 9776, seed=0x5EED, width=960, height=540)
    f = s.frame()
    ctx = gpu.Context(s, accel)
    ref = gpu.Context(s, accel)  # (prim -> leaf is the smallest leaf index: the same lists)
    parts = _produce_all(ctx, f, nranks)
    assert sum(sum(c) for _, c, _ in parts) > 0
    L = gpu_lib()
    for d in range(nranks):
        dptr, n, g = _consume_rank(ctx, f, d, nranks, parts)
        t_ext, st_ext = _tiles_of_rank(ctx, f, d, nranks)  # uses the consumed lists
        nt = gpu.rank_tile_count(f.width, f.height, d, nranks)
        e_ext = ctx.cand_tile_entries(nt)
        L.rt_hip_free(dptr)
        t_ref, st_ref = _tiles_of_rank(ref, f, d, nranks)
        e_ref = ref.cand_tile_entries(nt)
        assert np.array_equal(e_ext, e_ref), (d, int(e_ext.sum()), int(e_ref.sum()))
        assert st_ext["cand_entries"] == st_ref["cand_entries"] == n - g
        assert_bitexact(t_ext, t_ref, f"rank {d}/{nranks}: consumed vs per-rank lists")
        assert (st_ext["closest"], st_ext["shadow"]) == (st_ref["closest"], st_ref["shadow"])
    # the consumed lists are used once: the next render builds its own again
    t2, st2 = _tiles_of_rank(ctx, f, 0, nranks)
    t_ref, st_ref = _tiles_of_rank(ref, f, 0, nranks)
    assert_bitexact(t2, t_ref, "per-rank build after a consumed frame")


@pytest.mark.parametrize("nranks,grid", [(3, 6), (4, 6), (8, 6), (16, 1)])
def test_cand_exchange_local_matches_per_rank(gpu, nranks, grid):
    """the exchange rt_raytrace_multi makes over RCCL (from 4
    GPUs up), driven with N contexts on one GPU and the device-memcpy
    transport: every rank's render from the exchanged lists equals its render
    from its own per-rank lists, bit for bit, with the same entry count.
    Producers take interleaved blocks of 1,024 prims: 3 ranks (the blocks not
    a multiple of N), and one sphere (9,778 prims: 10 blocks) over 16 ranks,
    where 6 producers have no prims at all."""
    s = gpu.Scene.synthetic(grid, grid, 9776, seed=0x5EED, width=960, height=540)
    f = s.frame()
    ctxs = [gpu.Context(s, "octree_gpu") for _ in range(nranks)]
    ref = gpu.Context(s, "octree_gpu")
    gpu.cand_exchange_local(ctxs, f)
    for d in range(nranks):
        t_ext, st_ext = _tiles_of_rank(ctxs[d], f, d, nranks)
        t_ref, st_ref = _tiles_of_rank(ref, f, d, nranks)
        assert st_ext["cand_entries"] == st_ref["cand_entries"], d
        assert_bitexact(t_ext, t_ref, f"rank {d}/{nranks}: exchanged vs per-rank lists")
        assert (st_ext["closest"], st_ext["shadow"]) == (st_ref["closest"], st_ref["shadow"])
    with pytest.raises(gpu.RtError):
        gpu.cand_exchange_local([], f)


def test_produce_repeated_slice_is_identical(gpu):
    """A slice produced before for the same frame (the last produce of the
    context: each GPU produces its own rank's slice every frame) is rebuilt
    without the mid-build read-back (its sizes are known): the routed entries
    and the per-rank counts equal the read-back build's bit for bit."""
    import ctypes as C
    L = gpu_lib()
    s = gpu.Scene.synthetic(6, 6, 9776, seed=0x5EED, width=960, height=540)
    f = s.frame()
    ctx = gpu.Context(s, "octree_gpu")
    nranks = 4

    def produce(r):
        counts, ng = ctx.cand_produce(f, r, nranks)
        ptr, n = ctx.cand_send_buffer()
        host = np.empty((max(n, 1), 3), np.uint32)
        if n:
            assert L.rt_hip_memcpy_d2h(host.ctypes.data_as(C.c_void_p), C.c_void_p(ptr), n * 12) == 0
        return host[:n].copy(), counts, ng

    for r in range(nranks):
        h0, c0, g0 = produce(r)  # read-back build
        for _ in range(2):       # known sizes
            h1, c1, g1 = produce(r)
            assert (c0, g0) == (c1, g1), r
            assert np.array_equal(h0, h1), r
    total = sum(produce(0)[1])
    ctx.set_camera_bound_scale(1.5)  # other lists: read back again
    assert sum(produce(0)[1]) >= total


def test_consumed_lists_invalidated_by_a_later_build(gpu):
    """lists rt_hip_cand_consume leaves for a render live in the
    context's shared list buffers.  A produce (e.g. the next frame's) between
    consume and render overwrites them, so the render must build its own lists
    again rather than read clobbered ones: produce -> consume -> produce ->
    render equals the per-rank render bit for bit, with the same entry count.
    And the kept-entry count rt_hip_stats reports for a render survives a
    produce issued before the stats are read."""
    import ctypes as C
    s = gpu.Scene.synthetic(6, 6, 9776, seed=0x5EED, width=960, height=540)
    f = s.frame()
    ctx = gpu.Context(s, "octree_gpu")
    ref = gpu.Context(s, "octree_gpu")
    nranks, d = 4, 1
    parts = _produce_all(ctx, f, nranks)
    dptr, n, g = _consume_rank(ctx, f, d, nranks, parts)
    ctx.cand_produce(f, 2, nranks)  # rewrites the entry / offset buffers
    t_ctx, st_ctx = _tiles_of_rank(ctx, f, d, nranks)
    gpu_lib().rt_hip_free(dptr)
    t_ref, st_ref = _tiles_of_rank(ref, f, d, nranks)
    assert_bitexact(t_ctx, t_ref, "render after produce -> consume -> produce")
    assert st_ctx["cand_entries"] == st_ref["cand_entries"] > 0
    # render -> produce -> stats: the render's kept-entry count is kept
    L = gpu_lib()
    per = gpu.tile_buffer_floats(f.width, f.height, nranks)
    dt = C.c_void_p()
    assert L.rt_hip_malloc(0, per * 4, C.byref(dt)) == 0
    ctx.render(f, d, nranks, dt.value)
    ctx.cand_produce(f, 0, nranks)
    st2 = ctx.stats()
    L.rt_hip_free(dt)
    assert st2["cand_entries"] == st_ref["cand_entries"]


def test_async_lists_repeated_frame(gpu):
    """A frame whose per-rank candidate lists were built before is rebuilt
    without a host read-back (the render path is asynchronous;
    the lists of one frame are deterministic, so its earlier total sizes the
    buffers, and the emission, the item passes, the sort and the render read
    every count on the device).  Repeated frames equal the first, read-back
    build bit for bit, with the same counts; switching frames or rank splits
    on one context goes back to one read-back build per new frame."""
    import ctypes as C
    s = gpu.Scene.synthetic(6, 6, 9776, seed=0x5EED, width=960, height=540)
    f = s.frame()
    ref, st_ref = gpu.Context(s, "octree_gpu").render_image(f)  # one frame: read-back build
    ctx = gpu.Context(s, "octree_gpu")
    small = gpu.Scene.synthetic(6, 6, 9776, seed=0x5EED, width=240, height=136)
    for frame_no in range(6):
        # frames 1-5: asynchronous lists; from the second build after the
        # frame's first, the refinement's kept entries compacted before the sort
        img, st = ctx.render_image(f)
        assert_bitexact(img, ref, f"frame {frame_no}: asynchronous candidate lists")
        assert (st["closest"], st["shadow"], st["cand_entries"]) == \
            (st_ref["closest"], st_ref["shadow"], st_ref["cand_entries"])
        if frame_no == 1:
            ctx.render_image(small.frame())  # another frame in between
    # rank splits on the same context: each (frame, rank) once with a read-back
    t0, st0 = _tiles_of_rank(ctx, f, 1, 4)
    for _ in range(3):
        t1, st1 = _tiles_of_rank(ctx, f, 1, 4)  # asynchronous (then also compacted)
        assert_bitexact(t1, t0, "rank 1 of 4, asynchronous lists")
        assert st1["cand_entries"] == st0["cand_entries"] > 0


def _panned_frame(gpu, scene, du):
    """The scene's frame with the eye moved du world units along the film's
    u axis (bench.py --camera-pan's new cameras)."""
    import ctypes as C
    cam = gpu.Camera()
    C.pointer(cam)[0] = scene.s.camera
    f0 = scene.frame()
    u = np.array([f0.u.x, f0.u.y, f0.u.z], np.float64)
    u /= np.linalg.norm(u)
    cam.position.x += float(u[0] * du)
    cam.position.y += float(u[1] * du)
    cam.position.z += float(u[2] * du)
    f = gpu.Frame()
    gpu._check(gpu.lib().rt_frame_from_camera(C.byref(cam), C.byref(f)), "frame")
    return f


def test_async_lists_new_cameras(gpu):
    """New cameras of the same size build their lists without a read-back,
    sized from the last build + headroom (rt_lists.cpp cand_prepare: the
    estimated shape, the kept count of the last frame, buffers grown with
    headroom so the build never frees mid-frame): a panned sequence on one
    context equals, frame by frame, the read-back build of a fresh context
    for the same camera -- image bit for bit and counts.  A jump far past the
    estimate is reported (RT_EHITBUF: the frame's lists outgrew their
    buffers) and the frame rendered again equals the reference, never an
    incomplete image returned as complete."""
    s = gpu.Scene.synthetic(6, 6, 9776, seed=0x5EED, width=960, height=540)
    ctx = gpu.Context(s, "octree_gpu")
    ctx.render_image(s.frame())  # the first frame of the size: read-back build
    for k, du in enumerate((0.02, 0.05, 0.09, 0.14, 3.0)):
        f = _panned_frame(gpu, s, du)
        ref, st_ref = gpu.Context(s, "octree_gpu").render_image(f)
        try:
            img, st = ctx.render_image(f)
        except gpu.RtError as e:
            assert e.code == -10 and k == 4, (k, e.code)  # only the far jump may outgrow the estimate
            img, st = ctx.render_image(f)
        assert_bitexact(img, ref, f"camera {k} (pan {du}): asynchronous lists of a new camera")
        assert (st["closest"], st["shadow"], st["cand_entries"]) == \
            (st_ref["closest"], st_ref["shadow"], st_ref["cand_entries"])


def test_triangle_parallel_lists_two_processes(gpu):
    """Two processes (ranks of torch.distributed.run, both on GPU 0, gloo
    for the exchange since RCCL needs a device per rank): each produces its
    half of the triangles, the entries go through rtgpu.exchange_cand_entries
    (bench.py's all-to-all), and each rank's render from the consumed lists
    equals its render from its own per-rank lists (tests/gpu_dist_worker.py)."""
    import json
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(REPO, "tests", "gpu_dist_worker.py")],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert line, r.stdout[-2000:]
    res = json.loads(line[-1])
    assert res["ok"], res


def test_three_process_frame_gloo(gpu):
    """The N-rank frame as bench.py runs it, in three processes on GPU 0 with
    the collectives on gloo (RCCL needs a device per rank): triangle-parallel
    lists exchanged, each rank's tiles rendered from them, the tile buffers
    gathered to rank 0 and assembled there by rt_hip_assemble -- the image
    equals rank 0's single-rank render bit for bit, with the same summed
    query counts (tests/gpu_dist_worker.py frame)."""
    import json
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "3",
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(REPO, "tests", "gpu_dist_worker.py"), "frame"],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert line, r.stdout[-2000:]
    res = json.loads(line[-1])
    assert res["ok"], res


def test_triangle_parallel_lists_c5_rank3(gpu):
    """The same on C5 itself for rank 3 of 8: the consumed lists' per-tile
    counts equal the per-rank build's and the rank's tiles are bit-identical."""
    s = gpu.Scene.synthetic(32, 32, 9776, seed=0x5EED, width=3840, height=2160)
    f = s.frame()
    ctx = gpu.Context(s, "octree_gpu")
    parts = _produce_all(ctx, f, 8)
    dptr, n, g = _consume_rank(ctx, f, 3, 8, parts)
    t_ext, st_ext = _tiles_of_rank(ctx, f, 3, 8)
    nt = gpu.rank_tile_count(f.width, f.height, 3, 8)
    e_ext = ctx.cand_tile_entries(nt)
    gpu_lib().rt_hip_free(dptr)
    t_ref, st_ref = _tiles_of_rank(ctx, f, 3, 8)
    e_ref = ctx.cand_tile_entries(nt)
    assert np.array_equal(e_ext, e_ref) and e_ref.sum() > 0
    assert_bitexact(t_ext, t_ref, "C5 rank 3/8: consumed vs per-rank lists")
    assert (st_ext["closest"], st_ext["shadow"]) == (st_ref["closest"], st_ref["shadow"])


def test_zero_normal_is_an_error(gpu, tmp_path):
    """cpu/hit.c:79 skips an object whose closest hit has an exactly zero
    interpolated normal; that rule is not reproduced, so a render that meets
    it must fail loudly (RT_EZERONORMAL from rt_hip_stats), never write a
    silently different image."""
    # v0 = (-2,0,0), v1 = (2,0,0), v2 = (-2,2,0) (LIFO order), normals
    # +z, -z, +z: on x = 0 (u = 0.5 exactly for the camera rays of column 16)
    # the interpolated normal (0.5 - v) - 0.5 + v is exactly zero -- the
    # oracle skips those hits (6 pixels of column 16 differ from the same
    # scene with n1 = +z).  (A zero vn would not do: normalize(0) is NaN.)
    sv = tmp_path / "zn.svati"
    sv.write_text("camera 32 32 0 0 -5 1 0 0 0 -1 0 60\na_light 1 1 1\n\nobject 3\nKa 1 1 1\n"
                  "v -2 2 0\nv 2 0 0\nv -2 0 0\nvn 0 0 1\nvn 0 0 -1\nvn 0 0 1\n")
    s = gpu.Scene.load_svati(str(sv))
    with pytest.raises(gpu.RtError) as e:
        gpu.Context(s, "flat").render_image(s.frame())
    assert e.value.code == -9


# ------------------------------------------------ gpu/rt compatibility mode
COMPAT_SCENES = ["cube", "spheres", "car-on-road", "island_smooth", "dir-light-shadows",
                 "point-light", "sphere-spec_smooth", "dark-night"]


@pytest.mark.parametrize("accel", ["flat", "octree", "octree_gpu"])
@pytest.mark.parametrize("scene", COMPAT_SCENES)
def test_compat_matches_oracle(gpu, scene_dir, scene, accel):
    """rt_hip_render_compat (gpu/rt semantics: 3x3 supersampling, uint8
    colours, <= 11 bounces) == the oracle's restatement of gpu/, byte for
    byte, and the same query counts.  Parity with gpu/rt itself is unpinned
    (no CUDA, no gpu/rt output in the reference; tests/test_compat.py)."""
    import oracle as orc
    s = gpu.Scene.load_svati(os.path.join(scene_dir, scene + ".svati"))
    s.set_size(64, 36)
    img, st = gpu.Context(s, accel).render_compat(s.camera)
    ref, cnt = orc.render_gpu(s.ptr, 64, 36, threads=8)
    bad = np.argwhere((img != ref).any(axis=2))
    assert len(bad) == 0, f"{scene} {accel}: {len(bad)} pixels differ, first {bad[:4].tolist()}"
    assert (st["closest"], st["shadow"]) == (cnt["closest"], cnt["shadow"])


@pytest.mark.parametrize("accel", ["octree", "octree_gpu"])
def test_compat_full_frame_octree_vs_flat(gpu, accel):
    """gpu/rt compatibility mode over a whole frame of a million-triangle
    synthetic scene (10 x 10 spheres of 9,776 triangles + ground, 320 x 180
    output = 960 x 540 rays): the octree walk with the compat camera's
    candidate lists (csrc/rt_cand.hip CandParams::compat) equals brute force
    (RT_ACCEL_FLAT, the restated gpu/hit.cu test over every triangle) byte
    for byte -- grazing camera rays whose float garbage hit lies beyond the
    walk's slack included (/root/reference/gpu/raytracer.cu:87-129)."""
    s = gpu.Scene.synthetic(10, 10, 9776, seed=0x5EED, width=320, height=180)
    assert s.triangle_count > 970000
    img_f, st_f = gpu.Context(s, "flat").render_compat(s.camera)
    ctx = gpu.Context(s, accel)
    img_o, st_o = ctx.render_compat(s.camera)
    assert st_o["cand_entries"] > 0
    bad = np.argwhere((img_o != img_f).any(axis=2))
    assert len(bad) == 0, f"{len(bad)} pixels differ, first {bad[:4].tolist()}"
    assert (st_o["closest"], st_o["shadow"]) == (st_f["closest"], st_f["shadow"])
    ctx.set_exact_camera(False)  # A/B: the walk alone (reported, not asserted)
    img_n, _ = ctx.render_compat(s.camera)
    print(f"compat {accel}: {int((img_n != img_f).any(axis=2).sum())} pixels differ without the lists")


def test_compat_candidate_lists_match_host(gpu):
    """The compatibility mode's device-built camera lists (one sample per
    pixel of the 3x frame) equal the host re-derivation from the same
    classify/raster code, footprint by footprint and tile by tile."""
    s = gpu.Scene.synthetic(8, 6, 9776, seed=0x5EED, width=640, height=360)
    ctx = gpu.Context(s, "octree_gpu")
    ctx.render_compat(s.camera)
    v = ctx.cand_verify_compat(s.camera)
    assert v["listed"] > 0 and v["entries"] > 0, v
    assert v["fp_mismatch"] == 0 and v["tile_mismatch"] == 0 and v["filter_violation"] == 0, v


def test_compat_large_frame_sampled(gpu):
    """gpu/rt compatibility mode on the device-built octree at 1280x720
    (3840x2160 rays) of a 147k-triangle synthetic scene: 96 sampled output
    pixels (each the downscale of its 9 rays) byte-identical to the oracle."""
    import oracle as orc
    s = gpu.Scene.synthetic(4, 4, 9776, seed=0x5EED, width=1280, height=720)
    img, st = gpu.Context(s, "octree_gpu").render_compat(s.camera)
    assert st["pixels"] == 9 * 1280 * 720
    rng = np.random.default_rng(5)
    pix = np.stack([rng.integers(0, 720, 96), rng.integers(0, 1280, 96)], axis=1)
    ref, _ = orc.render_gpu(s.ptr, 1280, 720, pixels=pix, threads=8)
    assert np.array_equal(img[pix[:, 0], pix[:, 1]], ref)


def test_rt_gpu_cli_png(gpu, scene_dir, tmp_path):
    """lib/rt_gpu = gpu/rt's command line: same usage error, and the PNG it
    writes decodes to the oracle's gpu-mode image."""
    import oracle as orc
    from test_compat import decode_png
    exe = os.path.join(REPO, "raytracing-gpu_amd", "lib", "rt_gpu")
    r = subprocess.run([exe, "x.svati"], capture_output=True, text=True)
    assert r.returncode == 1 and "usage:" in r.stderr and "file.svati output.png" in r.stderr
    src = tmp_path / "sp.svati"
    text = open(os.path.join(scene_dir, "spheres.svati")).read().split("\n")
    text = [("camera 80 45 " + " ".join(l.split()[3:])) if l.startswith("camera") else l
            for l in text]
    src.write_text("\n".join(text))
    out = tmp_path / "sp.png"
    r = subprocess.run([exe, str(src), str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    s = gpu.Scene.load_svati(str(src))
    ref, _ = orc.render_gpu(s.ptr, 80, 45, threads=8)
    assert np.array_equal(decode_png(str(out)), ref)


@pytest.mark.parametrize("exact", [True, False])
@pytest.mark.parametrize("li", [1, 2])
def test_light_buffer_probe_grazing(gpu, li, exact):
    """Shadow rays built to graze triangles (module helper grazing_origins):
    the light buffer's answer equals brute force over every triangle for
    every origin when its footprints are proven (rt_hip_set_exact_shadows);
    the slack-grown default is reported, and must agree on this scene too."""
    s = gpu.Scene.synthetic(3, 3, 9776, seed=0x5EED, width=96, height=54)
    tri = s.triangles_array()
    L = s.s.lights[li]
    lv = np.array([L.v.x, L.v.y, L.v.z], np.float64)
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from grazing import grazing_origins
    o = grazing_origins(tri, int(L.type), lv, 4000, 40)
    assert len(o) > 50000
    ctx = gpu.Context(s, "octree_gpu")
    ctx.set_exact_shadows(exact)
    got = ctx.probe_shadows(li, o)
    ref = ctx.probe_shadows(li, o, brute=True)
    bad = np.flatnonzero(got != ref)
    assert 0.01 < ref.mean() < 0.99, ref.mean()
    assert len(bad) == 0, (f"{len(bad)} of {len(o)} grazing shadow rays differ from brute force "
                           f"(buffer lit, brute shadowed: {int((~got & ref).sum())}); first {bad[:5].tolist()}")


def _grazing_probe(gpu, scene_dir, scene):
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from grazing import grazing_rays
    if scene == "synthetic":
        s = gpu.Scene.synthetic(3, 3, 9776, seed=0x5EED, width=96, height=54)
    else:
        s = gpu.Scene.load_svati(os.path.join(scene_dir, scene + ".svati"))
    tri = s.triangles_array()
    o, d = grazing_rays(tri, 3000, 40)
    assert len(o) > 60000
    return s, tri, o, d


@pytest.mark.parametrize("scene,accel", [("synthetic", "octree_gpu"), ("synthetic", "octree"),
                                         ("car-on-road", "octree"), ("car-on-road", "octree_gpu")])
def test_reflection_probe_grazing(gpu, scene_dir, scene, accel):
    """Reflection rays exact by proof (rt_hip_set_exact_reflections, DESIGN.md
    §2 "Reflection rays").  Rays built to cross triangles' planes at grazing
    angles (1e-7 .. 3e-2 rad, tools/grazing.py grazing_rays: where the float
    Moller-Trumbore error region is widest), half of them from origins on
    other triangles as a reflection ray's are, queried through the proven
    reflection walk (rt_hip_probe_closest): the winner's prim and new_dist
    bits equal brute force over every triangle for EVERY ray -- including
    the coplanar-grazing rays the culling slack misses (round 5)."""
    s, tri, o, d = _grazing_probe(gpu, scene_dir, scene)
    ctx = gpu.Context(s, accel)
    ctx.set_exact_reflections(True)
    pw, dw = ctx.probe_closest(o, d)
    pb, db = ctx.probe_closest(o, d, brute=True)
    hit = pb != 0xFFFFFFFF
    assert 0.05 < hit.mean() < 0.999, hit.mean()
    bad = np.flatnonzero((pw != pb) | (dw.view(np.uint32) != db.view(np.uint32)))
    assert len(bad) == 0, (f"{len(bad)} of {len(o)} grazing reflection rays differ from brute force: "
                           f"first {bad[:5].tolist()}")


@pytest.mark.parametrize("scene,accel", [("synthetic", "octree_gpu"), ("car-on-road", "octree")])
def test_reflection_probe_grazing_slack_walk(gpu, scene_dir, scene, accel):
    """The same probe through the default reflection walk (the culling slack,
    not proven): a measurement of its residual class, not a guarantee.  Every
    differing ray must be a float garbage hit on a triangle whose plane
    (nearly) contains the ray (tools/grazing.py coplanar_grazing: a, s.h and
    d.q of cpu/hit.c:15-33 are all rounding noise) -- the class round 5 found
    and the exact mode closes."""
    s, tri, o, d = _grazing_probe(gpu, scene_dir, scene)
    ctx = gpu.Context(s, accel)
    pw, dw = ctx.probe_closest(o, d)
    pb, db = ctx.probe_closest(o, d, brute=True)
    bad = np.flatnonzero((pw != pb) | (dw.view(np.uint32) != db.view(np.uint32)))
    from grazing import coplanar_grazing, float_mt
    unexplained = []
    for i in bad:
        idx, dist = float_mt(tri, o[i], d[i])
        assert len(idx) and dist.min().view(np.uint32) == db[i].view(np.uint32), i  # brute's winner found
        if not coplanar_grazing(tri[idx[np.argmin(dist)]], o[i], d[i]):
            unexplained.append(int(i))
    print(f"{scene}/{accel} slack walk: {len(o)} grazing rays, {len(bad)} differ, all coplanar-grazing: "
          f"{not unexplained}")
    assert not unexplained, unexplained[:5]


def test_empty_rank_on_fresh_context(gpu, scene_dir, manifest):
    """A rank past the frame's last tile block renders nothing: 96x54 over 8
    ranks has 3 x 2 blocks of 4x4 tiles on the diagonal map (block (bx, by) ->
    rank (bx + by) mod 8), so ranks 4 to 7 own none.  On a fresh
    context the render succeeds with zero counts, and the 8-rank assemble of
    all ranks (the empty ones' buffers as padding) is the golden image."""
    import ctypes as C
    case = next(c for c in manifest if c["scene"] == "cube" and c["width"] == 96)
    s = gpu.Scene.load_svati(os.path.join(scene_dir, "cube.svati"))
    s.set_size(case["width"], case["height"])
    f = s.frame()
    assert gpu.rank_tile_count(f.width, f.height, 7, 8) == 0
    fresh = gpu.Context(s, "octree")
    t, st = _tiles_of_rank(fresh, f, 7, 8)
    assert len(t) == 0 and st["closest"] == 0 and st["shadow"] == 0 and st["pixels"] == 0
    ctx = gpu.Context(s, "octree")
    n = 8
    per = gpu.tile_buffer_floats(f.width, f.height, n)
    L = gpu.lib()
    dg, drgb = C.c_void_p(), C.c_void_p()
    assert L.rt_hip_malloc(0, per * n * 4, C.byref(dg)) == 0
    assert L.rt_hip_malloc(0, f.width * f.height * 12, C.byref(drgb)) == 0
    tot = 0
    for r in (7, 6, 0, 1, 2, 3, 4, 5):  # the empty ranks first, on this context too
        ctx.render(f, r, n, dg.value + r * per * 4)
        tot += ctx.stats()["closest"]
    ctx.assemble(f, dg.value, n, drgb.value)
    img = np.empty((f.height, f.width, 3), np.float32)
    ctx.stats()
    assert L.rt_hip_memcpy_d2h(img.ctypes.data_as(C.c_void_p), drgb, img.nbytes) == 0
    L.rt_hip_free(dg)
    L.rt_hip_free(drgb)
    assert_bitexact(img, golden_image(case), "8 ranks, two of them empty")
    assert tot == case["closest"]


@pytest.mark.parametrize("exact", [False, True])
def test_light_buffer_build_failure_falls_back_to_walk(gpu, exact):
    """A light buffer that cannot be built (here: capped at one entry by the
    test hook) leaves that light's shadow queries on the octree walk instead
    of failing the context -- the proven walk in the exact-shadow mode (the
    default); the image is unchanged and equals brute force."""
    s = gpu.Scene.synthetic(3, 3, 9776, seed=0x5EED, width=320, height=180)
    f = s.frame()
    img_f, st_f = gpu.Context(s, "flat").render_image(f)
    ctx = gpu.Context(s, "octree_gpu")
    ctx.set_exact_shadows(exact)
    img, st = ctx.render_image(f)
    assert ctx.info()["lightbuf_failed"] == 0 and ctx.info()["lightbuf_entries"] > 0
    assert ctx.info()["lightbuf_fail_reason"] == ""
    ctx.set_lightbuf_entry_cap(1)
    assert ctx.info()["lightbuf_failed"] == 2 and ctx.info()["lightbuf_entries"] == 0
    assert "entries" in ctx.info()["lightbuf_fail_reason"]
    img2, st2 = ctx.render_image(f)
    assert_bitexact(img2, img, "shadow queries on the walk after a failed light-buffer build")
    assert (st2["closest"], st2["shadow"]) == (st["closest"], st["shadow"])
    assert_bitexact(img2, img_f, "walk fallback vs brute force")
    if exact:
        assert ctx.info()["shadow_mu_max"] >= 1.0  # the proven walk's multipliers were built


def test_exact_shadows_more_than_32_lights(gpu, tmp_path):
    """Exact-shadow mode with 35 lights: the off-box queue carries the bits
    of lights 0..31 only, so it is off and every off-box query is counted
    (RT_EINEXACT) -- the render equals brute force or fails loudly, never
    silently drops lights 32 and up."""
    base = gpu.Scene.synthetic(3, 3, 9776, seed=0x5EED, width=160, height=90)
    src = tmp_path / "base.svati"
    base.write_svati(str(src))
    lines = open(src).read().split("\n")
    extra = [f"p_light 0.02 0.03 0.04 {-6 + 0.4 * k:.2f} {3 + 0.1 * k:.2f} -4" if k % 2 else
             f"d_light 0.03 0.02 0.01 {0.1 * (k - 16):.2f} -1 0.5" for k in range(32)]
    cam = next(i for i, ln in enumerate(lines) if ln.startswith("camera"))
    sv = tmp_path / "lights35.svati"
    sv.write_text("\n".join(lines[:cam + 1] + extra + lines[cam + 1:]))
    s = gpu.Scene.load_svati(str(sv))
    assert s.s.light_count == 35
    f = s.frame()
    img_f, st_f = gpu.Context(s, "flat").render_image(f)
    ctx = gpu.Context(s, "octree_gpu")
    ctx.set_exact_shadows(True)
    try:
        img, st = ctx.render_image(f)
    except gpu.RtError as e:
        assert e.code == gpu.Context.RT_EINEXACT, e
        return
    assert_bitexact(img, img_f, "35 lights, exact shadows vs brute force")
    assert (st["closest"], st["shadow"]) == (st_f["closest"], st_f["shadow"])


@pytest.mark.parametrize("exact", [False, True])
def test_light_buffer_entries_match_host_survey(gpu, exact):
    """The device build of the light buffers (count -> scan -> emit, small and
    workgroup footprints, band rows) lists exactly the entries the host survey
    of the same footprint code counts (rt_lightbuf_survey), light by light."""
    s = gpu.Scene.synthetic(4, 4, 9776, seed=0x5EED, width=96, height=54)
    ctx = gpu.Context(s, "octree_gpu")
    ctx.set_exact_shadows(exact)
    info = ctx.info()
    host = [s.lightbuf_survey(li, exact, 1) for li in range(s.s.light_count)
            if int(s.s.lights[li].type) in (1, 2)]
    assert info["lightbuf_entries"] == sum(h["entries"] for h in host), (info, host)
    assert info["lightbuf_global"] == sum(h["global"] for h in host)
    if exact:
        assert info["lightbuf_band"] == sum(h["band"] for h in host)
        assert info["lightbuf_never"] == sum(h["never"] for h in host)


@pytest.mark.parametrize("accel", ["octree_gpu", "octree"])
def test_camera_refine_on_off(gpu, accel):
    """The per-tile refinement of the candidate lists (rt_hip_set_camera_refine,
    csrc/rt_cand.hip tile_keep) only drops entries no camera ray of their tile
    can accept: the frame is bit-identical with it off, with fewer entries on;
    the host re-derivation matches the device lists both ways (the host applies
    the same refinement), N = 1 and rank 2 of 3."""
    s = gpu.Scene.synthetic(8, 6, 9776, seed=0x5EED, width=1920, height=1080)
    f = s.frame()
    ctx = gpu.Context(s, accel)
    img_on, st_on = ctx.render_image(f)
    ctx.set_camera_refine(False)
    img_off, st_off = ctx.render_image(f)
    assert np.array_equal(img_on.view(np.uint32), img_off.view(np.uint32))
    assert st_on["closest"] == st_off["closest"] and st_on["shadow"] == st_off["shadow"]
    assert 0 < st_on["cand_entries"] < st_off["cand_entries"], (st_on["cand_entries"], st_off["cand_entries"])
    for on in (False, True):
        ctx.set_camera_refine(on)
        for nranks, rank in ((1, 0), (3, 2)):
            _tiles_of_rank(ctx, f, rank, nranks)
            v = ctx.cand_verify(f, rank, nranks)
            assert v["fp_mismatch"] == 0 and v["tile_mismatch"] == 0, (on, nranks, rank, v)
            assert v["filter_violation"] == 0, (on, nranks, rank, v)


def test_bench_json_contract(gpu, tmp_path):
    """bench.py as the driver runs it (one GPU, a small workload, a short CPU
    baseline): one JSON line on stdout with the contract's fields -- the
    metric and unit, whole-job value, per-step times (replay and fresh
    camera), the roofline object of the dominant kernel and the CPU baseline
    whose sampled pixels match the GPU image bit for bit."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--workload", "c1", "--steps", "3",
                        "--warmup", "1", "--cpu-seconds", "2", "--cpu-threads", "2"],
                       capture_output=True, text=True, timeout=240, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "ms_per_step_fresh",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["metric"] == "Mrays/sec (primary+shadow) at 3840x2160" and d["unit"] == "Mrays/s"
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["ms_per_step_fresh"] > 0
    assert "workload" in d["config"]
    rf = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rf, k
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and 0 < rf["frac"] < 1
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    cpu = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cpu, k
    assert cpu["kind"] == "port" and cpu["cores"] == 2 and cpu["value"] > 0
    assert cpu["sample_pixels_bitexact_vs_gpu"] is True
