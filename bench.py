#!/usr/bin/env python3
"""bench.py -- Mrays/s (closest-hit + shadow queries) of the MI355X render path.

A "step" renders one whole frame of the workload: every rank builds the
frame's camera-ray candidate lists (per rank, or triangle-parallel with one
all-to-all from N = 4) and renders its 8x8 tiles (4x4-tile blocks, block
(bx, by) to rank (bx + by) mod N, csrc/rt_tiles.h) through the C ABI of
lib/librtgpu.so on torch's current stream, rank
tile buffers are gathered to rank 0 with one RCCL gather (torch.distributed
"nccl" backend = RCCL over xGMI), and rank 0 assembles the PPM-order float
image.  Scene image and octree are built and uploaded before timing (inputs
resident in HBM).  The render kernel's own duration is measured with HIP
events on its stream (rt_hip_set_timing), every timed step.

Default workload = config C5 (BASELINE.json): the deterministic synthetic
10M-triangle sphere field at 3840x2160, octree traversal.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c5|c4|c3|c2|c1]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Prints ONE JSON line on rank 0 (plus progress on stderr).
"""
import argparse
import ctypes
import gzip
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
import rtgpu  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
# Algorithmic bytes of one render launch: every record the
# kernel fetches (a wave-uniform fetch of the packet walk counts once) plus
# the rays' own state and the framebuffer write.
NODE_BYTES = 32        # octree node record (host/rt_cull.h)
TRI_BYTES = 48         # triangle record (host/rt_internal.h)
RAY_BYTES = 24         # origin + direction of a query
NORMAL_BYTES = 36      # 3 vertex normals of a closest-hit winner
PIXEL_BYTES = 12       # f32 RGB written per pixel
HIT_RECORD_BYTES = 36  # hit record (P, N, coef, object: 2 float4) + its path link
MATERIAL_BYTES = 48    # material of the hit object
TERM_BYTES = 16        # a record's reflection term (float4)
NODE_MU_BYTES = 8      # a node's shadow slack multipliers (csrc/rt_shadow.hip)
N_SIMD = 1024          # 256 CUs x 4 SIMDs (MI355X_MICROARCH.md)
N_XCD = 8

WORKLOADS = {
    "c5": dict(kind="synthetic", accel="octree_gpu", W=3840, H=2160,
               desc="C5 synthetic 10M-triangle sphere field (32x32 UV spheres of 53 stacks x 94 "
                    "slices = 9776 tris + ground quad, seed 0x5EED, BASELINE.md), 3840x2160, "
                    "device-built octree, exact camera rays (per-frame candidate lists)"),
    "c4": dict(kind="svati", scene="car-on-road", accel="octree", W=3840, H=2160,
               desc="C4 car-on-road.svati at 3840x2160, octree"),
    "c3": dict(kind="svati", scene="island_smooth", accel="octree", W=1920, H=1080,
               desc="C3 island_smooth.svati at 1920x1080, octree"),
    "c2": dict(kind="svati", scene="spheres", accel="flat", W=1920, H=1080,
               desc="C2 spheres.svati at 1920x1080, flat triangle list"),
    "c1": dict(kind="svati", scene="cube", accel="flat", W=256, H=256,
               desc="C1 cube.svati at 256x256, flat triangle list"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def load_scene(wl, tmpdir):
    if wl["kind"] == "synthetic":
        return rtgpu.Scene.synthetic(32, 32, 9776, seed=0x5EED, width=wl["W"], height=wl["H"])
    src = os.path.join(REPO, "tests", "golden", "scenes", wl["scene"] + ".svati.gz")
    path = os.path.join(tmpdir, wl["scene"] + ".svati")
    with gzip.open(src, "rb") as i, open(path, "wb") as o:
        o.write(i.read())
    s = rtgpu.Scene.load_svati(path)
    s.set_size(wl["W"], wl["H"])
    return s


def _oracle():
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc
    orc.lib()
    return orc


def _sample_loop(orc, scene, W, H, pixels, seconds, threads, gpu_img, out):
    """Render pixels (deterministic order) with the oracle until `seconds`
    pass; accumulates queries, pixels and mismatches vs the GPU image."""
    t0 = time.perf_counter()
    done = 0
    batch = max(1, threads)
    while time.perf_counter() - t0 < seconds and done < len(pixels):
        pix = pixels[done:done + batch]
        vals, cnt = orc.render(scene.ptr, W, H, pixels=pix, threads=threads)
        out["closest"] += cnt["closest"]
        out["shadow"] += cnt["shadow"]
        if gpu_img is not None:
            g = gpu_img[pix[:, 0], pix[:, 1]]
            out["mism"] += int((g.view(np.uint32) != vals.view(np.uint32)).any(axis=1).sum())
        done += len(pix)
        if time.perf_counter() - t0 < seconds / 4:
            batch *= 2
    out["pixels"] += done


def cgroup_cpu_quota():
    """CPUs the process's cgroup may use (quota / period), None when unlimited
    or unreadable: cgroup v2 cpu.max, else v1 cfs_quota_us / cfs_period_us."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else round(q / per, 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(scene, W, H, seconds, threads, gpu_img):
    """The oracle (plain-C restatement of cpu/rt, brute force like the
    reference) on bounded deterministic pixel samples of the same frame, in
    the reference's own mode (SURVEY.md §8(d) "Mode A": 4 threads, one image
    quadrant each, cpu/raytracer.c:92-127) and on all the cores this process
    may use ("Mode B").  Returns the Mode B line with Mode A beside it."""
    import threading
    orc = _oracle()
    rng = np.random.default_rng(1234)

    def pix_of(idx):
        return np.stack([idx // W, idx % W], axis=1).astype(np.int32)

    # Mode A: quadrant q = (row half, column half) of cpu/raytracer.c:99-114,
    # each thread its own quadrant's pixels in a deterministic random order
    quads = []
    for rh in (0, 1):
        for ch in (0, 1):
            rows = np.arange(rh * (H // 2), H // 2 + rh * (H - H // 2))
            cols = np.arange(ch * (W // 2), W // 2 + ch * (W - W // 2))
            idx = (rows[:, None] * W + cols[None, :]).ravel()
            quads.append(pix_of(rng.permutation(idx)))
    res_a = [dict(closest=0, shadow=0, pixels=0, mism=0) for _ in quads]
    t0 = time.perf_counter()
    th = [threading.Thread(target=_sample_loop,
                           args=(orc, scene, W, H, q, seconds / 2, 1, gpu_img, r))
          for q, r in zip(quads, res_a)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    el_a = time.perf_counter() - t0
    qa = sum(r["closest"] + r["shadow"] for r in res_a)
    # Mode B: every core of this process's share, one shared pixel sample
    res_b = dict(closest=0, shadow=0, pixels=0, mism=0)
    t0 = time.perf_counter()
    _sample_loop(orc, scene, W, H, pix_of(rng.permutation(W * H)), seconds / 2, threads, gpu_img,
                 res_b)
    el_b = time.perf_counter() - t0
    qb = res_b["closest"] + res_b["shadow"]
    mism = res_b["mism"] + sum(r["mism"] for r in res_a)
    return {
        "value": qb / el_b / 1e6,
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "sample": f"Mode B: {res_b['pixels']} pixels ({res_b['closest']} closest + {res_b['shadow']} "
                  f"shadow queries) of the same {W}x{H} frame, deterministic random order, "
                  f"{el_b:.1f} s on {threads} threads; oracle/rt_oracle.c (brute force like cpu/rt, "
                  f"-O2)",
        "host_cpus": os.cpu_count(),
        # what this process may actually run on, observed (not asserted)
        "affinity_cpus": len(os.sched_getaffinity(0)),
        "cgroup_cpu_quota": cgroup_cpu_quota(),
        "mode_a": {"value": qa / el_a / 1e6, "unit": "Mrays/s", "cores": 4,
                   "sample": f"{sum(r['pixels'] for r in res_a)} pixels, {el_a:.1f} s, 4 threads, "
                             f"one image quadrant each (cpu/raytracer.c:92-127)"},
        "sample_pixels_bitexact_vs_gpu": (mism == 0) if gpu_img is not None else None,
    }


def device_code_hash():
    """sha256 of everything that decides what the kernels do: the HIP and
    C-ABI sources (raytracing-gpu_amd/csrc/), the host headers they include,
    the public headers and the build flags (Makefile).  tools/gpu_profile.sh
    writes it next to the PMC passes it takes (device_hash.txt)."""
    import glob
    import hashlib
    pk = os.path.join(REPO, "raytracing-gpu_amd")
    files = sorted(glob.glob(os.path.join(pk, "csrc", "*")) + glob.glob(os.path.join(pk, "host", "*.h")) +
                   glob.glob(os.path.join(REPO, "include", "*.h")) + [os.path.join(pk, "Makefile")])
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.relpath(f, REPO).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def latest_profile(workload, name):
    """Newest profiles/r*_<workload>/<name> (round-letter order) whose PMC
    passes were taken of THIS device code (its device_hash.txt equals
    device_code_hash()), or None: counters of other kernels are never
    reported as this run's."""
    import glob
    want = device_code_hash()
    for hit in sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_{workload}", name)), reverse=True):
        hf = os.path.join(os.path.dirname(hit), "device_hash.txt")
        if os.path.exists(hf) and open(hf).read().strip() == want:
            return hit
    return None


def frame_checked(ctx, rank, world, frame, steps, what, fatal=True):
    """The device's per-frame checks of the frames rendered since the last
    reset (rt_hip_frame_check): refuses (SystemExit, no JSON line) unless
    every one was complete and exact by rt_hip_stats' conditions.  Returns
    the frames' closest-hit + shadow queries summed over the ranks (not
    fatal: None and the reason instead of exiting)."""
    fl, nf, qc, qs = ctx.frame_check()
    has_tiles = rtgpu.rank_tile_count(frame.width, frame.height, rank, world) > 0
    bad = fl != 0 or (has_tiles and nf != steps)
    t = torch.tensor([1.0 if bad else 0.0, float(qc + qs)], dtype=torch.float64, device=f"cuda:{torch.cuda.current_device()}")
    if world > 1:
        dist.all_reduce(t)
    if bad or t[0].item() > 0:
        why = ", ".join(v for k, v in ctx.FRAME_FLAGS.items() if fl & k) or f"{nf} of {steps} frames checked"
        if not fatal:
            return None, why
        raise SystemExit(f"[rank {rank}] {what} loop: incomplete frame(s) ({why}): no value printed")
    return (float(t[1].item()), None) if not fatal else float(t[1].item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="c5", choices=sorted(WORKLOADS))
    ap.add_argument("--accel", default=None, choices=["flat", "octree", "octree_gpu"])
    ap.add_argument("--cpu-seconds", type=float, default=20.0,
                    help="CPU baseline budget (split between Mode A and Mode B)")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="Mode B threads (default: this process's CPU share -- the box's "
                         "OMP_NUM_THREADS -- capped by os.cpu_count())")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--camera-pan", type=float, default=1.0,
                    help="after the replay loop, time --steps more frames each with its own camera, "
                         "moved along the image's u axis by this many pixels of image shift per step at "
                         "the scene centre's depth (a new view every frame: nothing of an earlier "
                         "identical frame is reused); 0 = skip")
    ap.add_argument("--cull-slack", type=float, default=None,
                    help="octree culling slack override (tuning; default = library default)")
    ap.add_argument("--camera-slack", type=float, default=None,
                    help="camera-ray culling slack override (tuning; default = library default)")
    ap.add_argument("--policy", type=int, default=None,
                    help="octree traversal policy (A/B only; rt_hip_set_policy, default = library "
                         "default 0)")
    ap.add_argument("--exact-shadows", type=int, default=None, choices=[0, 1],
                    help="shadow queries through proven (1) or slack-grown (0) light buffers "
                         "(rt_hip_set_exact_shadows; default = library default, proven)")
    ap.add_argument("--exact-reflections", type=int, default=None, choices=[0, 1],
                    help="reflection rays through the proven walk (rt_hip_set_exact_reflections; default off)")
    ap.add_argument("--lists", default=None, choices=["rank", "partition"],
                    help="camera candidate lists of an N-GPU frame: built by every rank for its "
                         "tiles over all triangles ('rank'), or triangle-parallel -- each rank "
                         "1/N of the triangles for every rank's tiles, one all-to-all "
                         "('partition', rt_hip_cand_produce / consume); default: partition "
                         "when N >= 4")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC summary (tools/pmc_traffic.py) to report as roofline.traffic")
    ap.add_argument("--valu-json", default=None,
                    help="PMC summary (tools/gpu_profile.sh pmc_sq.json, SQ counters) to report as sq")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    wl = dict(WORKLOADS[args.workload])
    if args.accel:
        wl["accel"] = args.accel
        wl["desc"] = wl["desc"] + f" [accel overridden: {args.accel}]"
    W, H = wl["W"], wl["H"]

    with tempfile.TemporaryDirectory() as td:
        t = time.perf_counter()
        scene = load_scene(wl, td)
    ntri = scene.triangle_count
    ctx = rtgpu.Context(scene, wl["accel"], device=local)
    if args.cull_slack is not None:
        ctx.set_cull_slack(args.cull_slack)
    if args.camera_slack is not None:
        ctx.set_camera_slack(args.camera_slack)
    if args.policy is not None:
        ctx.set_policy(args.policy)
    if args.exact_shadows is not None:
        ctx.set_exact_shadows(bool(args.exact_shadows))
    if args.exact_reflections:
        ctx.set_exact_reflections(True)
    info = ctx.info()
    log(f"[rank {rank}] scene {ntri} triangles, accel {wl['accel']}: {info['tri_refs']} records, "
        f"{info['nodes']} nodes, build {info['build_seconds']:.1f}s, setup {time.perf_counter()-t:.1f}s")
    frame = scene.frame()
    per = rtgpu.tile_buffer_floats(W, H, world)
    tiles = torch.empty(per, dtype=torch.float32, device=dev)
    gathered = torch.empty(per * world, dtype=torch.float32, device=dev) if rank == 0 else None
    rgb = torch.empty(W * H * 3, dtype=torch.float32, device=dev) if rank == 0 else None
    # a real (non-null) stream: the render, the events around it, the gather
    # and the assemble are all ordered on it
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    sh = stream.cuda_stream
    assert sh, "expected a non-null HIP stream handle"

    # instrumented pass (untimed): algorithmic work per frame for the roofline
    ctx.set_count_work(True)
    for attempt in range(2):
        ctx.render(frame, rank, world, tiles.data_ptr(), sh)
        try:
            work = ctx.stats()
            break
        except rtgpu.RtError as e:  # RT_EHITBUF: the buffer grew to the frame's need
            if e.code != -10 or attempt:
                raise
    ctx.set_count_work(False)

    # N >= 4: the per-rank lists' fixed part (every triangle on every rank)
    # outweighs the second sort and the exchange
    partition = (args.lists or ("partition" if world >= 4 else "rank")) == "partition" and \
        wl["accel"] != "flat"
    send = [None]
    part_ms = []  # host wall time of produce + exchange + consume enqueue, timed steps only
    timed = [False]

    def exchange_lists(frame):
        # triangle-parallel lists: this rank's slice of the triangles for
        # every rank's tiles -> all-to-all over RCCL -> this rank's lists
        counts, ng = ctx.cand_produce(frame, rank, world, sh)
        ptr, n = ctx.cand_send_buffer()
        if send[0] is None or send[0].shape[0] < n:
            send[0] = torch.empty((n + n // 4 + 1024, 3), dtype=torch.int32, device=dev)
        rtgpu.lib().rt_hip_memcpy_d2d(ctypes.c_void_p(send[0].data_ptr()), ctypes.c_void_p(ptr), n * 12,
                                      ctypes.c_void_p(sh))
        if world > 1:
            recv, g = rtgpu.exchange_cand_entries(dist, send[0], counts, ng)
        else:
            recv, g = send[0][:n], ng
        ctx.cand_consume(frame, rank, world, recv.data_ptr(), int(recv.shape[0]), g, sh)

    def step(frame=frame):
        if partition:
            t = time.perf_counter()
            exchange_lists(frame)
            if timed[0]:
                part_ms.append((time.perf_counter() - t) * 1e3)
        ctx.render(frame, rank, world, tiles.data_ptr(), sh)
        if world > 1:
            dist.gather(tiles, list(gathered.view(world, per)) if rank == 0 else None, dst=0)
            if rank == 0:
                ctx.assemble(frame, gathered.data_ptr(), world, rgb.data_ptr(), sh)
        else:
            ctx.assemble(frame, tiles.data_ptr(), 1, rgb.data_ptr(), sh)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    retry = 0
    try:
        st = ctx.stats()
    except rtgpu.RtError as e:  # the first frame sized the hit-record buffer: once more
        if e.code != -10:
            raise
        retry = 1
    # every rank steps again if any rank must (step() holds a collective)
    flag = torch.tensor([retry], dtype=torch.int32, device=dev)
    if world > 1:
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
    if int(flag.item()):
        step()
        torch.cuda.synchronize()
        st = ctx.stats()
    assert st["depth_overflow"] == 0 and st["shadow_unproven"] == 0
    counts = torch.tensor([st["closest"], st["shadow"], st["hits"], st["pixels"],
                           work["node_visits"], work["tri_tests"], work["hits"],
                           work["closest"] + work["shadow"],
                           work["closest_node_lanes"], work["closest_tri_lanes"],
                           work["shadow_node_lanes"], work["shadow_tri_lanes"],
                           work["closest"], work["shadow"], st["cand_entries"],
                           work["shadow_node_visits"], work["shadow_tri_tests"]],
                          dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(counts)
    (closest, shadow, hits, pixels, nodes, tris, whits, wq, cl_nodes, cl_tris, sh_nodes, sh_tris,
     wcl, wsh, cand_entries, sh_wnodes, sh_wtris) = [float(x) for x in counts.tolist()]

    # HIP events around the candidate lists and the render kernel of every
    # timed step, on the stream they run on (rt_hip_set_timing)
    ctx.set_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.frame_check()  # reset: the timed frames' own checks and query counts follow
    t0 = time.perf_counter()
    timed[0] = True
    for _ in range(args.steps):
        step()
    timed[0] = False
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    ft = ctx.frame_times(min(args.steps, 1024))
    kt = ctx.kernel_times(min(args.steps, 1024))
    # every timed frame complete: the conditions rt_hip_stats reports, checked
    # on the device at the end of each frame (rt_hip_frame_check) -- a line is
    # never printed for a timed region with an incomplete or unproven frame
    timed_q = frame_checked(ctx, rank, world, frame, args.steps, "timed")
    ctx.set_timing(False)

    # the same number of frames again, each with a new camera (panned
    # --camera-pan pixels per step): a one-shot render or an animation
    # reuses nothing of an earlier identical frame (the lists' sizes, kept
    # count and work order are rebuilt with their read-backs)
    # the timed frame's image, for the CPU baseline's pixel check (the
    # fresh-camera frames below overwrite rgb with panned views)
    img_timed = rgb.clone() if rank == 0 and world == 1 and not args.no_cpu else None
    fresh = None
    if args.camera_pan > 0:
        cam0 = rtgpu.Camera()
        ctypes.pointer(cam0)[0] = scene.s.camera
        fu = (frame.u.x, frame.u.y, frame.u.z)
        # cpu/rt's film lies L world units from the eye with one unit per
        # pixel (cpu/raytracer.c:82-86), so moving the eye by D / L units
        # shifts the image of a point at depth D by one pixel
        ctr = info["scene_center"]
        depth = float(np.linalg.norm(np.array(ctr) - np.array([cam0.position.x, cam0.position.y, cam0.position.z])))
        film = float(np.linalg.norm(np.array([frame.C.x - frame.position.x, frame.C.y - frame.position.y,
                                              frame.C.z - frame.position.z])))
        step_units = args.camera_pan * max(depth, 1e-3) / film
        frames = []
        for k in range(1, args.steps + 1):
            cam = rtgpu.Camera()
            ctypes.pointer(cam)[0] = cam0
            sh_ = step_units * k
            cam.position.x = cam0.position.x + fu[0] * sh_
            cam.position.y = cam0.position.y + fu[1] * sh_
            cam.position.z = cam0.position.z + fu[2] * sh_
            fr = rtgpu.Frame()
            rtgpu._check(rtgpu.lib().rt_frame_from_camera(ctypes.byref(cam), ctypes.byref(fr)), "frame")
            frames.append(fr)
        ctx.set_timing(True)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        ctx.frame_check()
        t1 = time.perf_counter()
        for fr in frames:
            step(fr)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el_f = time.perf_counter() - t1
        ftf = ctx.frame_times(min(args.steps, 1024))
        ktf = ctx.kernel_times(min(args.steps, 1024))
        # (an extra measurement: an incomplete frame here -- a new camera whose
        # lists outgrew the estimate from the last frame, rendered again by a
        # caller that checks rt_hip_stats -- voids only these numbers)
        fresh_q, why = frame_checked(ctx, rank, world, frames[-1], args.steps, "fresh-camera", fatal=False)
        ctx.set_timing(False)
        tf = torch.tensor([el_f, sum(a for a, _ in ftf) / len(ftf)] +
                          [sum(k[i] for k in ktf) / len(ktf) for i in range(3)], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(tf, op=dist.ReduceOp.MAX)
        el_f, lists_f, trace_f, shade_f, fold_f = tf.tolist()
        fresh = {"pan_px_per_step": args.camera_pan, "pan_world_units_per_step": round(step_units, 6),
                 "frames": args.steps,
                 "ms_per_step": round(el_f / args.steps * 1e3, 3) if fresh_q is not None else None,
                 "value": round(fresh_q / el_f / 1e6, 3) if fresh_q is not None else None,
                 "candidate_lists_ms": round(lists_f, 3),
                 "kernel_ms": {"trace": round(trace_f, 3), "shade": round(shade_f, 3), "fold": round(fold_f, 3)},
                 "incomplete": why}
    trace_ms = sum(a for a, _, _ in kt) / len(kt)
    shade_ms = sum(b for _, b, _ in kt) / len(kt)
    fold_ms = sum(c for _, _, c in kt) / len(kt)
    lists_ms = sum(a for a, _ in ft) / len(ft)
    if part_ms:  # the render built no lists: the produce / all-to-all / consume wall time instead
        lists_ms = sum(part_ms) / len(part_ms)
    kern_ms = sum(b for _, b in ft) / len(ft)
    tt = torch.tensor([el, kern_ms, lists_ms, trace_ms, shade_ms, fold_ms], dtype=torch.float64,
                      device=dev)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    el, kern_ms, lists_ms, trace_ms, shade_ms, fold_ms = tt.tolist()

    queries = closest + shadow
    cyc = [float(work[k]) for k in ("cycles_camera", "cycles_cand", "cycles_secondary")]
    # instrumented pass: shares of the trace kernel's wave clocks per phase
    phase_share = ({k: round(v / sum(cyc), 4) for k, v in
                    zip(("camera_walk", "camera_candidates", "secondary_walks"), cyc)}
                   if sum(cyc) > 0 else None)
    # the timed frames' own queries (device-counted per frame, every rank)
    if abs(timed_q - queries * args.steps) > 0.5:
        raise SystemExit(f"timed frames made {timed_q:.0f} queries, {queries * args.steps:.0f} expected "
                         "(the same frame every step): no value printed")
    value = timed_q / el / 1e6
    # Algorithmic bytes per launch of each kernel (DESIGN.md §4 "Roofline"),
    # per rank: the records a wave pulls from the memory system (a record
    # several lanes load with one instruction counts once) plus the rays' and
    # hit records' own state.
    kb = {
        # closest-hit queries: ray, wave-distinct node / triangle fetches,
        # the winner's normals, one hit record (2 float4 + prev) per hit,
        # each lane's deepest-record index per item
        "trace": (wcl * RAY_BYTES + nodes * NODE_BYTES + tris * TRI_BYTES +
                  whits * (NORMAL_BYTES + HIT_RECORD_BYTES) + pixels * 4 * 4),
        # per hit record: the record, its material, one term written; per
        # shadow query: the ray and the walk's node (+ multipliers) and
        # triangle fetches
        "shade": (whits * (HIT_RECORD_BYTES + MATERIAL_BYTES + TERM_BYTES) + wsh * RAY_BYTES +
                  sh_wnodes * (NODE_BYTES + NODE_MU_BYTES) + sh_wtris * TRI_BYTES),
        # per pixel: 4 deepest indices, the chain's terms and links, the output
        "fold": pixels * (4 * 4 + PIXEL_BYTES) + whits * (TERM_BYTES + 4),
    }
    kms = {"trace": trace_ms, "shade": shade_ms, "fold": fold_ms}
    dom = max(("trace", "shade"), key=lambda k: kms[k])  # the dominant kernel
    per_launch = kb[dom] / world
    achieved = per_launch / (kms[dom] * 1e-3) / 1e9
    traffic = traffic_hi = None
    traffic_src = None
    if world == 1 and args.traffic_json is None and args.cull_slack is None and \
            args.camera_slack is None and args.policy is None and args.accel is None and \
            args.exact_shadows is None and not args.exact_reflections:
        # default run: the newest committed rocprofv3 PMC passes of this
        # workload (profiles/r*_<workload>/, tools/gpu_profile.sh); a PMC
        # pass cannot run inside the bench, so the line says where it came from
        args.traffic_json = latest_profile(args.workload, "traffic.json")
        if args.valu_json is None:
            args.valu_json = latest_profile(args.workload, "pmc_sq.json")
    kern_pmc = {}
    if args.traffic_json and os.path.exists(args.traffic_json):
        with open(args.traffic_json) as f:
            tj = json.load(f)
        # per-kernel format (tools/pmc_traffic.py): FETCH_SIZE is exact for
        # scattered 64 B requests and half the bytes of wide coalesced reads
        # (MI355X_MICROARCH.md "HBM"): x1 lower bound, x2 upper
        for k in ("trace", "shade", "fold"):
            e = tj.get(k + "_kernel")
            if e and "fetch_size_kib_raw" in e:
                wb = e.get("write_bytes_per_launch", 0.0)
                kern_pmc[k] = {"hbm_bytes": e["fetch_size_kib_raw"] * 1024 + wb,
                               "hbm_bytes_upper": e["fetch_size_kib_raw"] * 2048 + wb}
        if dom in kern_pmc:
            traffic = kern_pmc[dom]["hbm_bytes"]
            traffic_hi = kern_pmc[dom]["hbm_bytes_upper"]
            traffic_src = os.path.relpath(args.traffic_json, REPO)
    sq = {}
    if args.valu_json and os.path.exists(args.valu_json):
        # SQ counters per kernel (tools/pmc_pass.sh, two passes merged by
        # tools/gpu_profile.sh).  SQ_* cycle counters count quad-cycles
        # (MI355X_MICROARCH.md); GRBM_GUI_ACTIVE sums the 8 XCDs' busy clocks.
        with open(args.valu_json) as f:
            pj = json.load(f)
        for k in ("trace", "shade"):
            pm = pj.get(k + "_kernel")
            if not pm or "SQ_WAVE_CYCLES" not in pm:
                continue
            cycles = pm["GRBM_GUI_ACTIVE"] / N_XCD           # shader clocks of the dispatch
            wc = pm["SQ_WAVE_CYCLES"]                           # quad-cycles, summed over waves
            e = {
                # a wave64 VALU instruction holds a 32-lane SIMD for >= 2 clocks
                "valu_pipe_occupancy": round(pm["SQ_INSTS_VALU"] * 2 / (N_SIMD * cycles), 4),
                "valu_lane_util": round(pm["SQ_THREAD_CYCLES_VALU"] / (64.0 * pm["SQ_ACTIVE_INST_VALU"]), 4),
                "valu_insts_per_launch": pm["SQ_INSTS_VALU"],
                "waves_per_simd": round(wc / (N_SIMD * cycles / 4.0), 3),
                "clock_ghz": round(cycles / (kms[k] * 1e-3) / 1e9, 3),
                # where a resident wave's clocks go (disjoint; sums to ~1)
                "stall": {"issuing": round(pm["SQ_ACTIVE_INST_ANY"] / wc, 4),
                          "wait_dependency": round(pm["SQ_WAIT_ANY"] / wc, 4),
                          "wait_issue": round(pm["SQ_WAIT_INST_ANY"] / wc, 4)},
                "valu_active_per_wave": round(pm["SQ_ACTIVE_INST_VALU"] / wc, 4),
            }
            for c in ("SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_SALU"):
                if c in pm:
                    e[c.lower()[3:] + "_per_launch"] = pm[c]
            if "SQ_ACTIVE_INST_LDS" in pm:
                e["lds_active_per_wave"] = round(pm["SQ_ACTIVE_INST_LDS"] / wc, 4)
            sq[k] = e
        sq["source"] = os.path.relpath(args.valu_json, REPO)

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu:
            img = img_timed.view(H, W, 3).cpu().numpy()
            thr = args.cpu_threads or min(len(os.sched_getaffinity(0)) or 1,
                                          int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or 16)
            log(f"[rank 0] cpu baseline: {args.cpu_seconds:.0f}s of samples (Mode A 4 threads, "
                f"Mode B {thr} threads)")
            cpu = cpu_baseline(scene, W, H, args.cpu_seconds, thr, img)
        out = {
            "metric": "Mrays/sec (primary+shadow) at 3840x2160",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3),
            # the same number of frames with a new camera each (--camera-pan):
            # nothing of an earlier identical frame reused
            "ms_per_step_fresh": fresh["ms_per_step"] if fresh else None,
            "fresh_camera": fresh,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic" if wl["kind"] == "synthetic" else f"reference scene {wl['scene']}.svati",
            "config": {
                "workload": wl["desc"],
                "width": W, "height": H, "triangles": ntri, "accel": wl["accel"],
                "accel_build": {"seconds": round(info["build_seconds"], 3),
                                "where": "device" if wl["accel"] == "octree_gpu" else "host",
                                "records": info["tri_refs"], "nodes": info["nodes"],
                                "light_buffer_entries": info["lightbuf_entries"],
                                "light_buffer_global": info["lightbuf_global"],
                                "light_buffer_never": info["lightbuf_never"],
                                "light_buffer_band": info["lightbuf_band"],
                                "light_buffer_seconds": round(info["lightbuf_seconds"], 3),
                                "persistent_grid": {"trace": info["trace_grid"], "shade": info["shade_grid"]}},
                "parallelism": f"image tiles over {world} GPU(s) + RCCL gather" if world > 1
                               else "1 GPU",
                # camera rays: candidate lists; shadow rays: proven light buffers
                # (the library default) or slack-grown ones (--exact-shadows 0)
                "candidate_lists": ("triangle-parallel: rt_hip_cand_produce over 1/N of the "
                                    "triangles, RCCL all-to-all, rt_hip_cand_consume" if partition
                                    else "per rank: every triangle, this rank's tiles"),
                "exactness": {"camera_rays": "proven (candidate lists, refined per tile)",
                              "shadow_rays": ("measured (slack-grown light buffers)"
                                              if args.exact_shadows == 0 else
                                              "proven (light buffers + off-box brute force)"),
                              "reflection_rays": ("proven (error-region growth per node, csrc/rt_reflect.hip)"
                                                  if args.exact_reflections else
                                                  "tested (culling slack; grazing probes, whole-frame checks)")},
                "queries_per_frame": {"closest": int(closest), "shadow": int(shadow),
                                      "closest_hits": int(hits), "pixels": int(pixels)},
            },
            "roofline": {
                # priced against HBM; the dominant kernel of
                # the render (trace: camera + reflection paths; shade: shadow
                # queries + Phong) -- see "kernels" for all three
                "bound": "hbm",
                "kernel": f"{dom}_kernel<{'FLAT' if wl['accel'] == 'flat' else 'OCTREE'}>",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "traffic_upper": traffic_hi,
                "hbm_measured_GBs": (round(traffic / (kms[dom] * 1e-3) / 1e9, 2)
                                     if traffic is not None else None),
                "traffic_source": (f"committed profile {traffic_src} (not measured in this run; "
                                   f"taken of this device code, sha256 {device_code_hash()[:12]})"
                                   if traffic is not None else
                                   f"none: no committed PMC profile of this device code "
                                   f"(sha256 {device_code_hash()[:12]})"),
                "kernel_ms": round(kms[dom], 3),
                "algorithmic_bytes_per_launch": int(per_launch),
                "kernels": {k: {"ms": round(kms[k], 3),
                                "algorithmic_bytes_per_launch": int(kb[k] / world),
                                "achieved_GBs": round(kb[k] / world / (kms[k] * 1e-3) / 1e9, 2),
                                "hbm_bytes_per_launch": (kern_pmc[k]["hbm_bytes"]
                                                         if k in kern_pmc else None),
                                "hbm_measured_GBs": (round(kern_pmc[k]["hbm_bytes"] /
                                                           (kms[k] * 1e-3) / 1e9, 2)
                                                     if k in kern_pmc else None)}
                            for k in ("trace", "shade", "fold")},
                "render_ms": round(kern_ms, 3),
                "candidate_lists_ms": round(lists_ms, 3),
                # wave-distinct record fetches per query (a record several lanes
                # load with one instruction counts once) ...
                "closest_fetches_per_query": {"nodes": round(nodes / wcl, 3) if wcl else None,
                                              "tris": round(tris / wcl, 3) if wcl else None},
                "shadow_fetches_per_query": {"nodes": round(sh_wnodes / wsh, 3) if wsh else None,
                                             "tris": round(sh_wtris / wsh, 3) if wsh else None},
                # ... and the per-lane work behind them (SURVEY.md §8(d) N_node, N_tri)
                "per_lane": {
                    "closest_nodes_per_query": round(cl_nodes / wcl, 3) if wcl else None,
                    "closest_tris_per_query": round(cl_tris / wcl, 3) if wcl else None,
                    "shadow_nodes_per_query": round(sh_nodes / wsh, 3) if wsh else None,
                    "shadow_tris_per_query": round(sh_tris / wsh, 3) if wsh else None,
                    "stack_spill_pushes": int(work["stack_spills"]),
                },
                "candidate_entries": int(cand_entries),
                "shadow_global_prims": info.get("shadow_global"),
                "shadow_mu_max": info.get("shadow_mu_max"),
                # instrumented pass: shares of the trace kernel's wave clocks
                "trace_phase_share": phase_share,
            },
            # SQ counters of the committed PMC passes, per kernel
            "sq": sq or None,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
