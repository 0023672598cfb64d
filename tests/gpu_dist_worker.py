"""One rank of the two-process triangle-parallel list test
(tests/test_gpu.py::test_triangle_parallel_lists_two_processes): both ranks
share GPU 0 (RCCL needs one device per rank, so the exchange runs on gloo
with host tensors -- the same rtgpu.exchange_cand_entries bench.py calls over
RCCL).  Each rank produces its slice of the triangles, exchanges, consumes,
renders its tiles, renders them again with its own per-rank lists, and rank 0
prints one JSON line: every rank's tiles bit-identical and equal counts.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port P tests/gpu_dist_worker.py [frame]

`frame`: the whole frame as bench.py runs it (lists exchanged, tiles rendered,
gathered to rank 0 and assembled there), compared with one rank's render.
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
import rtgpu  # noqa: E402


def render_tiles(ctx, L, f, rank, n):
    per = rtgpu.tile_buffer_floats(f.width, f.height, n)
    d = C.c_void_p()
    assert L.rt_hip_malloc(0, per * 4, C.byref(d)) == 0
    ctx.render(f, rank, n, d.value)
    st = ctx.stats()
    out = np.empty(per, np.float32)
    assert L.rt_hip_memcpy_d2h(out.ctypes.data_as(C.c_void_p), d, out.nbytes) == 0
    L.rt_hip_free(d)
    return out, st


def frame(rank, n, L):
    """The whole N-rank frame as bench.py runs it (triangle-parallel lists,
    render, gather of the tile buffers to rank 0, rt_hip_assemble), the
    exchanges on gloo; rank 0 compares the assembled image with its own
    single-rank render of the frame."""
    s = rtgpu.Scene.synthetic(4, 4, 9776, seed=0x5EED, width=640, height=360)
    f = s.frame()
    ctx = rtgpu.Context(s, "octree_gpu", device=0)
    counts, ng = ctx.cand_produce(f, rank, n)
    ptr, m = ctx.cand_send_buffer()
    send = np.empty((max(m, 1), 3), np.int32)
    if m:
        assert L.rt_hip_memcpy_d2h(send.ctypes.data_as(C.c_void_p), C.c_void_p(ptr), m * 12) == 0
    recv, g = rtgpu.exchange_cand_entries(dist, torch.from_numpy(send), counts, ng)
    recv = np.ascontiguousarray(recv.numpy())
    dr = C.c_void_p()
    assert L.rt_hip_malloc(0, max(recv.nbytes, 16), C.byref(dr)) == 0
    if recv.size:
        assert L.rt_hip_memcpy_h2d(dr, recv.ctypes.data_as(C.c_void_p), recv.nbytes) == 0
    ctx.cand_consume(f, rank, n, dr.value, len(recv), g)
    tiles, st = render_tiles(ctx, L, f, rank, n)
    L.rt_hip_free(dr)
    gathered = [torch.empty(len(tiles)) for _ in range(n)] if rank == 0 else None
    dist.gather(torch.from_numpy(tiles), gathered, dst=0)
    q = torch.tensor([st["closest"], st["shadow"]], dtype=torch.int64)
    dist.reduce(q, dst=0)
    if rank != 0:
        return None
    g_all = np.ascontiguousarray(torch.cat(gathered).numpy())
    dg, drgb = C.c_void_p(), C.c_void_p()
    assert L.rt_hip_malloc(0, g_all.nbytes, C.byref(dg)) == 0
    assert L.rt_hip_malloc(0, f.width * f.height * 12, C.byref(drgb)) == 0
    assert L.rt_hip_memcpy_h2d(dg, g_all.ctypes.data_as(C.c_void_p), g_all.nbytes) == 0
    ctx.assemble(f, dg.value, n, drgb.value)
    ctx.stats()  # waits
    img = np.empty((f.height, f.width, 3), np.float32)
    assert L.rt_hip_memcpy_d2h(img.ctypes.data_as(C.c_void_p), drgb, img.nbytes) == 0
    L.rt_hip_free(dg)
    L.rt_hip_free(drgb)
    ref, st1 = ctx.render_image(f)
    return {"ok": bool(np.array_equal(img.view(np.uint32), ref.view(np.uint32))) and
            [int(x) for x in q.tolist()] == [st1["closest"], st1["shadow"]],
            "queries": [int(x) for x in q.tolist()], "single": [st1["closest"], st1["shadow"]]}


def main():
    dist.init_process_group("gloo")
    rank, n = dist.get_rank(), dist.get_world_size()
    if len(sys.argv) > 1 and sys.argv[1] == "frame":
        res = frame(rank, n, rtgpu.lib())
        if rank == 0:
            print(json.dumps(res), flush=True)
        dist.destroy_process_group()
        return
    L = rtgpu.lib()
    s = rtgpu.Scene.synthetic(4, 4, 9776, seed=0x5EED, width=640, height=360)
    f = s.frame()
    ctx = rtgpu.Context(s, "octree_gpu", device=0)
    counts, ng = ctx.cand_produce(f, rank, n)
    ptr, m = ctx.cand_send_buffer()
    send = np.empty((max(m, 1), 3), np.int32)
    if m:
        assert L.rt_hip_memcpy_d2h(send.ctypes.data_as(C.c_void_p), C.c_void_p(ptr), m * 12) == 0
    recv, g = rtgpu.exchange_cand_entries(dist, torch.from_numpy(send), counts, ng)
    recv = np.ascontiguousarray(recv.numpy())
    dr = C.c_void_p()
    assert L.rt_hip_malloc(0, max(recv.nbytes, 16), C.byref(dr)) == 0
    if recv.size:
        assert L.rt_hip_memcpy_h2d(dr, recv.ctypes.data_as(C.c_void_p), recv.nbytes) == 0
    ctx.cand_consume(f, rank, n, dr.value, len(recv), g)
    t_ext, st_ext = render_tiles(ctx, L, f, rank, n)  # the consumed lists
    L.rt_hip_free(dr)
    t_ref, st_ref = render_tiles(ctx, L, f, rank, n)  # this rank's own lists
    ok = (bool(np.array_equal(t_ext.view(np.uint32), t_ref.view(np.uint32))) and
          st_ext["closest"] == st_ref["closest"] and st_ext["shadow"] == st_ref["shadow"] and
          st_ext["cand_entries"] == st_ref["cand_entries"] and st_ref["cand_entries"] > 0)
    res = [None] * n
    dist.all_gather_object(res, {"rank": rank, "ok": ok, "entries": int(st_ext["cand_entries"]),
                                 "received": int(len(recv)), "globals": int(g)})
    if rank == 0:
        print(json.dumps({"ranks": res, "ok": all(r["ok"] for r in res)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
