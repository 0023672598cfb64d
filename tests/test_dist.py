"""Multi-rank path on CPU (gloo, world_size 2 and 3): each rank produces the
tile buffer the renderer writes for it (4x4-tile blocks, block b -> rank b %
N, csrc/rt_tiles.h), rank 0 gathers them rank-major exactly as bench.py does
with RCCL, and the assemble index map (mirrored from the HIP assemble kernel)
restores the PPM-order image."""
import os
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import REPO, golden_image, load_manifest_static


def _worker(rank, world, store, case, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
    import rtgpu
    # a file rendezvous: no port to race for with other tests on the machine
    dist.init_process_group("gloo", init_method="file://" + store, rank=rank, world_size=world)
    img = golden_image(case)
    mine = torch.from_numpy(rtgpu.tiles_from_image_numpy(img, rank, world).ravel().copy())
    per = mine.numel()
    gathered = torch.empty(per * world) if rank == 0 else None
    dist.gather(mine, list(gathered.view(world, per)) if rank == 0 else None, dst=0)
    if rank == 0:
        out = rtgpu.assemble_tiles_numpy(gathered.numpy(), case["width"], case["height"], world)
        q.put(bool(np.array_equal(out.view(np.uint32), img.view(np.uint32))))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("size", [(96, 54), (192, 108)])
def test_gather_assemble_gloo(world, size, tmp_path):
    case = next(c for c in load_manifest_static()
                if (c["width"], c["height"]) == size and c["scene"] == "island_smooth")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = str(tmp_path / "rendezvous")
    procs = [ctx.Process(target=_worker, args=(r, world, store, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get(timeout=10) is True


def test_tile_ownership_is_a_partition():
    sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
    import rtgpu
    W, H = 3840, 2160
    for n in (1, 2, 4, 8):
        tx, ty = (W + 7) // 8, (H + 7) // 8
        nt = tx * ty
        tpr = -(-nt // n)
        owned = np.zeros(nt, np.int32)
        for r in range(n):
            for local in range(tpr):
                g = local * n + r
                if g < nt:
                    owned[g] += 1
        assert (owned == 1).all()
        assert tpr * n >= nt


@pytest.mark.parametrize("W,H,n", [(96, 54, 2), (96, 54, 3), (192, 108, 8), (3840, 2160, 8),
                                   (3840, 2160, 7), (1920, 1080, 3), (40, 24, 5)])
def test_tile_map_partitions_the_frame(built, W, H, n):
    """Every pixel belongs to exactly one (rank, tile-buffer slot); the host
    mirror's sizes agree with the library's (rt_hip_tiles_per_rank); every
    rank holds close to 1/n of the tiles (whole blocks)."""
    sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
    import rtgpu
    tpr = rtgpu.tiles_per_rank(W, H, n)
    assert tpr == rtgpu.tiles_per_rank_host(W, H, n)
    seen = np.zeros((H, W), np.int32)
    counts = []
    for r in range(n):
        pix = rtgpu.tile_pixels(W, H, r, n)
        assert len(pix) <= tpr
        ok = pix[..., 0] >= 0
        np.add.at(seen, (pix[..., 0][ok], pix[..., 1][ok]), 1)
        counts.append(int(ok.sum()))
        tx, ty = rtgpu.tile_xy(np.arange(len(pix)), r, n, W, H)
        rk, loc = rtgpu.tile_local(tx, ty, n, W, H)
        assert (rk == r).all() and (loc == np.arange(len(pix))).all()
    assert (seen == 1).all()
    # diagonals: per rank, the same count from every n block rows, and within
    # the last partial period at most one block per row more or less
    assert max(counts) - min(counts) <= 32 * 32 * n
    img = np.random.default_rng(1).random((H, W, 3), dtype=np.float32)
    g = np.stack([rtgpu.tiles_from_image_numpy(img, r, n) for r in range(n)])
    assert np.array_equal(rtgpu.assemble_tiles_numpy(g, W, H, n), img)


@pytest.mark.parametrize("W,H,n", [(96, 54, 2), (96, 54, 3), (192, 108, 8), (480, 272, 8),
                                   (3840, 216, 8), (3840, 216, 7), (40, 24, 5)])
def test_tile_map_row_arithmetic(built, W, H, n):
    """The O(1) row counts and run-order emission of csrc/rt_tiles.h (the
    candidate lists' per-row tile counts, emit_interval and kth_rank_col
    follow them) agree with a brute-force walk of every tile row, every rank,
    every column interval up to 40 tiles wide (rt_tile_map_check)."""
    import ctypes as C
    sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
    import rtgpu
    out = (C.c_ulonglong * 2)()
    assert rtgpu.lib().rt_tile_map_check(W, H, n, 40, out) == 0
    assert out[0] > 0 and out[1] == 0, (out[0], out[1])


@pytest.mark.parametrize("W,H", [(3840, 2160), (1920, 1080), (2560, 1440)])
def test_tile_map_balances_rows_and_columns(built, W, H):
    """with block b -> rank b mod n, 4K's 120 blocks per
    row (a multiple of 2, 4, 8) gave every rank the same block columns in every
    row -- column stripes.  On diagonals every rank holds each block column in
    1/n of the block rows and 1/n of each block row (each up to one block), so
    a cost that varies by column or by row alone is split evenly; the library's
    buffer stride is the largest rank's count."""
    sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
    import rtgpu
    for n in (2, 3, 4, 7, 8):
        tb, bx, by = rtgpu._blocks(W, H, n)
        rk, _ = rtgpu._rank_block_grid(W, H, n)
        for c in range(bx):
            share = np.bincount(rk[:, c], minlength=n)
            assert share.max() - share.min() <= 1, (n, c, share)
        for r in range(by):
            share = np.bincount(rk[r, :], minlength=n)
            assert share.max() - share.min() <= 1, (n, r, share)
        per = [rtgpu.rank_tile_count(W, H, r, n) for r in range(n)]
        assert rtgpu.tiles_per_rank(W, H, n) == max(per)
        if (W, H) == (3840, 2160) and n in (2, 4, 8):
            assert min(per) == max(per)  # 120 x 68 blocks: exactly even


def _a2a_worker(rank, world, store, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
    import rtgpu
    dist.init_process_group("gloo", init_method="file://" + store, rank=rank, world_size=world)
    # what every producer r routes to every rank d (csrc/rt_cand.hip pack
    # format: local tile or tpr, prim, skip bits), deterministic per (r, d)
    def block(r, d):
        rng = np.random.default_rng(1000 * r + d)
        n = int(rng.integers(0, 50)) if (r + d) % 3 else 0  # some empty blocks
        return rng.integers(0, 2**31, (n, 3), dtype=np.int64).astype(np.int32)
    blocks = [block(rank, d) for d in range(world)]
    counts = [len(b) for b in blocks]
    send = torch.from_numpy(np.concatenate(blocks + [np.zeros((7, 3), np.int32)]))  # slack rows past the counts
    recv, g = rtgpu.exchange_cand_entries(dist, send, counts, nglobal=rank + 1)
    want = np.concatenate([block(r, rank) for r in range(world)])
    q.put((rank, bool(np.array_equal(recv.numpy(), want)), g == sum(r + 1 for r in range(world))))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_triangle_parallel_list_exchange_gloo(world, tmp_path):
    """rtgpu.exchange_cand_entries (bench.py's all-to-all of the routed list
    entries, rt_hip_cand_produce -> rt_hip_cand_consume) on gloo: every rank
    receives exactly the blocks every producer routed to it, in source-rank
    order (empty blocks included), and the producers' global counts summed."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = str(tmp_path / "rendezvous")
    procs = [ctx.Process(target=_a2a_worker, args=(r, world, store, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(world))
    assert all(ok and gok for _, ok, gok in res), res


@pytest.mark.parametrize("size,n", [((3840, 2160), 8), ((3840, 2160), 4), ((1920, 1080), 3), ((96, 54), 8),
                                    ((640, 360), 2)])
def test_triangle_parallel_route_keys(size, n):
    """The routing of rt_hip_cand_produce (csrc/rt_cand.hip route_kernel,
    mirrored with rtgpu.tile_local): every scanline tile of the one-rank build
    maps to one (rank, local tile) with local < tpr, so the key
    rank * (tpr + 1) + local is unique, below nranks * (tpr + 1), sorts by rank
    first, and never takes the local slot tpr that marks a global triangle;
    each rank receives exactly its own tiles (rt_hip_cand_consume's ntiles)."""
    sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
    import rtgpu
    W, H = size
    tx, ty = (W + 7) // 8, (H + 7) // 8
    t = np.arange(tx * ty)
    rk, loc = rtgpu.tile_local(t % tx, t // tx, n, W, H)
    tpr = rtgpu.tiles_per_rank_host(W, H, n)
    assert (loc < tpr).all() and (rk < n).all()
    key = rk * (tpr + 1) + loc
    assert len(np.unique(key)) == len(key) and key.max() < n * (tpr + 1)
    assert ((key // (tpr + 1)) == rk).all()
    for r in range(n):
        mine = np.sort(loc[rk == r])
        nt = rtgpu.rank_tile_count(W, H, r, n)
        assert len(mine) <= nt and (mine < nt).all()
        # the rank's real tiles are exactly its tile slots that hold a pixel
        px = rtgpu.tile_pixels(W, H, r, n)
        real = np.flatnonzero((px[..., 0] >= 0).any(axis=1)) if len(px) else np.array([], int)
        assert np.array_equal(mine, real)
