// rt_tiles.h -- how the frame's 8x8-pixel tiles are dealt to ranks, shared
// by the device kernels (render, candidate lists, assemble) and their host
// mirrors (rt_hip.cpp, the host re-derivation of the candidate lists).
//
// Tiles are grouped into blocks of tb x tb tiles, tb = rt_block_side(nranks):
// 4 (32 x 32 pixels) when the frame is split, 1 (plain scanline tile order)
// for one rank.  Block b (scanline order, blocks_x = ceil(tiles_x / tb) per
// row) belongs to rank b mod nranks.  A rank's tile buffer holds its blocks
// in order, each as tb^2 tiles in row-major order (tiles past the frame's
// edge are padding: their pixels are invalid and written as 0).  With whole blocks a
// camera-ray candidate footprint (csrc/rt_cand.hip) of a few tiles touches
// one or two ranks instead of one rank per 8-pixel column (the round-2
// interleave t mod nranks made every rank classify every footprint wider
// than 8 nranks pixels), and every rank still holds 1/nranks of every block
// row, so the per-rank cost stays balanced.
//
// cpu/rt splits the frame into 4 quadrants for its 4 pthreads
// (cpu/raytracer.c:92-127); this is the same idea sized for 8 GPUs x 256 CUs.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define RT_TILES_FN __host__ __device__ inline
#else
#define RT_TILES_FN static inline
#endif

#define RT_TB 4  // block side of a split frame, in tiles

RT_TILES_FN int rt_block_side(int nranks) { return nranks > 1 ? RT_TB : 1; }
RT_TILES_FN int rt_blocks_x(int tiles_x, int tb) { return (tiles_x + tb - 1) / tb; }
RT_TILES_FN int rt_blocks_y(int tiles_y, int tb) { return (tiles_y + tb - 1) / tb; }

// blocks of rank r (b = r, r + n, ... < nblocks)
RT_TILES_FN uint32_t rt_rank_blocks(uint32_t nblocks, uint32_t n, uint32_t r) {
  return nblocks > r ? (nblocks - r + n - 1) / n : 0u;
}

// (tx, ty) of rank-local tile t of rank r
RT_TILES_FN void rt_tile_xy(uint32_t t, uint32_t r, uint32_t n, uint32_t blocks_x, uint32_t tb,
                            int* tx, int* ty) {
  const uint32_t b = (t / (tb * tb)) * n + r, k = t % (tb * tb);
  *tx = (int)((b % blocks_x) * tb + k % tb);
  *ty = (int)((b / blocks_x) * tb + k / tb);
}

// rank and rank-local index of tile (tx, ty)
RT_TILES_FN uint32_t rt_tile_local(int tx, int ty, uint32_t n, uint32_t blocks_x, uint32_t tb,
                                   uint32_t* rank) {
  const uint32_t b = (uint32_t)ty / tb * blocks_x + (uint32_t)tx / tb;
  *rank = b % n;
  return (b / n) * tb * tb + ((uint32_t)ty % tb) * tb + (uint32_t)tx % tb;
}

// Rank r's tiles in tile row ty, columns [x0, x1] (x0 <= x1): the blocks of
// the row whose index is r mod n, each contributing its columns inside the
// interval.  first_bx (out, optional) = the first such block column.
RT_TILES_FN uint32_t rt_rank_row_tiles(int ty, int x0, int x1, uint32_t n, uint32_t r,
                                       uint32_t blocks_x, uint32_t tb, int* first_bx) {
  const uint32_t by = (uint32_t)ty / tb;
  const uint32_t bx0 = (uint32_t)x0 / tb, bx1 = (uint32_t)x1 / tb;
  // block columns bx with (by blocks_x + bx) mod n == r: bx = res + m n
  const uint32_t res = (uint32_t)((r + n - (uint32_t)(((uint64_t)by * blocks_x) % n)) % n);
  const uint32_t f = bx0 <= res ? res : bx0 + (res + n - bx0 % n) % n;  // first match >= bx0
  if (first_bx) *first_bx = (int)f;
  if (f > bx1) return 0;
  const uint32_t m = (bx1 - f) / n + 1;  // matching blocks
  uint32_t c = m * tb;
  if (f == bx0) c -= (uint32_t)x0 - bx0 * tb;                 // cut on the left
  const uint32_t last = f + (m - 1) * n;
  if (last == bx1) c -= bx1 * tb + tb - 1 - (uint32_t)x1;     // cut on the right
  return c;
}
