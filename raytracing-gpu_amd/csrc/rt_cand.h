// rt_cand.h -- per-frame camera-ray candidate lists (csrc/rt_cand.hip).
//
// Exactness of the octree walk for camera rays: a triangle
// whose float Moller-Trumbore error region (tools/mt_bound.py) fits inside
// the walk's culling slack is found by the walk; every other triangle is
// rasterised, with its whole error region, into the candidate lists of the
// 8x8 tiles whose camera rays could pass through that region, and the render
// kernel tests those candidates exactly after the walk.  Not part of the
// public C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rtc {
struct Footprint;
}

// prims per block of a producer's interleaved slice (CandParams::sl_stride)
#define RT_SLICE_BLOCK 1024u

struct CandParams {
  const float4* tri;      // prim-order triangle records (3 float4 each)
  const float4* node;     // octree nodes (2 float4 each: box + words), may be NULL
  const uint32_t* prim_leaf;  // nprim: a leaf holding a record of the prim (NULL: none)
  uint32_t nprim;
  uint32_t prim0, prim1;  // the prims this build lists: [prim0, prim1) (else [0, nprim)), or
  uint32_t sl_stride, sl_rank;  // with sl_stride > 1, the i-th of prim1 - prim0 prims of
                          // the blocks of RT_SLICE_BLOCK prims b = sl_rank mod sl_stride
                          // (a producer's slice of a triangle-parallel multi-GPU build:
                          // interleaved blocks spread a scene region's cost over the producers)
  double pos[3];          // eye (camera position)
  double u[3], v[3];      // image-plane axes (normalised camera u, v)
  double C[3];            // image-plane origin
  double n[3];            // unit normal of the image plane (u x v)
  double plane;           // (C - pos) . n
  double ginv[3];         // inverse Gram matrix of (u, v): [g0 g1; g1 g2]
  double k0, l0;          // image coordinates of pos - C: ginv (u . (pos - C), v . (pos - C))
  // tile (tx, ty)'s sample rectangle (rt_cand.hip tile_keep): centre (k00 +
  // tx dk, l00 + ty dl), half sides hk, hl; pos - its film centre = p00 - tx du
  // - ty dv (du = dk u, dv = dl v); per axis |u_i| hk + |v_i| hl; the world
  // half diagonal hk |u| + hl |v|
  double tile_k00, tile_l00, tile_dk, tile_dl, tile_hk, tile_hl;
  double tile_p00[3], tile_du[3], tile_dv[3], tile_w[3];
  double tile_hd;
  double gscale;          // a bound of its norm
  double lmax;            // max |o - pos| over the frame's camera origins
  double omax;            // max |o| over them
  double dline;           // max distance of a float camera line from pos
  double dorig;           // float rounding of a camera origin (world units)
  double eps_avail;       // culling slack every camera ray gets, minus the slab test's rounding
  double c_dot, c_a;      // error-bound constants (tools/mt_bound.py C_DOT, C_A)
  double kmin, kmax, lmin, lmax_;  // sample coordinates of the frame
  // sample model: 0 = cpu/rt's (pixel (r, c) samples k in [W/2 - c, W/2 - c
  // + 1/2], l likewise, cpu/raytracer.c:55-58); 1 = gpu/rt's compatibility
  // mode (one ray per pixel of the 3x frame at k = c - W/2, l = r - H/2,
  // gpu/raytracer.cu:97-103; one rank)
  int compat;
  int W, H, tiles_x, tiles_y, rank, nranks, ntiles_local;
  int blocks_x, tb;       // tile blocks per block row, block side (csrc/rt_tiles.h: ranks own whole blocks)
  uint32_t* list;         // nprim: prims the float fast path cannot prove safe (pass 0)
  rtc::Footprint* fp;     // nprim: footprint of list entry j with a big footprint (pass 1, read by
                          // the big passes); of every entry with tiles when store_fp (host check)
  uint4* sfp;             // 2 nprim: a small footprint's rows as column intervals (pass 1 -> emit_kernel;
                          // NULL: emit_kernel reads fp, which store_fp must then keep)
  uint32_t store_fp;
  uint32_t* visits;       // nprim + 1: pass 0 flags, then tile entries of list entry j (pass 1)
  const uint32_t* off;    // nprim + 1: exclusive scan of visits
  uint32_t* keys;         // entries: local tile index (pass 2)
  uint32_t* vals;         // entries: prim
  uint32_t* global;       // nprim: prims whose footprint is unbounded
  uint32_t* ctr;          // [1] global prims, [2] big footprints, [3] list length,
                          // [4] big emission items (item_kernel),
                          // [5] 1 = more than item_cap items (big_kernel emits instead),
                          // [6] the entry total, [7] 1 = an entry past key_cap
  uint32_t* big;          // nprim: list entries with big footprints (rt_cand.hip kSmallRows)
  float* skip;            // nprim: depth-skip bound of each listed prim
  uint32_t* big_lane;     // big_cap x 64: per big footprint, each lane's row-count subtotal
  uint32_t big_cap;       // (big_count_kernel -> big_kernel; beyond it big_kernel recounts)
  uint2* items;           // item_cap: (big footprint, chunk of its entries), big_item_kernel's waves
  uint32_t item_cap;
  uint32_t chunk_shift;   // entries per item = 1 << chunk_shift
  uint32_t* wave_items;   // rt_cand_big_waves() + 1: items of each big_count wave ([last] = 0)
  const uint32_t* wave_base;  // its exclusive scan ([last] = all items)
  // 1: the big footprints' entries are refined per tile (rt_cand.hip
  // tile_keep); an entry it drops is written with key drop_key (= the tile
  // count: it sorts after every tile and bounds_kernel leaves it out)
  uint32_t refine;
  uint32_t drop_key;
  // entries the key / value buffers hold (0: sized to the frame's exact total
  // by a host read-back, no check).  Asynchronous builds size them from the
  // previous frame's total: an entry past key_cap is not written and sets
  // ctr[7] (rt_hip_stats then reports the frame and grows the buffers)
  uint32_t key_cap;
};

// Host mirror for surveys (same classify/raster code): safe / footprint /
// global triangle counts, tile entries of this rank, and a log2 histogram of
// entries per footprint triangle.  Returns -1 when the per-row tile count of
// the device count pass disagrees with the tiles the raster emits.
extern "C" int rt_cand_survey_host(const CandParams* p, const float* tri, const float* node,
                                   const uint32_t* prim_leaf, int threads,
                                   unsigned long long out[88]);
// Host sample of the per-tile refinement's decisions (tests; see rt_cand.hip)
extern "C" size_t rt_cand_refine_sample_host(const CandParams* p, const float* tri, uint32_t stride,
                                             uint32_t* out, size_t cap, size_t* total);
// Host check of one frame's device-built lists (tests; see rt_cand.hip)
extern "C" int rt_cand_verify_host(const CandParams* p, const float* tri, const float* node,
                                   const uint32_t* prim_leaf, const uint32_t* list, uint32_t nlist,
                                   const void* fp_dev, const uint32_t* start, const uint32_t* cand,
                                   uint32_t ntiles, unsigned long long out[7]);
// prim_leaf[prim] = a leaf node holding a record of prim (scene build time)
extern "C" hipError_t rt_cand_prim_leaf(const float4* node, uint32_t nnode, const float4* tri,
                                        uint32_t* prim_leaf, hipStream_t s);

// pass 0 (float fast path flags) -> scan -> scatter (compact list of the
// rest) -> pass 1 (their footprints and tile counts) -> exclusive scan ->
// pass 2 ((tile, prim) pairs at the offsets) -> radix sort by tile ->
// per-tile offsets
extern "C" hipError_t rt_cand_quick(const CandParams* p, hipStream_t s);
extern "C" hipError_t rt_cand_scatter(const CandParams* p, hipStream_t s);
extern "C" hipError_t rt_cand_count(const CandParams* p, hipStream_t s);
extern "C" size_t rt_cand_footprint_bytes(void);
// pass 1b: tile counts of the big footprints (one wave each)
extern "C" hipError_t rt_cand_big_count(const CandParams* p, hipStream_t s);
extern "C" hipError_t rt_cand_emit(const CandParams* p, hipStream_t s);
extern "C" hipError_t rt_cand_big(const CandParams* p, uint32_t nbig, hipStream_t s);
// big emission work items: wave_items (big_count_kernel) -> scan -> wave_base
// -> rt_cand_items writes them; pass 2b, entry-parallel: one wave per
// (big footprint, chunk of its entries) item (used when ctr[5] == 0)
extern "C" uint32_t rt_cand_big_waves(void);
extern "C" hipError_t rt_cand_items(const CandParams* p, hipStream_t s);
extern "C" hipError_t rt_cand_big_items(const CandParams* p, uint32_t nitems, int check, hipStream_t s);
extern "C" hipError_t rt_cand_scan(const uint32_t* in, uint32_t* out, uint32_t n, void* temp,
                                   size_t* temp_bytes, hipStream_t s);
// exclusive scan of in[0 .. n], n = min(*n_dev, nmax) read on the device
// (n_dev NULL: nmax): out[0 .. n], *total = out[n] (total may be NULL);
// bsum: rt_cand_scan_dev_tiles(nmax) words of scratch
extern "C" uint32_t rt_cand_scan_dev_tiles(uint32_t nmax);
extern "C" hipError_t rt_cand_scan_dev(const uint32_t* in, uint32_t* out, uint32_t nmax, const uint32_t* n_dev,
                                       uint32_t* total, uint32_t* bsum, hipStream_t s);
// the fast path's flags (p->visits over the slice) scanned straight into the
// compact list (p->list) and its length (p->ctr[3]): scan_dev + scatter fused
extern "C" hipError_t rt_cand_scan_scatter(const CandParams* p, uint32_t* bsum, hipStream_t s);
extern "C" hipError_t rt_cand_sort(uint32_t* keys_in, uint32_t* keys_out, uint32_t* vals_in,
                                   uint32_t* vals_out, uint32_t n, int begin_bit, int end_bit, void* temp,
                                   size_t* temp_bytes, hipStream_t s);
// out[i] = skip[cand[i]]: the sorted lists' per-entry depth-skip bounds
// keys[i] = key for i in [*total_dev, n) (an asynchronous build's unused tail)
extern "C" hipError_t rt_cand_fill_tail(uint32_t* keys, const uint32_t* total_dev, uint32_t n, uint32_t key,
                                        hipStream_t s);
extern "C" hipError_t rt_cand_entry_skip(const uint32_t* cand, const float* skip, float* out,
                                         uint32_t n, const uint32_t* n_dev, hipStream_t s);
// snap (optional): the build's counters, ctr[0 .. 7] copied to [16 .. 23]
extern "C" hipError_t rt_cand_bounds(const uint32_t* keys, uint32_t n, uint32_t* start,
                                     uint32_t ntiles, uint32_t* snap, hipStream_t s);
// Triangle-parallel multi-GPU lists (rt_hip_cand_produce / rt_hip_cand_consume):
// a whole-frame build (one rank, scanline tiles) of a slice of the prims, its
// entries routed to the N-rank tile map.  route: key = scanline tile ->
// dest_rank << tbits | rank-local tile (tpr = tiles per rank < 2^tbits), and
// drop_key (an entry the refinement dropped) -> nranks << tbits; globals:
// one entry per rank with the local slot tpr.  Then partitioned by rank
// (part_*, below) into 3 words per entry (local tile or tpr, prim, skip
// bits).  unpack (consumer):
// keys = local tile (tpr -> ntiles: the globals sort last), idx = i.
// gather: the sorted entries' prims and skip bounds.
extern "C" hipError_t rt_cand_route_globals(const uint32_t* global, uint32_t nglobal, int nranks, uint32_t tpr,
                                            uint32_t tbits, uint32_t* keys, uint32_t* vals, hipStream_t s);
// Stable partition of n routed keys by rank (rank nranks: dropped), packed
// 3 words per entry in out (the dropped ones not written), start[d] = first
// entry of rank d (start[nranks] = the routed entries; start[nranks + 1 ..
// nranks + 8] = ctr[0 .. 7], for one read-back): part_count ->
// hist[(nranks + 1) x rt_cand_part_waves(n)] -> exclusive scan (off) ->
// part_scatter.  nranks <= 256.
extern "C" uint32_t rt_cand_part_waves(uint32_t n);
// part_count routes the first nroute keys itself (route_kernel's mapping;
// total_dev: an asynchronous build's own entry count, the rest dropped) and
// writes them back; the keys past nroute come routed (the globals)
extern "C" hipError_t rt_cand_part_count(uint32_t* keys, uint32_t n, uint32_t tbits, int nranks, uint32_t* hist,
                                         uint32_t nroute, int tiles_x, int blocks_x, int tb, uint32_t drop_key,
                                         const uint32_t* total_dev, hipStream_t s);
extern "C" hipError_t rt_cand_part_scatter(const uint32_t* keys, const uint32_t* prims, const float* skip,
                                           uint32_t n, uint32_t tbits, int nranks, const uint32_t* off,
                                           uint32_t* start, uint32_t* out, const uint32_t* ctr, hipStream_t s);
// Stable compaction of the entries whose key is not drop_key into
// keys_out / vals_out (at most cap; beyond it *ctr7 = 1; a shorter result's
// tail up to cap written as drop_key; n_dev (optional): only the first
// *n_dev of the n entries are the build's): per-wave counts
// (cnt, rt_cand_part_waves(n) + 1 words) -> exclusive scan (off, off[nw] =
// the kept total) -> scatter.  tmp == NULL: *tmp_bytes = the scan's need.
extern "C" hipError_t rt_cand_compact(const uint32_t* keys, const uint32_t* vals, uint32_t n, const uint32_t* n_dev,
                                      uint32_t drop_key, uint32_t cap, uint32_t* cnt, uint32_t* off, void* tmp,
                                      size_t* tmp_bytes, uint32_t* keys_out, uint32_t* vals_out, uint32_t* ctr7,
                                      hipStream_t s);
extern "C" hipError_t rt_cand_unpack(const uint32_t* in, uint32_t n, uint32_t ntiles, uint32_t tpr, uint32_t* keys,
                                     uint32_t* idx, hipStream_t s);
extern "C" hipError_t rt_cand_gather(const uint32_t* in, const uint32_t* idx, uint32_t n, uint32_t* cand,
                                     float* skip, hipStream_t s);
// longest-first work order of the tiles (heavy candidate lists first):
// perm[position] = tile.  tmp == NULL: *tmp_bytes = the scan's need.
// item_cost / cost_sum / waves (optional): the per-item clocks, their sum
// and the grid of an earlier trace of the same frame: tiles with an item
// longer than a quarter of a wave's balanced share also go first.
extern "C" hipError_t rt_cand_order(const uint32_t* start, uint32_t ntiles, uint32_t total,
                                    uint32_t* flags, uint32_t* pos, uint32_t* perm, const uint32_t* item_cost,
                                    const unsigned long long* cost_sum, uint32_t waves, void* tmp,
                                    size_t* tmp_bytes, hipStream_t s);
