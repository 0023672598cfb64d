/*
 * rt_hip_test.h -- test, tuning and measurement hooks of librtgpu.so.
 *
 * Not part of the drop-in boundary (rt_hip.h): host-side models and
 * validators of the acceleration structures, device-side re-derivations and
 * probes the parity tests compare against brute force, A/B
 * knobs of the traversal and the candidate lists, and the per-phase timing
 * and instrumented counters bench.py and tools/ read.  Plain pointers and
 * sizes, like rt_hip.h.
 */
#ifndef RT_HIP_TEST_H
#define RT_HIP_TEST_H

#include "rt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif


/* Host-only: build the acceleration structure rt_hip_create would build and
 * report its sizes (no device needed). */
int rt_accel_build_info(const rt_scene *scene, int accel, rt_accel_info *out);
/* Host-only: build it and check its invariants (every triangle referenced by
 * a leaf, every leaf box contains its triangles, every node box contains its
 * children).  0 = valid, RT_EINVAL = violated (rt_last_error says where). */
int rt_accel_validate(const rt_scene *scene, int accel);

/* Host-only traversal model of the device octree walk (tuning / checking):
 * camera-ray closest-hit queries of every sample_stride-th pixel; with check,
 * each winner is compared with brute force over all triangles. */
typedef struct rt_accel_probe_result {
  unsigned long long queries, hits, node_visits, tri_tests, max_stack, mismatches;
  /* shadow rays of the camera hits (one per non-ambient light, any-hit) */
  unsigned long long shadow_queries, shadow_hits, shadow_node_visits, shadow_tri_tests;
} rt_accel_probe_result;
int rt_accel_probe(const rt_scene *scene, int accel, int sample_stride, int check,
                   rt_accel_probe_result *out);
/* Downloads the context's scene image and checks the invariants of
 * rt_accel_validate on it (any accel, including device-built octrees). */
int rt_hip_accel_validate(const rt_hip_ctx *ctx);
/* Host-only self-check of the tile map's O(1) row arithmetic (the candidate
 * lists' counts and emission order) against a brute-force walk over the
 * frame's tiles: every tile row, column intervals [x0, x1] of every width
 * up to `maxw` tiles.  out[0] = intervals checked, out[1] = mismatches. */
int rt_tile_map_check(int width, int height, int nranks, int maxw, unsigned long long out[2]);
/* The same conditions checked on the device at the end of every render (no
 * host wait), sticky until read: *flags = their OR since the last call (0 =
 * every frame complete and exact; bits RT_FRAME_* of csrc/rt_kernels.h: 1
 * hit-record overflow, 2 depth, 4 zero normal, 8 undecided exact shadow
 * queries, 16 an asynchronous list build's overflow), *frames = renders
 * checked, queries[0] / [1] = their closest-hit / shadow queries; all reset.
 * For callers that render many frames between rt_hip_stats calls. */
int rt_hip_frame_check(rt_hip_ctx *ctx, unsigned *flags, unsigned *frames, unsigned long long queries[2]);
/* Octree culling slack, in units of 2^-24 x (ray-origin-to-scene distance):
 * boxes are grown by that much so a triangle the reference's float
 * Moller-Trumbore test accepts is never culled (DESIGN.md "Conservative
 * culling").  Default RT_EPS_ULPS_DEFAULT (64).  Tuning knob: below the
 * default rt_hip_stats returns RT_EINEXACT (reflection rays rely on it). */
int rt_hip_set_cull_slack(rt_hip_ctx *ctx, float ulps);
/* The same slack for camera rays only (bounce depth 0; rt_hip_set_cull_slack
 * sets both).  A wider camera slack costs a few more node visits and lets
 * the walk find triangles the per-frame candidate lists would otherwise have
 * to carry; exactness holds for every value. */
int rt_hip_set_camera_slack(rt_hip_ctx *ctx, float ulps);
/* Phase timing: with enable, every rt_hip_render records HIP events on its
 * stream before the camera candidate lists, before and after each of its
 * three kernels (a ring of the last 1024 frames; enabling clears it).
 * rt_hip_frame_times waits for the last n timed frames and returns their two
 * spans in milliseconds, oldest first (lists_ms ~0 without lists). */
int rt_hip_set_timing(rt_hip_ctx *ctx, int enable);
int rt_hip_frame_times(rt_hip_ctx *ctx, int n, float *lists_ms, float *render_ms);
/* The render span of the same frames split by kernel: trace (closest-hit
 * paths -> hit records), shade (shadow queries + Phong terms per record),
 * fold (terms -> tile buffer). */
int rt_hip_frame_kernel_times(rt_hip_ctx *ctx, int n, float *trace_ms, float *shade_ms,
                              float *fold_ms);
/* Instrumented build: also count node visits and triangle tests (slower). */
int rt_hip_set_count_work(rt_hip_ctx *ctx, int enable);
/* Shader clocks of every work item -- (tile t, sample s) at index 4t + s,
 * rank-local tile order -- of the last instrumented render (n <= 4 x tiles
 * of the rank): the load-balance picture of a frame. */
int rt_hip_tile_cycles(rt_hip_ctx *ctx, unsigned long long *out, size_t n);
/* The same items' phase clocks (trace kernel): phase 0 = the item's total
 * (= rt_hip_tile_cycles), 1 camera walk, 2 camera candidate tests, 3
 * secondary walks; 4 and 5 are counts, not clocks: the most node visits and
 * triangle tests one lane of the item made in per-lane secondary walks.
 * Shadow queries run in the shade kernel, per hit record. */
int rt_hip_tile_phase_cycles(rt_hip_ctx *ctx, int phase, unsigned long long *out, size_t n);
/* Exact camera rays (default 1): per-frame candidate lists of the triangles
 * whose float Moller-Trumbore error region the octree slack does not cover
 * (csrc/rt_cand.hip).  0 = octree walk only (A/B timing; rt_hip_stats then
 * returns RT_EINEXACT: cpu/rt parity is not guaranteed for grazing camera rays). */
int rt_hip_set_exact_camera(rt_hip_ctx *ctx, int enable);
/* Light buffers for the shadow queries of the default walk (1, the default):
 * per directional / point light a grid over the light's view whose cells list
 * the triangles a shadow ray starting there can meet (csrc/rt_lightbuf.hip),
 * built once per scene and slack; 0: every shadow query walks the octree.
 * Both are exact in the same sense (DESIGN.md §2 "Shadow rays"). */
int rt_hip_set_light_buffers(rt_hip_ctx *ctx, int enable);
/* Test hook: a light buffer of more than cap entries fails its build (0 = no
 * cap), exercising the fallback (that light's queries walk the octree,
 * rt_accel_info.lightbuf_failed); rebuilds the buffers now. */
int rt_hip_set_lightbuf_entry_cap(rt_hip_ctx *ctx, unsigned long long cap);
/* Host-only survey (no device) of light `light`'s buffer as rt_hip_create
 * builds it for this scene (exact = proven footprints), every stride-th
 * triangle: out[0] entries, [1] triangles never accepted, [2] global, [3] band
 * triangles, [4] big footprints, [5] triangles surveyed, [6] band-row entries,
 * [7] largest per-triangle count, [8] its triangle (prim order), [9] entries of
 * triangles with more than 1024, [10] with 65..1024, [11] triangles with more than 64. */
int rt_lightbuf_survey(const rt_scene *scene, unsigned light, int exact, unsigned stride,
                       unsigned long long out[12]);
/* Shadow-query probe (tests, tools): light `light`'s shadow ray
 * (cpu/light.c:53,78) from each of n origins (x, y, z floats), answered
 * through the context's light buffer (brute = 0) or by brute force over every
 * triangle (brute = 1, cpu/hit.c:93-109); hit[i] = 1 when shadowed. */
int rt_hip_probe_shadows(rt_hip_ctx *ctx, unsigned light, const float *origins, size_t n, int brute,
                         unsigned char *hit);
/* Closest-hit probe (tests, tools): n rays (origins[3 i..], dirs[3 i..],
 * floats) queried as reflection rays are -- the per-lane octree walk at the
 * secondary rays' culling slack (brute = 0; octree contexts) -- or by brute
 * force over every triangle (brute = 1, cpu/hit.c:72-91).  prim[i] = the
 * winner (object-major LIFO index, ~0 = no hit), dist[i] = its new_dist. */
int rt_hip_probe_closest(rt_hip_ctx *ctx, const float *origins, const float *dirs, size_t n, int brute,
                         unsigned *prim, float *dist);
/* Octree traversal policy (default 0): 0 = staged packet walk for camera
 * rays (>= 8 querying lanes), per-lane walks otherwise; 1 = every query per lane;
 * 2 = every query as a staged packet; 3 = 0 plus staged packet walks for
 * directional-light shadow rays.  All are exact; 1-3 exist for tests and A/B
 * measurements (each is its own kernel, so the default has no switch). */
int rt_hip_set_policy(rt_hip_ctx *ctx, int policy);
/* Scale of the error-bound constants the candidate lists use (1 = the
 * proven bound of tools/mt_bound.py; smaller = a calibrated model, faster,
 * exactness then verified rather than proven: rt_hip_stats returns RT_EINEXACT). */
int rt_hip_set_camera_bound_scale(rt_hip_ctx *ctx, double scale);
/* Per-tile refinement of the candidate lists (default 1): the entries of a
 * triangle whose footprint spans more than 2 tile rows or 32 tiles are kept
 * only where the error bound evaluated for that tile's own rays (their
 * directions, origins and grazing cosine) still reaches the tile
 * (csrc/rt_cand.hip tile_keep) -- proven like the per-triangle bound, so the
 * lists stay exact.  0: the per-triangle footprints alone (A/B timing). */
int rt_hip_set_camera_refine(rt_hip_ctx *ctx, int enable);
/* Host-only survey of the camera candidate lists of a scene's frame (no
 * device): out = {safe, footprint, global} triangle counts, tile entries,
 * then 16 log2 buckets of triangles by entries and 16 of their entries,
 * then 16 log2 buckets of footprint triangles by how far their error region
 * (grown by its distance error) reaches beyond the triangle, in units of the
 * walk's slack, and 16 of their entries; out[68] the entries with the per-tile
 * refinement (rt_hip_set_camera_refine), [69] / [70] the refined footprints'
 * entries before / after it; [71..77] the float fast path's verdicts: listed,
 * of those f64-safe through a leaf box, f64-safe otherwise, footprints with
 * no tile, global; proven safe, away (off the frame); [78] / [79] the listed
 * ones f64-safe because their error region stays within the slack / no line
 * is steep enough to be accepted; [80] fast-path verdicts "safe" the f64
 * classification does not confirm (must be 0); use_leaves: also accept
 * triangles whose error region fits a leaf box of the host-built octree. */
int rt_cand_survey(const rt_scene *scene, float eps_ulps, double bound_scale, int threads,
                   int use_leaves, unsigned long long out[88]);

/* Host-only sample of the per-tile refinement (rt_hip_set_camera_refine) of
 * a scene's frame: every stride-th entry of the refined footprints as (prim,
 * tile x, tile y, kept) -- tests check each dropped entry against the
 * reference's float test on every camera sample of its tile.  compat: the
 * gpu/rt compatibility mode's frame (3x the camera, one ray per pixel).
 * *n = entries written (at most cap), *total = entries sampled. */
int rt_cand_refine_sample(const rt_scene *scene, float eps_ulps, double bound_scale, unsigned stride,
                          int compat, unsigned *out, size_t cap, size_t *n, size_t *total);
/* Test hook: after an rt_hip_render of (frame, rank, nranks) with exact
 * camera rays, re-derive its candidate lists on the host from the same code
 * and compare.  out = {listed prims, entries, footprint mismatches, tiles
 * whose list differs, prims on the global list, fast-path filter violations
 * (a prim not listed whose footprint reaches this rank), prims the fast
 * path's rank/frame filter dropped}. */
int rt_hip_cand_verify(rt_hip_ctx *ctx, const rt_frame *frame, int rank, int nranks,
                       unsigned long long out[7]);

/* The same after an rt_hip_render_compat of `camera` (its 3x frame's lists,
 * one sample per high-resolution pixel). */
int rt_hip_cand_verify_compat(rt_hip_ctx *ctx, const rt_camera *camera, unsigned long long out[7]);

/* Test hook: after an rt_hip_render, shade every stride-th hit record of
 * each region again through the context's walk and by brute force over every
 * triangle (cpu/hit.c:93-109), and compare each record's shadow outcome per
 * light.  out = {records compared, shadow queries compared, records whose
 * outcomes differ, queries the walk found lit and brute force shadowed}.
 * The render's image and stats are untouched. */
int rt_hip_verify_shadows(rt_hip_ctx *ctx, unsigned stride, unsigned long long out[4]);
/* The same from the first-th record of each region on (first < stride: the
 * calls for first = 0 .. stride-1 cover every record once). */
int rt_hip_verify_shadows_from(rt_hip_ctx *ctx, unsigned stride, unsigned first, unsigned long long out[4]);

/* Diagnostic: candidate-list entries of each of the first n rank-local tiles
 * of the last render (n <= that rank's tile count). */
int rt_hip_cand_tile_entries(rt_hip_ctx *ctx, unsigned int *out, size_t n);

/* Test hook: at most cap work items for the entry-parallel emission of the
 * big candidate footprints (default 2^20); a frame needing more emits them
 * one wave per footprint instead (the same lists). */
int rt_hip_set_cand_item_cap(rt_hip_ctx *ctx, unsigned cap);

#ifdef __cplusplus
}
#endif
#endif
