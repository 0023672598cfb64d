/*
 * rt_hip.h -- C ABI of the MI355X (gfx950) render path.
 *
 * Plain pointers and sizes only.  This is the drop-in boundary for the
 * reference's hot path:
 *
 *   rt_raytrace()        replaces  void raytrace(const char *input, const char *output)
 *                                  (/root/reference/cpu/headers/raytracer.h:4,
 *                                   cpu/raytracer.c:79-136)
 *   rt_hip_create()      replaces  struct scene *to_cuda(const struct scene *)
 *                                  (/root/reference/gpu/headers/scene.h:52, gpu/scene.cu:224-352)
 *                                  + create_octree() (gpu/partitioning/octree.h:39, octree.cu:362-411)
 *   rt_hip_render()      replaces  render(...) (gpu/headers/raytracer.h:6, gpu/raytracer.cu:177-253)
 *                                  with cpu/rt semantics: 2x2 SSAA in cpu order, float
 *                                  channels, unbounded-by-design reflection recursion
 *                                  (cpu/raytracer.c:19-77), collide/collide_dist/apply_light
 *                                  (cpu/hit.c:72-109, cpu/light.c:33-100) on the device
 *   rt_hip_assemble()    (new)     tile buffers of all ranks -> PPM-order float image
 *   rt_raytrace_multi()  (new)     in-process 1..8 GPU render + RCCL gather over xGMI
 *
 * Threading: calls on distinct contexts may run concurrently on distinct host
 * threads; one context is not re-entrant.  rt_hip_render is asynchronous on
 * the given stream (NULL = the context's own stream); rt_hip_stats and
 * rt_hip_render_image synchronise.
 */
#ifndef RT_HIP_H
#define RT_HIP_H

#include "rt_scene.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Camera frame, cpu/raytracer.c:82-86: u = norm(cam.u), v = norm(cam.v),
 * C = pos + (u x v) * L with L = (float)(W / (2 tan(fov*pi/360))). */
typedef struct rt_frame {
  rt_vec3 u, v, C, position;
  int width, height;
} rt_frame;

/* Fails with RT_EINVAL for odd widths or heights: cpu/rt's output is
 * undefined there (cpu/raytracer.c:89-91,128-134 index the framebuffer two
 * different ways that agree only for even sizes). */
int rt_frame_from_camera(const rt_camera *cam, rt_frame *out);

/* Acceleration structure selection.  OCTREE: SAH octree built on the host
 * (host/accel.c); OCTREE_GPU: octree built on the device by rt_hip_create
 * (csrc/rt_build.hip, Morton keys + radix sort).  Both
 * render the same image; they differ in build time and traversal cost. */
enum { RT_ACCEL_FLAT = 0, RT_ACCEL_OCTREE = 1, RT_ACCEL_OCTREE_GPU = 2 };

/* Per-render counters.  closest = closest-hit queries
 * (collide() calls: camera + reflection rays), shadow = shadow queries
 * (collide_dist() calls), camera = 4*pixels rendered.  node_visits and
 * tri_tests (closest-hit queries) and shadow_node_visits / shadow_tri_tests
 * are only filled by the instrumented kernels (rt_hip_set_count_work) and
 * give the algorithmic bytes of the roofline. */
typedef struct rt_stats {
  unsigned long long closest, shadow, camera;
  unsigned long long node_visits, tri_tests;
  unsigned long long depth_overflow;   /* paths past RT_MAX_BOUNCES or a stack overflow (must be 0) */
  unsigned long long zero_normal;      /* winners with an exactly-zero interpolated normal */
  unsigned long long pixels;
  unsigned long long hits;             /* closest-hit queries that hit geometry */
  /* camera-ray exactness: triangles whose float test the
   * octree slack cannot guarantee, their tile-list entries (each tested by
   * the 64 pixels x 4 samples of the tile), and those every camera ray tests */
  unsigned long long cand_prims, cand_entries, cand_global;
  /* per-lane work of the instrumented pass (rt_hip_set_count_work): node
   * visits and triangle tests summed over the lanes that made them (a record
   * tested by k lanes of a wave counts k times; node_visits / tri_tests count
   * it once), for closest-hit and for shadow queries */
  unsigned long long closest_node_lanes, closest_tri_lanes;
  unsigned long long shadow_node_lanes, shadow_tri_lanes;
  /* instrumented pass: shader clocks the waves spent in the camera-ray walk,
   * the camera candidate tests, the secondary closest-hit walks and the
   * shadow queries (summed over waves) */
  unsigned long long cycles_camera, cycles_cand, cycles_secondary, cycles_shadow;
  unsigned long long cycles_shadow_directional;  /* the directional-light share of cycles_shadow */
  unsigned long long stack_spills;  /* per-lane stack pushes beyond the LDS entries (instrumented pass) */
  unsigned long long shadow_zero_risk;  /* shadow rays whose first hit lies on an object that can
                                         * interpolate a zero normal (must be 0, RT_EZERONORMAL) */
  unsigned long long hit_records;   /* closest hits recorded for shading (trace -> shade) */
  /* instrumented pass: wave-distinct node / triangle record fetches of the
   * shadow queries (shade kernel); node_visits / tri_tests are then those of
   * the closest-hit queries (trace kernel) */
  unsigned long long shadow_node_visits, shadow_tri_tests;
  /* point-light shadow rays whose origin lies beyond the extent the exact
   * shadow walk assumes (csrc/rt_shadow.hip; must be 0, RT_EINEXACT) */
  unsigned long long shadow_unproven;
  /* exact-shadow mode: shadow queries from origins off the proof box (float
   * garbage hits far past a triangle), decided by brute force after the
   * shade pass (rt_hip_set_exact_shadows) */
  unsigned long long shadow_deferred;
  /* exact reflection rays (rt_hip_set_exact_reflections): queries outside the
   * proven walk's assumption |d| <= RT_RF_DLMAX (must be 0, RT_EINEXACT) */
  unsigned long long closest_unproven;
} rt_stats;

/* Sizes of the device-side scene image, for the roofline accounting. */
typedef struct rt_accel_info {
  unsigned long long triangles;        /* scene triangles                        */
  unsigned long long tri_refs;         /* triangle records in traversal order    */
  unsigned long long nodes;            /* octree nodes (0 for FLAT)              */
  unsigned long long leaves;
  unsigned long long max_depth;
  unsigned long long tri_record_bytes; /* bytes per triangle record             */
  unsigned long long node_record_bytes;
  unsigned long long device_bytes;     /* total device memory of the scene image */
  double build_seconds;                /* build time (flatten + octree, host or device) */
  unsigned long long max_leaf;         /* largest leaf (triangle records)        */
  /* exact shadow rays (octree, csrc/rt_shadow.hip): triangles every
   * unshadowed shadow ray tests outside the walk, and the largest per-node
   * multiplier of the shadow walk's culling slack */
  unsigned long long shadow_global;
  double shadow_mu_max;
  /* light buffers of the default shadow queries (csrc/rt_lightbuf.hip):
   * cell entries over all lights, and triangles every query of their light
   * tests (footprint unbounded) */
  unsigned long long lightbuf_entries;
  unsigned long long lightbuf_global;
  double lightbuf_seconds;             /* their build time (device, at rt_hip_create) */
  /* proven light buffers (rt_hip_set_exact_shadows): triangles no shadow ray
   * of a light can make the float test accept (listed nowhere), and
   * triangles listed along a band of a point light's cube map */
  unsigned long long lightbuf_never;
  unsigned long long lightbuf_band;
  /* lights whose buffer could not be built (too many entries or cells, out
   * of device memory, a directional light with a zero vector): their shadow
   * queries walk the octree instead (the proven walk in the exact-shadow
   * mode).  Any other build failure fails the call (RT_EHIP). */
  unsigned long long lightbuf_failed;
  char lightbuf_fail_reason[96]; /* the last such fallback's cause ("" if none) */
  int trace_grid, shade_grid;    /* persistent one-wave workgroups of the default
                                    trace / shade kernels (occupancy-derived) */
  float scene_center[3], scene_radius;  /* the scene's box centre and half-extent (max-norm) */
} rt_accel_info;

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

typedef struct rt_hip_ctx rt_hip_ctx;

int rt_hip_device_count(int *n);

/* Deep-copies the scene into device memory of `device` (flattened SoA
 * triangle records, pre-normalised vertex normals, materials, lights) and
 * builds the acceleration structure.  The caller keeps ownership of scene. */
int rt_hip_create(int device, const rt_scene *scene, int accel, rt_hip_ctx **out);
int rt_hip_accel_info(const rt_hip_ctx *ctx, rt_accel_info *out);
/* Downloads the context's scene image and checks the invariants of
 * rt_accel_validate on it (any accel, including device-built octrees). */
int rt_hip_accel_validate(const rt_hip_ctx *ctx);
void rt_hip_destroy(rt_hip_ctx *ctx);

/* Image tiling (csrc/rt_tiles.h): 8x8-pixel tiles grouped in blocks of tb x
 * tb tiles, tb = 4 (32x32 pixels) when nranks > 1 and 1 (scanline tile order)
 * for one rank; blocks b (scanline order over ceil(tiles_x/tb) x
 * ceil(tiles_y/tb) blocks) come in runs of nranks, run g = b / nranks holding
 * one block of every rank: block b belongs to rank (b % nranks + g) % nranks
 * as that rank's g-th block.  A rank's tile buffer holds its blocks in order,
 * tb*tb tiles each in row-major order, each tile 64 pixels x 3 floats (pixel
 * p of a tile = row p/8, col p%8 inside the tile); slots past the frame's
 * edge are padding (0).  rt_hip_tiles_per_rank() = the largest rank's tile
 * count, the size of every rank's buffer in a gather. */
int rt_hip_tiles_per_rank(int width, int height, int nranks);
size_t rt_hip_tile_buffer_floats(int width, int height, int nranks);
/* Host-only self-check of the tile map's O(1) row arithmetic (the candidate
 * lists' counts and emission order) against a brute-force walk over the
 * frame's tiles: every tile row, column intervals [x0, x1] of every width
 * up to `maxw` tiles.  out[0] = intervals checked, out[1] = mismatches. */
int rt_tile_map_check(int width, int height, int nranks, int maxw, unsigned long long out[2]);

/* Renders every tile of `rank` into d_tiles (device memory of the context's
 * device, rt_hip_tile_buffer_floats() floats).  Asynchronous on `stream`
 * (a hipStream_t; NULL = the context's stream). */
int rt_hip_render(rt_hip_ctx *ctx, const rt_frame *frame, int rank, int nranks, float *d_tiles,
                  void *stream);
/* Waits for the last render and returns its counters.  The counters are
 * filled in whatever the return code: RT_EHITBUF (render again),
 * RT_EDEPTH / RT_EZERONORMAL (the image may differ from cpu/rt's there),
 * RT_EINEXACT (a parity-breaking tuning knob below was active, or a
 * point-light shadow ray left from beyond the proven extent). */
int rt_hip_stats(rt_hip_ctx *ctx, rt_stats *out);
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
/* Shader clocks of every work item -- (tile t, sample s) at index 4t + s,
 * rank-local tile order -- of the last instrumented render (n <= 4 x tiles
 * of the rank): the load-balance picture of a frame. */
int rt_hip_tile_cycles(rt_hip_ctx *ctx, unsigned long long *out, size_t n);
int rt_hip_set_count_work(rt_hip_ctx *ctx, int enable);
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
/* Shadow rays exact by proof (default 1; rt_hip_set_exact_shadows rebuilds
 * the buffers now).  Each light buffer lists a triangle in every cell from
 * which some shadow ray can make the float Moller-Trumbore test accept it
 * (proven footprints, csrc/rt_lightbuf.hip); a query whose origin lies off the
 * proof's box (a float garbage hit far past a triangle) is deferred and
 * decided by brute force over every record after the shade pass (lights
 * 0..31; with more lights it is counted -> RT_EINEXACT).  Queries that walk
 * the octree (staged policies, light buffers off, a failed buffer, the
 * compatibility mode) use the proven walk: each node's box grown by a
 * per-node multiple of the culling slack covering every triangle below it,
 * plus a global list (csrc/rt_shadow.hip).  0: slack-grown
 * buffers and the plain-slack walk, whose decisions are measured against
 * brute force (rt_hip_verify_shadows), not proven; ~0.26 ms faster on C5. */
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
int rt_hip_set_exact_shadows(rt_hip_ctx *ctx, int enable);
/* Reflection rays exact by proof (default 0; builds the per-node bounds now).
 * The reflection walk grows each node's box by the reach of the reference
 * float Moller-Trumbore test's error region for that ray -- bounded through
 * the node's normal cone (the ray's cosine with every plane below it) and the
 * 1e-7f accept threshold -- and prunes with the matching distance error, so
 * every triangle the float test could accept is tested (csrc/rt_reflect.hip,
 * DESIGN.md §2).  0: the culling slack, whose reflection decisions are
 * tested (rt_hip_probe_closest), not proven.  Default traversal policy only
 * (rt_hip_render fails with RT_EINVAL otherwise); the closest-hit probe uses
 * the same walk. */
int rt_hip_set_exact_reflections(rt_hip_ctx *ctx, int enable);
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

/* Triangle-parallel camera candidate lists of an nranks-way frame (new; the
 * per-rank build of rt_hip_render runs the float fast path, classification
 * and emission over every triangle on every rank).  Each rank:
 *   1. rt_hip_cand_produce: the whole frame's list entries of triangles
 *      [rank P / nranks, (rank + 1) P / nranks), routed to the ranks that own
 *      their tiles; counts[d] = entries for rank d (global triangles included,
 *      one entry per rank each), *nglobal = this slice's global triangles.
 *      Synchronises its stream (the entry total).
 *   2. rt_hip_cand_send_buffer: the routed entries (device memory of the
 *      context, 3 x 32-bit words each, destination-rank order: counts[0]
 *      entries for rank 0, then rank 1's, ...), valid until the next produce.
 *   3. an all-to-all of those blocks (e.g. RCCL / torch.distributed
 *      all_to_all_single), every rank receiving its blocks from every rank,
 *      and the sum of the producers' *nglobal;
 *   4. rt_hip_cand_consume: this rank's lists from the n received entries
 *      (any source order); the next rt_hip_render of the same frame, rank and
 *      nranks uses them instead of building its own (once).
 * The lists equal the per-rank build's, tile by tile, as multisets (the
 * render is order-independent: the lexicographic (new_dist, prim) key).
 * Octree contexts with exact camera rays only (else RT_EINVAL).  stream:
 * as rt_hip_render. */
int rt_hip_cand_produce(rt_hip_ctx *ctx, const rt_frame *frame, int rank, int nranks, unsigned *counts,
                        unsigned *nglobal, void *stream);
int rt_hip_cand_send_buffer(const rt_hip_ctx *ctx, const void **d_entries, size_t *n);
int rt_hip_cand_consume(rt_hip_ctx *ctx, const rt_frame *frame, int rank, int nranks, const void *d_entries,
                        size_t n, unsigned nglobal, void *stream);
/* Steps 1-4 for n contexts of this process at once (ctx[r] = rank r, any
 * devices, e.g. all on one GPU): produce on every rank, the blocks moved by
 * device memcpys, consume on every rank; synchronous.  rt_raytrace_multi
 * makes the same exchange over RCCL (grouped ncclSend / ncclRecv) from 4
 * GPUs up. */
int rt_hip_cand_exchange_local(rt_hip_ctx **ctx, int n, const rt_frame *frame);

/* d_gathered = nranks consecutive tile buffers (rank-major, as an RCCL gather
 * delivers them); writes the PPM-order image (W*H*3 floats) to d_rgb. */
int rt_hip_assemble(rt_hip_ctx *ctx, const rt_frame *frame, const float *d_gathered, int nranks,
                    float *d_rgb, void *stream);

/* Convenience: single-GPU render of the whole frame into host memory
 * h_rgb (W*H*3 floats, PPM order); synchronous. */
int rt_hip_render_image(rt_hip_ctx *ctx, const rt_frame *frame, float *h_rgb, rt_stats *stats);

/* Device memory helpers so C callers need no HIP headers. */
/* gpu/rt compatibility mode (gpu/raytracer.cu:31-129,
 * gpu/light.cu, gpu/colors.cu): the camera's frame rendered at 3x width and
 * height with one ray per high-resolution pixel, uint8 saturating colours,
 * reflections summed front to back over at most 11 closest-hit queries, then
 * a 3x3 box downscale.  h_rgba receives width x height RGBA8 pixels (alpha
 * 255) in gpu/rt's PNG row order.  stats as rt_hip_stats (camera = pixels =
 * high-resolution rays).  Camera rays keep the exactness of cpu mode: the
 * per-frame candidate lists of the 3x frame's one-ray-per-pixel camera
 * (csrc/rt_cand.hip, CandParams::compat). */
int rt_hip_render_compat(rt_hip_ctx *ctx, const rt_camera *cam, unsigned char *h_rgba,
                         rt_stats *stats);
/* Drop-in for gpu/rt's main (gpu/rt.cpp:56-97): load, render in
 * compatibility mode on GPU 0, write an 8-bit RGBA PNG.  accel < 0: choose. */
int rt_raytrace_gpu(const char *input, const char *output, int accel);

int rt_hip_malloc(int device, size_t bytes, void **d_ptr);
int rt_hip_free(void *d_ptr);
int rt_hip_memcpy_d2h(void *h_dst, const void *d_src, size_t bytes);
int rt_hip_memcpy_h2d(void *d_dst, const void *h_src, size_t bytes);
/* device -> device, asynchronous on stream (NULL: the null stream) */
int rt_hip_memcpy_d2d(void *d_dst, const void *d_src, size_t bytes, void *stream);

/* Drop-in for raytrace() (cpu/raytracer.c:79-136): parse, render on GPU 0,
 * write the P3 PPM.  Returns an RT_E* code instead of exiting. */
int rt_raytrace(const char *input, const char *output);

/* Same with the frame tiled over `ngpus` devices of this node and gathered
 * to device 0 with one RCCL gather over xGMI.  accel = RT_ACCEL_*.
 * stats (optional) receives the summed counters; render_ms the wall time of
 * render + gather. */
int rt_raytrace_multi(const char *input, const char *output, int ngpus, int accel,
                      rt_stats *stats, double *render_ms);

/* rt_raytrace_multi with rank g on device devices[g].  Distinct devices: as
 * rt_raytrace_multi (RCCL).  A device shared by several ranks (tests running
 * N ranks on one GPU): the same frame with device memcpys in place of the
 * RCCL calls (the candidate lists' exchange from 4 ranks up, the gather). */
int rt_raytrace_multi_dev(const char *input, const char *output, int ngpus, const int *devices, int accel,
                          rt_stats *stats, double *render_ms);

#ifdef __cplusplus
}
#endif
#endif
