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
 * Test, tuning and measurement hooks (probes, surveys, verification, A/B
 * knobs, phase timing) are declared in rt_hip_test.h.
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

typedef struct rt_hip_ctx rt_hip_ctx;

int rt_hip_device_count(int *n);

/* Deep-copies the scene into device memory of `device` (flattened SoA
 * triangle records, pre-normalised vertex normals, materials, lights) and
 * builds the acceleration structure.  The caller keeps ownership of scene. */
int rt_hip_create(int device, const rt_scene *scene, int accel, rt_hip_ctx **out);
int rt_hip_accel_info(const rt_hip_ctx *ctx, rt_accel_info *out);
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

/* Device memory helpers so C callers need no HIP headers. */
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
