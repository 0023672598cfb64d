// rt_kernels.h -- parameter block shared by the render kernels and their
// host-side launcher (rt_hip.cpp).  Not part of the public C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_device.h"
#include "rt_lightbuf.h"

#define RT_ACCEL_FLAT_D 0
#define RT_ACCEL_OCTREE_D 1
#define RT_MAT_FLOATS_D 12
#define RT_LIGHT_FLOATS_D 8
// closest-hit queries one path may make before the render reports RT_EDEPTH:
// cpu/rt recurses while coef >= 0.01 (cpu/raytracer.c:19-34), which is
// unbounded for mirrors of Nr >= 1; paths of Nr < 1 end long before this
#define RT_MAX_BOUNCES 16384
#define RT_NSTATS 23
// the counters are kept in RT_STAT_SETS copies RT_STAT_STRIDE words apart,
// wave b adding to copy b % 8 (its XCD's): every wave of a launch flushes
// its counters with a few 64-bit atomics, and on a small frame (C1: 4,096
// waves of one work item each) one copy queued them for most of the kernel;
// rt_hip_stats sums the copies
#define RT_STAT_SETS 8
#define RT_STAT_STRIDE 32
// per-lane global overflow area of the traversal stack (entries beyond LDS)
#define RT_SPILL_STACK 112
// hit records (the wavefront split, rt_render.hip): 8 regions, one per
// item stream, each with its own append counter; a record index is
// region | (slot << 3), RT_NO_REC = none
#define RT_HIT_REGIONS 8
#define RT_NO_REC 0xffffffffu
// occupancy target of the render kernels' launch bounds (waves per SIMD).
// The kernels need 123 VGPRs and 9.7 KB of LDS, so they still run 4 waves
// per SIMD; a target of 3 only changes the scheduler's trade-offs (measured,
// C5 render kernel: 13.86 ms at 4, 13.70 at 3 and at 2; profiles/r02m_waves/).
#ifndef RT_MIN_WAVES
#define RT_MIN_WAVES 3
#endif
// occupancy targets of the wavefront split's kernels (waves per SIMD):
// trace_kernel (closest-hit walks, candidate tests) needs 104 registers left
// alone, 96 at 5 waves (C5 trace 7.35 -> 6.34 ms, profiles/r03d/); shade_kernel
// (shadow queries + Phong per hit record) fits 64 at 8 (7.19 -> 6.89 ms).
// Re-measured with light buffers (profiles/r04c_validate/ab.log, C5): shade
// 1.92 ms at 8, 1.99 at 7, 2.01 at 6; trace 6.22 ms at 5, 7.12 at 4
#ifndef RT_TRACE_MIN_WAVES
#define RT_TRACE_MIN_WAVES 5
#endif
#ifndef RT_SHADE_MIN_WAVES
#define RT_SHADE_MIN_WAVES 7  // 72 VGPRs: the light-buffer scan's record one ahead (rt_render.hip RT_LB_AHEAD)
#endif
// the staged test policies' shade kernels (packet any-hit walks, test / A/B
// only) need more registers than 8 waves allow: their own, reachable, target
#ifndef RT_STAGED_SHADE_MIN_WAVES
#define RT_STAGED_SHADE_MIN_WAVES 4
#endif
// the brute-force (FLAT) shade kernel streams records through LDS, two at a
// time (mt_candidate2): at 8 waves it spilled 96 B per lane
#ifndef RT_FLAT_SHADE_MIN_WAVES
#define RT_FLAT_SHADE_MIN_WAVES 5
#endif
// triangle record flag (q2.w bits, host/accel.c rt_flatten): the record's
// object has a triangle whose interpolated normal can be exactly zero, so
// cpu/hit.c:99 may skip the object in collide_dist (early any-hit exit is
// then not known to be exact)
#define RT_REC_ZERO_RISK 1u
// traversal policies (one kernel instantiation each, rt_render.hip); the
// others exist for tests and A/B measurements
#define RT_POLICY_DEFAULT 0     // staged packet closest hit for coherent queries, per-lane shadows
#define RT_POLICY_LANE 1        // every octree query per lane
#define RT_POLICY_STAGED 2      // every octree query as a staged packet
#define RT_POLICY_DIR_STAGED 3  // default + staged packet directional-light shadows
// shade kernel only, chosen by the host (never by rt_hip_set_policy): the
// default policy when every directional / point light has a light buffer --
// the shadow queries compile to the buffer scan alone, without the octree
// walk's registers and code (the default's fallback for lights without one)
#define RT_POLICY_LBUF 4
// trace kernel only, chosen by the host (rt_hip_set_exact_reflections with
// the default policy): the default plus reflection rays through the proven
// walk (csrc/rt_reflect.hip: per-node error-region growth)
#define RT_POLICY_EXACT_REFL 5
#define RT_NPOLICIES 6

// wave-total counters (wave-uniform, so they live in SGPRs; 32-bit per wave,
// widened to 64-bit by the final atomics)
struct WorkCount {
  uint32_t closest, shadow, pixels, nodes, tris, overflow, zero_normal, hits;
  // per-lane node visits / triangle tests of closest-hit and shadow queries
  // (COUNT pass): a record tested by k lanes counts k times
  uint32_t cl_nodes, cl_tris, sh_nodes, sh_tris;
  // COUNT pass: shader clocks a wave spent in the camera-ray walk, the
  // camera candidate tests, the secondary closest-hit walks and the shadow
  // queries (wall clock of the wave, so shares of its time)
  uint32_t cy_cam, cy_cand, cy_sec, cy_shadow;
  uint32_t cy_shadow_dir;  // the directional-light part of cy_shadow
  uint32_t stack_spills;   // per-lane stack pushes past the LDS entries (COUNT pass)
  uint32_t zero_risk;      // shadow hits on objects whose interpolated normal can vanish
  uint32_t sh_unproven;    // point-light shadow rays from beyond the proof's assumed extent
  uint32_t cl_unproven;    // exact reflection walk: queries with |d| past RT_RF_DLMAX
  // COUNT pass, per work item (rt_hip_tile_phase_cycles phases 4, 5): the
  // most node visits / triangle tests one lane made in per-lane secondary walks
  uint32_t sec_lane_nodes, sec_lane_tris;
};

struct KParams {
  const float4* tri;    // triangle records, 3 float4 each (host/rt_internal.h)
  const float* nrm;     // 9 floats per prim
  const float* mat;     // RT_MAT_FLOATS_D per object
  const float* light;   // RT_LIGHT_FLOATS_D per light
  const float4* node;   // 2 float4 per octree node (NULL for FLAT)
  uint32_t nrec, nlight;
  rt::f3 u, v, C, pos;  // camera frame (cpu/raytracer.c:82-86)
  int W, H;
  int tiles_x, ntiles_total, rank, nranks, ntiles_local;
  float* out;                   // rank's tile buffer (written by fold_kernel)
  // wavefront split (rt_render.hip): trace_kernel appends one hit record per
  // closest hit, shade_kernel turns each into its reflection term, fold_kernel
  // sums every path's terms deepest-first and a pixel's four samples
  float4* hit;                  // RT_HIT_REGIONS x hit_cap records: P.xyz N.x | N.yz coef obj
  uint32_t* hit_prev;           // per record: the path's previous record (RT_NO_REC)
  float4* hit_term;             // per record: color_mul(apply_light(...), coef), rgb
  uint32_t* hit_count;          // RT_HIT_REGIONS append counters, 32 words apart
  uint32_t hit_cap;             // records per region
  uint32_t* last;               // per (item, lane): the path's deepest record (RT_NO_REC)
  uint32_t* shade_counter;      // RT_HIT_REGIONS chunk counters of shade_kernel, 32 words apart
  // shadow verification (rt_hip_verify_shadows; NULL / 0 in renders): the
  // shade pass writes each shaded record's unshadowed-light mask (lights
  // 0..31) and shades only every shade_stride-th record of each region
  uint32_t* hit_lit;
  uint32_t shade_stride;
  uint32_t shade_first;  // ... starting with the shade_first-th
  // exact shadow rays (csrc/rt_shadow.hip): per-node (mu, nu) multipliers of
  // the shadow walk's slack, and the prims every unshadowed shadow ray tests
  // light buffers (csrc/rt_lightbuf.hip), per light; NULL: every shadow query walks
  const RtLightBuf* lbuf;
  const float2* node_mu;
  // exact reflection rays (csrc/rt_reflect.hip, policy RT_POLICY_EXACT_REFL
  // and the closest-hit probe): 3 float4 of error-region bounds per node
  const float4* node_rf;
  const uint32_t* sh_global;
  uint32_t n_sh_global;
  float sh_omax;  // point-light shadow origins with |o - c|_max beyond this are counted unproven
  // exact-shadow mode (proven light buffers): shadow queries of lights 0..31
  // from origins off the proof box are deferred -- shade_kernel appends
  // (record, pending lights, lit lights, 0) and shades with them lit;
  // rt_launch_shade_fixup decides them by brute force and re-shades the record
  uint4* oob;
  uint32_t* oob_count;
  uint32_t oob_cap;
  uint32_t* tile_counter;       // 8 item-stream counters, 32 words apart; zeroed before launch
  unsigned long long* stats;    // RT_NSTATS counters, zeroed before launch
  uint2* spill;                 // grid*64 lanes x RT_SPILL_STACK stack entries
  rt::f3 scene_c;               // scene box centre
  float scene_cmag;             // max-norm of scene_c
  float scene_r;                // scene box half-extent (max-norm)
  float eps_rel;                // culling slack, rt_cull.h rt_cull_eps()
  float eps_rel_cam;            // the same for camera rays (bounce depth 0)
  unsigned long long* tile_cycles;  // COUNT pass: shader clocks of each work item (tile, sample) (NULL: none)
  // camera-ray candidate lists (csrc/rt_cand.hip); cand_start == NULL: none
  const uint32_t* cand_start;   // ntiles_local + 1 offsets into cand
  const uint32_t* cand;         // prims
  const uint32_t* cand_global;  // prims every camera ray tests
  uint32_t n_cand_global;
  const uint32_t* n_cand_global_dev;  // their count on the device (an asynchronous list build), or NULL
  const float4* tri_prim;       // prim-order triangle records
  const float* cand_skip;       // per cand entry: lower bound of new_dist - |pos - o| (depth skip)
  const uint32_t* tile_order;   // trace_kernel's work order: position -> rank-local tile (NULL: identity)
  // the trace's per-item cost (shader clocks of each (tile, sample) item,
  // saturated to 32 bits) and their sum (zeroed before launch), for the next
  // frame's work order (rt_cand_order); NULL: not recorded
  uint32_t* item_cost;
  unsigned long long* cost_sum;
  // the heavy tiles at the front of tile_order (rt_cand_order's count, on
  // the device; NULL: none): their items run at raised wave priority
  const uint32_t* n_heavy;
  // per-frame completeness check (fold_kernel, the frame's last launch): the
  // conditions rt_hip_stats reports as errors, ORed into frame_check[0]
  // (RT_FRAME_*), frame_check[1] += 1 frame, [2] / [3] += its closest-hit /
  // shadow queries -- sticky across frames until rt_hip_frame_check reads
  // them, so a timed loop of many frames is checked and counted as a whole.
  // list_flag: the frame's asynchronous list build's overflow flag (ctr[7]),
  // or NULL
  unsigned long long* frame_check;
  const uint32_t* list_flag;
};
#define RT_FRAME_HITBUF 1u     // hit records past a region's capacity
#define RT_FRAME_DEPTH 2u      // bounce limit or traversal stack overflow
#define RT_FRAME_ZERO 4u       // zero interpolated normal (closest or shadow)
#define RT_FRAME_UNPROVEN 8u   // shadow queries the exact mode could not decide
#define RT_FRAME_LISTS 16u     // asynchronous list build overflow

// The three launches of one render (policy = RT_POLICY_*, octree only):
// trace (closest hits -> hit records), shade (shadow queries + Phong per
// record -> terms), fold (terms -> the rank's tile buffer)
extern "C" hipError_t rt_launch_trace(const KParams* p, int accel, int count_work, int policy,
                                      int grid, hipStream_t stream);
extern "C" hipError_t rt_launch_shade(const KParams* p, int accel, int count_work, int policy,
                                      int grid, hipStream_t stream);
// exact-shadow mode: the deferred queries of shade_kernel (p->oob), brute
// force over the nprim prim-order records, then their records re-shaded
extern "C" hipError_t rt_launch_shade_fixup(const KParams* p, uint32_t nprim, hipStream_t stream);
extern "C" hipError_t rt_launch_fold(const KParams* p, hipStream_t stream);
// shadow-query probe: light li's shadow ray from each of n origins through
// the light buffer p->lbuf[li] (brute = 0) or brute force over nprim
// prim-order records p->tri_prim (brute = 1); out[i] = shadowed
extern "C" hipError_t rt_launch_probe_shadow(const KParams* p, const float* org, uint32_t n, uint32_t li,
                                             uint32_t nprim, int brute, uint32_t* out, hipStream_t stream);
// closest-hit probe: ray i = (org[i], dir[i]) through the per-lane walk of a
// reflection ray (brute = 0) or brute force over nprim prim-order records
// (brute = 1); out[2 i] = winner prim (~0: none), out[2 i + 1] = new_dist bits.
// The walk's spill area p->spill holds `grid` waves: n <= 64 grid.
extern "C" hipError_t rt_launch_probe_closest(const KParams* p, const float* org, const float* dir, uint32_t n,
                                              uint32_t nprim, int brute, uint32_t* out, int grid, hipStream_t stream);
// persistent grid (one-wave workgroups) of trace (trace = 1) or shade on `cus` CUs
extern "C" hipError_t rt_render_grid(int trace, int accel, int count_work, int policy, int cus,
                                     int* grid);
// gpu/rt compatibility mode: p->W x p->H = the 3x upscaled frame, p->out =
// its packed RGBA8 image; then the 3x3 downscale to W x H (PNG row order)
extern "C" hipError_t rt_launch_compat(const KParams* p, int accel, int grid, hipStream_t stream);
extern "C" hipError_t rt_launch_downscale(const uint32_t* hi, uint32_t* lo, int W, int H,
                                          hipStream_t stream);
extern "C" hipError_t rt_launch_assemble(const float* tiles, float* rgb, int W, int H, int tiles_x,
                                         int ntiles, int nranks, int tiles_per_rank,
                                         hipStream_t stream);
