// rt_ctx.h -- the device context (rt_hip_ctx) shared by the host side of the
// C ABI (include/rt_hip.h, include/rt_hip_test.h), split by concern:
//   rt_hip.cpp     context lifetime, settings, light buffers, render, stats,
//                  assemble, the gpu/rt compatibility mode, rt_raytrace
//   rt_lists.cpp   the camera rays' candidate lists (per rank and
//                  triangle-parallel produce / consume) and their surveys
//   rt_verify.cpp  probes, verification, timing and measurement hooks
//   rt_multi.cpp   rt_raytrace_multi: N GPUs, RCCL exchange and gather
// Internal, not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "rt_build.h"
#include "rt_cand.h"
#include "rt_kernels.h"
#include "rt_lightbuf.h"
#include "rt_shadow.h"
#include "rt_reflect.h"
#include "rt_tiles.h"

extern "C" {
#include "../host/rt_cull.h"
#include "../host/rt_internal.h"
}

#ifndef RT_EPS_ULPS_DEFAULT
#define RT_EPS_ULPS_DEFAULT 64
#endif
#ifndef RT_OOB_CAP
#define RT_OOB_CAP (1u << 20)  // deferred shadow queries per render (exact-shadow mode)
#endif
// camera rays (bounce depth 0): a wider slack lets the walk itself find most
// triangles whose float-MT error region is beyond the secondary rays' slack,
// so far fewer go through the per-frame candidate lists
#ifndef RT_CAM_EPS_ULPS_DEFAULT
#define RT_CAM_EPS_ULPS_DEFAULT 64
#endif

#define HIP_TRY(expr)                                                                    \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess)                                                                \
      return rt_set_error(RT_EHIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                          __LINE__);                                                     \
  } while (0)

#define RT_TIMED_FRAMES 1024

// the trace's work order puts the long items of the same frame's previous
// trace first (rt_cand.hip heavy_flag_kernel); 0: entries only (A/B knob)
// asynchronous list builds compact the refinement's kept entries before the
// sort (rt_cand_compact); 0: sort them all (A/B knob)
#ifndef RT_COMPACT_LISTS
#define RT_COMPACT_LISTS 1
#endif
// asynchronous list builds for a new camera of the same size and rank split,
// sized from the last build + headroom (cand_prepare; A/B knob)
#ifndef RT_ASYNC_NEW_CAMERA
#define RT_ASYNC_NEW_CAMERA 1
#endif
// ... also in a fresh (non-asynchronous) build, with a read-back of the kept
// count (A/B knob)
#ifndef RT_COMPACT_FRESH
#define RT_COMPACT_FRESH 1
#endif
#ifndef RT_COST_ORDER
#define RT_COST_ORDER 1
#endif

// per-frame counters (one allocation, rt_hip_ctx::d_counter): 8 item-stream
// counters 128 B apart, the stats, RT_HIT_REGIONS hit-record and as many
// shade-chunk counters 32 words apart
static constexpr size_t kItemCounterBytes = 8 * 128;
static_assert(RT_NSTATS <= RT_STAT_STRIDE, "stat copies overlap");
static constexpr size_t kStatBytes = RT_STAT_SETS * RT_STAT_STRIDE * sizeof(unsigned long long);
static constexpr size_t kHitCounterBytes = 2 * RT_HIT_REGIONS * 32 * sizeof(uint32_t);
static constexpr size_t kCostBytes = 64;  // the trace's item-clock sum (KParams::cost_sum)
static constexpr size_t kFrameCounterBytes =
    kItemCounterBytes + kStatBytes + kHitCounterBytes + kCostBytes;

// The sizes of one list build, which are deterministic for its (camera
// frame, rank, nranks): a later build of the same frame sizes its buffers and
// launches from them instead of reading its own back (async_lists).
struct ListShape {
  int valid = 0;
  rt_frame frame{};
  int rank = -1, nranks = 0;
  uint32_t total = 0, nglobal = 0;           // entries, global prims
  uint32_t nbig = 0, nitems = 0, over = 0;   // the big-emission launch shape
  bool same(const rt_frame* f, int r, int n) const {
    return valid && rank == r && nranks == n && std::memcmp(&frame, f, sizeof *f) == 0;
  }
  // the same image size and rank split (the same tiles), any camera
  bool same_grid(const rt_frame* f, int r, int n) const {
    return valid && rank == r && nranks == n && frame.width == f->width && frame.height == f->height;
  }
  void set(const rt_frame* f, int r, int n) {
    valid = 1;
    frame = *f;
    rank = r;
    nranks = n;
  }
};

struct rt_hip_ctx {
  int device = 0;
  int accel = RT_ACCEL_FLAT;
  int count_work = 0;
  int grid = 0;
  hipStream_t stream = nullptr;
  hipStream_t last_stream = nullptr;
  float4* d_tri = nullptr;
  float* d_nrm = nullptr;
  float* d_mat = nullptr;
  float* d_light = nullptr;
  float4* d_node = nullptr;
  uint32_t* d_counter = nullptr;
  unsigned long long* d_stats = nullptr;
  uint2* d_spill = nullptr;
  uint32_t nrec = 0, nlight = 0;
  rt_accel_info info{};
  float scene_c[3]{}, scene_r = 0;
  float scene_lo[3]{}, scene_hi[3]{};  // the triangles' bounding box
  float eps_ulps = RT_EPS_ULPS_DEFAULT;
  float cam_eps_ulps = RT_CAM_EPS_ULPS_DEFAULT;
  int policy = RT_POLICY_DEFAULT;  // traversal policy (tests / A/B only: rt_hip_set_policy)
  unsigned long long* d_tile_cycles = nullptr;  // COUNT pass: per-item clocks
  // wavefront split (rt_render.hip): hit records of RT_HIT_REGIONS regions
  float4* d_hit = nullptr;          // 2 float4 per record
  uint32_t* d_hit_prev = nullptr;   // per record
  float4* d_hit_term = nullptr;     // per record
  uint32_t* d_hit_count = nullptr;  // RT_HIT_REGIONS append counters + as many shade chunk counters
  size_t hit_cap = 0;               // records per region
  size_t hit_need = 0;              // per region: what the last overflowing frame needed
  uint32_t* d_last = nullptr;       // per (item, lane): a path's deepest record
  size_t last_cap = 0;              // items
// per-rank candidate lists built without a host read-back (VERDICT r04
// "render is async"): 1 = on (the first frame still reads its total back)
#ifndef RT_ASYNC_LISTS_DEFAULT
#define RT_ASYNC_LISTS_DEFAULT 1
#endif
  int grid_of[2][RT_NPOLICIES][2] = {};  // persistent grids [trace][policy][count_work] (4: shade only, 5: trace only)
  int cus = 0;                      // compute units of the device
  std::vector<uint32_t> light_type; // per light (rt_hip_verify_shadows)
  std::vector<float> light_v;       // per light: l.v (3 floats)
  // light buffers (csrc/rt_lightbuf.hip), built for the slack lb_ulps
  int light_buffers = 1;            // rt_hip_set_light_buffers
  std::vector<LBDevice*> lb_dev;    // per light (nullptr: the walk)
  RtLightBuf* d_lbuf = nullptr;     // per light, device
  float lb_ulps = -1.0f;
  int lb_proven = -1;               // built proven (exact_shadows) or slack-grown
  unsigned long long lb_entry_cap = 0;  // test hook: fail builds past this many entries (0: none)
  KParams last_p{};                 // the last render's parameters (rt_hip_verify_shadows)
  // exact shadow rays (csrc/rt_shadow.hip), built for the slack sh_ulps
  float2* d_prim_mu = nullptr;
  float2* d_node_mu = nullptr;
  uint4* d_oob = nullptr;       // exact-shadow mode: deferred off-box shadow queries
  uint32_t* d_oob_count = nullptr;
  unsigned long long* d_frame_check = nullptr;  // KParams::frame_check: sticky per-frame checks (rt_hip_frame_check)
  uint32_t* d_sh_global = nullptr;
  uint32_t n_sh_global = 0;
  // exact reflection rays (csrc/rt_reflect.hip, rt_hip_set_exact_reflections):
  // per-node error-region bounds, built once per tree when the mode is enabled
  int exact_refl = 0;
  float4* d_node_rf = nullptr;
  unsigned long long rf_unbounded = 0;  // leaves holding a triangle no bound covers
  float sh_ulps = -1.0f;
  float sh_omax = 0.0f;
  float sh_mu_max = 1.0f;
  // shadow rays exact by proof (rt_hip_set_exact_shadows, default on): proven
  // light buffers, the per-node multiplier walk where a light has none
  int exact_shadows = 1;
  size_t tile_cycles_cap = 0, tile_cycles_n = 0;
  // exact camera rays (csrc/rt_cand.hip)
  int exact_camera = 1;
  // the big footprints' entries refined per tile (rt_hip_set_camera_refine,
  // default on; RT_CAND_REFINE=0 at context creation turns it off)
#ifndef RT_CAND_REFINE_DEFAULT
#define RT_CAND_REFINE_DEFAULT 1
#endif
  int cand_refine = RT_CAND_REFINE_DEFAULT;
  const uint32_t* d_cand_valid = nullptr;  // device word: the last built lists' entries with a tile
  double bound_scale = 1.0;  // 1 = the proven float-MT error bound (tools/mt_bound.py)
  float4* d_tri_prim = nullptr;  // prim-order records (== d_tri for FLAT)
  uint32_t nprim = 0;
  uint32_t* d_cand_list = nullptr;    // nprim
  void* d_cand_fp = nullptr;          // nprim footprints (rt_cand_footprint_bytes each)
  uint4* d_cand_sfp = nullptr;        // 2 nprim: compact small footprints (CandParams::sfp)
  int cand_store_fp = 0;              // keep every footprint (rt_hip_cand_verify's re-derivation)
  uint32_t* d_cand_visits = nullptr;  // nprim + 1
  uint32_t* d_cand_off = nullptr;     // nprim + 1
  uint32_t* d_cand_start = nullptr;   // ntiles + 1
  uint32_t* d_cand_keys = nullptr;    // entries (tile), emit order
  uint32_t* d_cand_keys2 = nullptr;   // entries (tile), sorted
  uint32_t* d_cand_vals = nullptr;    // entries (prim), emit order
  uint32_t* d_cand_global = nullptr;  // nprim
  uint32_t* d_cand_big = nullptr;     // nprim
  uint32_t* d_cand_ctr = nullptr;     // 4
  float* d_cand_skip = nullptr;       // nprim
  uint32_t* d_cand_big_lane = nullptr;  // kBigLaneCap x 64 lane subtotals of big footprints
  uint2* d_cand_items = nullptr;        // kItemCap big-emission work items
  uint32_t* d_cand_wave_items = nullptr;  // rt_cand_big_waves() + 1 each: items per big_count wave,
  uint32_t* d_cand_wave_base = nullptr;   // and their exclusive scan
  uint32_t* d_scan_bsum = nullptr;        // rt_cand_scan_dev_tiles(nprim) tile sums of the device-length scans
  uint32_t cand_item_cap = 0xffffffffu;  // test hook: fewer items (min with kItemCap)
  uint32_t* d_prim_leaf = nullptr;    // nprim: a leaf holding each prim (camera-independent)
  uint32_t* d_cand = nullptr;
  uint32_t* d_order = nullptr;        // 3 x (ntiles + 1): heavy flags, their scan, the work order
  size_t cand_cap = 0, cand_tiles_cap = 0, order_cap = 0;
  void* d_scan_tmp = nullptr;
  size_t scan_tmp_bytes = 0;
  uint32_t* h_cand = nullptr;  // pinned: a read-back build's ctr[0..7] (rt_cand.h CandParams::ctr)
  // asynchronous per-rank builds (no host read-back in the render path): the
  // entry buffers are sized from an earlier frame's total, read back without
  // waiting when its build has finished
  int async_lists = RT_ASYNC_LISTS_DEFAULT;
  // the frame (camera frame, rank, nranks) whose per-rank lists were last
  // built with a read-back, and their sizes: the same frame's lists are
  // deterministic, so they are rebuilt without reading the total back
  ListShape known;
  ListShape pknown;  // the same for the last read-back produce (rt_hip_cand_produce)
  // the frame (camera frame, rank, nranks) whose trace last recorded its
  // per-item clocks (d_item_cost, their sum in the frame counters) and its
  // grid: the same frame's next work order puts its long items first
  // the entries the refinement kept (start[ntiles]) in the last build of
  // kept_for's frame, read back without waiting (h_kept, ev_kept): the same
  // frame's asynchronous builds compact the entries to that many before the
  // sort instead of sorting the dropped ones too
  ListShape kept_for;
  uint32_t* h_kept = nullptr;   // pinned: [0] the kept count, [1..8] an asynchronous build's counters ctr[0..7]
  hipEvent_t ev_kept = nullptr;
  int snap_pending = 0;         // h_kept[1..8] will hold the last estimated-shape build's counters (ev_kept)
  int kept_ready = 0;           // kept holds kept_for's count
  ListShape kept_pend;          // the frame whose kept count is on its way into h_kept[0] (ev_kept)
  int kept_pending = 0;
  uint32_t kept = 0;
  ListShape cost_hist;
  uint32_t cost_waves = 0;
  uint32_t* d_item_cost = nullptr;  // 4 x ntiles_local
  size_t item_cost_cap = 0;
  int last_async = 0;                 // the last render's lists came from an asynchronous build
  unsigned long long cand_prims = 0, cand_entries = 0, cand_global = 0;
  // triangle-parallel lists (rt_hip_cand_produce / rt_hip_cand_consume)
  uint32_t* d_send = nullptr;   // 3 words per routed entry, destination-rank order
  size_t send_cap = 0;          // words
  uint32_t send_n = 0;          // entries of the last produce
  uint32_t* d_part = nullptr;    // the partition's per-wave rank counts and their scan
  size_t part_cap = 0;          // words
  uint32_t* d_rstart = nullptr;  // nranks + 1 first entries per destination
  uint32_t* h_rstart = nullptr;  // pinned copy
  size_t rstart_cap = 0;
  KParams ext{};                // the consumed lists' kernel parameters
  int ext_ready = 0, ext_rank = -1, ext_nranks = 0;
  rt_frame ext_frame{};         // the frame they were built for (compared bytewise)
  uint32_t ext_total = 0;
  // phase timing (rt_hip_set_timing): per frame, events before the
  // candidate lists, before the render kernel and after it, on the render's
  // stream; a ring of the last RT_TIMED_FRAMES frames
  int timing = 0;
  hipEvent_t ev[RT_TIMED_FRAMES][5] = {};  // lists | trace | shade | fold |
  unsigned long long frames = 0;  // timed frames recorded
};

// A setting that changes the lists: no earlier build's sizes or kept count
// apply any more (the read-backs on their way are discarded too)
static inline void lists_changed(rt_hip_ctx* c) {
  c->known.valid = c->pknown.valid = c->kept_for.valid = 0;
  c->kept_pending = c->snap_pending = 0;
}


int cand_params(const rt_frame* f, const float scene_c[3], float scene_r, float eps_ulps, double bound_scale,
                int rank, int nranks, CandParams* out, int compat = 0);

static inline int tiles_x_of(int W) { return (W + 7) / 8; }
static inline int tiles_y_of(int H) { return (H + 7) / 8; }

// tiles rank `rank` renders (whole blocks, edge padding included; csrc/rt_tiles.h)
static inline int rank_tile_count(int W, int H, int rank, int nranks) {
  const int tb = rt_block_side(nranks);
  return (int)(rt_rank_blocks((uint32_t)rt_blocks_x(tiles_x_of(W), tb), (uint32_t)rt_blocks_y(tiles_y_of(H), tb),
                              (uint32_t)nranks, (uint32_t)rank) * tb * tb);
}


// shared between the files above (defined in the file named)
int shadow_prepare(rt_hip_ctx* c, hipStream_t s);                                  // rt_hip.cpp
void lb_fill(LBParams& lp, const float scene_c[3], float scene_r, const float aabb_lo[3], const float aabb_hi[3],
             float eps_ulps, uint32_t type, const float lv[3], uint32_t nprim, int proven);  // rt_hip.cpp
int lbuf_prepare(rt_hip_ctx* c, hipStream_t s);                                    // rt_hip.cpp
int reflect_prepare(rt_hip_ctx* c, hipStream_t s);                                 // rt_hip.cpp
int choose_accel(const rt_scene* s);                                               // rt_hip.cpp
int cand_prepare(rt_hip_ctx* c, const rt_frame* f, KParams* kp, hipStream_t s, int compat = 0);  // rt_lists.cpp
unsigned long long* cost_sum_of(rt_hip_ctx* c);                                    // rt_lists.cpp

