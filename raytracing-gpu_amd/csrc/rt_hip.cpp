// rt_hip.cpp -- host side of the C ABI declared in include/rt_hip.h.
//
// Owns device memory, streams and launches; the scene preparation (flatten,
// octree) is host C (host/accel.c).  No CPU fallback: every entry point fails
// with RT_ENODEV / RT_EHIP when the gfx950 device or the kernels are missing.
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
  int kept_ready = 0;           // h_kept holds kept_for's count
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

static int cand_params(const rt_frame* f, const float scene_c[3], float scene_r, float eps_ulps,
                       double bound_scale, int rank, int nranks, CandParams* out, int compat = 0);

static int tiles_x_of(int W) { return (W + 7) / 8; }
static int tiles_y_of(int H) { return (H + 7) / 8; }

// tiles rank `rank` renders (whole blocks, edge padding included; csrc/rt_tiles.h)
static int rank_tile_count(int W, int H, int rank, int nranks) {
  const int tb = rt_block_side(nranks);
  return (int)(rt_rank_blocks((uint32_t)rt_blocks_x(tiles_x_of(W), tb), (uint32_t)rt_blocks_y(tiles_y_of(H), tb),
                              (uint32_t)nranks, (uint32_t)rank) * tb * tb);
}

extern "C" int rt_hip_tiles_per_rank(int width, int height, int nranks) {
  if (width <= 0 || height <= 0 || nranks <= 0) return 0;
  const int tb = rt_block_side(nranks);
  return (int)(rt_max_rank_blocks((uint32_t)rt_blocks_x(tiles_x_of(width), tb),
                                  (uint32_t)rt_blocks_y(tiles_y_of(height), tb), (uint32_t)nranks) * tb * tb);
}

extern "C" int rt_tile_map_check(int width, int height, int nranks, int maxw, unsigned long long out[2]) {
  if (!out || width <= 0 || height <= 0 || nranks <= 0 || maxw <= 0) return rt_set_error(RT_EINVAL, "bad argument");
  out[0] = out[1] = 0;
  const int tx = tiles_x_of(width), ty = tiles_y_of(height), tb = rt_block_side(nranks);
  const uint32_t bx = (uint32_t)rt_blocks_x(tx, tb), n = (uint32_t)nranks;
  // every tile: local index <-> (tx, ty) round trip, inside the rank's count,
  // each (rank, local) slot used once
  {
    std::vector<uint32_t> cnt(n, 0);
    std::vector<std::vector<char>> used(n);
    for (uint32_t r = 0; r < n; r++) used[r].assign((size_t)rank_tile_count(width, height, (int)r, nranks), 0);
    uint32_t mx = 0;
    for (int y = 0; y < ty; y++)
      for (int x = 0; x < tx; x++) {
        uint32_t rk;
        const uint32_t loc = rt_tile_local(x, y, n, bx, (uint32_t)tb, &rk);
        int x2 = -1, y2 = -1;
        rt_tile_xy(loc, rk, n, bx, (uint32_t)tb, &x2, &y2);
        const bool bad = rk >= n || loc >= used[rk].size() || used[rk][loc] || x2 != x || y2 != y;
        if (!bad) used[rk][loc] = 1;
        out[0]++;
        out[1] += bad ? 1 : 0;
      }
    for (uint32_t r = 0; r < n; r++) mx = std::max(mx, (uint32_t)used[r].size());
    out[0]++;
    out[1] += mx == (uint32_t)rt_hip_tiles_per_rank(width, height, nranks) ? 0 : 1;
  }
  for (int y = 0; y < ty; y++)
    for (int x0 = 0; x0 < tx; x0++)
      for (int x1 = x0; x1 < tx && x1 < x0 + maxw; x1++)
        for (uint32_t r = 0; r < n; r++) {
          // brute force: the rank's tiles of the interval in column order
          std::vector<int> want;
          for (int x = x0; x <= x1; x++) {
            uint32_t rk;
            (void)rt_tile_local(x, y, n, bx, (uint32_t)tb, &rk);
            if (rk == r) want.push_back(x);
          }
          int f = 0;
          const uint32_t c = rt_rank_row_tiles(y, x0, x1, n, r, bx, (uint32_t)tb, &f);
          bool bad = c != want.size();
          // the emission order (emit_interval): blocks f, f + n, ... at
          // consecutive rank-local block indices from rt_block_local
          uint32_t blk = c ? rt_block_local((uint32_t)f, (uint32_t)(y / tb), n, bx, r) : 0;
          size_t k = 0;
          for (int b = f; !bad && k < c; b += (int)n, blk++)
            for (int x = std::max(x0, b * tb); x <= std::min(x1, b * tb + tb - 1); x++, k++) {
              uint32_t rk;
              const uint32_t loc = rt_tile_local(x, y, n, bx, (uint32_t)tb, &rk);
              if (k >= want.size() || want[k] != x || rk != r || loc / (uint32_t)(tb * tb) != blk) bad = true;
            }
          out[0]++;
          out[1] += bad ? 1 : 0;
        }
  return RT_OK;
}

extern "C" size_t rt_hip_tile_buffer_floats(int width, int height, int nranks) {
  return (size_t)rt_hip_tiles_per_rank(width, height, nranks) * 64 * 3;
}

extern "C" int rt_hip_device_count(int* n) {
  if (!n) return rt_set_error(RT_EINVAL, "null argument");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess || c <= 0) {
    *n = 0;
    return rt_set_error(RT_ENODEV, "no HIP device (%s)", hipGetErrorString(e));
  }
  *n = c;
  return RT_OK;
}

template <class T>
static int upload(T** dst, const void* src, size_t bytes) {
  if (bytes == 0) bytes = 16;
  HIP_TRY(hipMalloc((void**)dst, bytes));
  if (src) HIP_TRY(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
  return RT_OK;
}

extern "C" void rt_hip_destroy(rt_hip_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipFree(c->d_tri);
  (void)hipFree(c->d_nrm);
  (void)hipFree(c->d_mat);
  (void)hipFree(c->d_light);
  (void)hipFree(c->d_node);
  (void)hipFree(c->d_counter);  // also holds d_stats and d_hit_count (kFrameCounterBytes)
  (void)hipFree(c->d_spill);
  (void)hipFree(c->d_tile_cycles);
  (void)hipFree(c->d_hit);
  (void)hipFree(c->d_hit_prev);
  (void)hipFree(c->d_hit_term);
  (void)hipFree(c->d_last);
  (void)hipFree(c->d_prim_mu);
  (void)hipFree(c->d_node_mu);
  (void)hipFree(c->d_oob);
  (void)hipFree(c->d_oob_count);
  (void)hipFree(c->d_frame_check);
  (void)hipFree(c->d_node_rf);
  (void)hipFree(c->d_sh_global);
  for (LBDevice* d : c->lb_dev) rt_lightbuf_free(d);
  (void)hipFree(c->d_lbuf);
  if (c->d_tri_prim != c->d_tri) (void)hipFree(c->d_tri_prim);
  (void)hipFree(c->d_cand_list);
  (void)hipFree(c->d_cand_fp);
  (void)hipFree(c->d_cand_sfp);
  (void)hipFree(c->d_cand_visits);
  (void)hipFree(c->d_cand_off);
  (void)hipFree(c->d_cand_start);
  (void)hipFree(c->d_cand_keys);
  (void)hipFree(c->d_cand_keys2);
  (void)hipFree(c->d_cand_vals);
  (void)hipFree(c->d_cand_global);
  (void)hipFree(c->d_cand_big);
  (void)hipFree(c->d_cand_ctr);
  (void)hipFree(c->d_cand_big_lane);
  (void)hipFree(c->d_cand_items);
  (void)hipFree(c->d_cand_wave_items);
  (void)hipFree(c->d_cand_wave_base);
  (void)hipFree(c->d_scan_bsum);
  (void)hipFree(c->d_cand_skip);
  (void)hipFree(c->d_prim_leaf);
  (void)hipFree(c->d_cand);
  (void)hipFree(c->d_order);
  (void)hipFree(c->d_scan_tmp);
  if (c->h_cand) (void)hipHostFree(c->h_cand);
  (void)hipFree(c->d_send);
  (void)hipFree(c->d_rstart);
  (void)hipFree(c->d_part);
  (void)hipFree(c->d_item_cost);
  if (c->h_kept) (void)hipHostFree(c->h_kept);
  if (c->ev_kept) (void)hipEventDestroy(c->ev_kept);
  if (c->h_rstart) (void)hipHostFree(c->h_rstart);
  for (auto& f : c->ev)
    for (hipEvent_t e : f)
      if (e) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

// Per-node slack multipliers of the shadow walk for the context's culling
// slack (csrc/rt_shadow.hip): once per scene and slack, on the context's
// stream, synchronous (setup; it reads back the global list's length).
static int shadow_prepare(rt_hip_ctx* c, hipStream_t s) {
  if (!c->exact_shadows || c->accel != RT_ACCEL_OCTREE || !c->d_node) return RT_OK;
  if (c->d_node_mu && c->sh_ulps == c->eps_ulps) return RT_OK;
  const size_t np = c->nprim, nn = c->info.nodes;
  if (!c->d_node_mu) {
    HIP_TRY(hipMalloc((void**)&c->d_prim_mu, (np + 1) * sizeof(float2)));
    HIP_TRY(hipMalloc((void**)&c->d_sh_global, (np + 1) * sizeof(uint32_t)));
    HIP_TRY(hipMalloc((void**)&c->d_node_mu, (nn + 1) * sizeof(float2)));
  }
  uint32_t* d_n = nullptr;
  HIP_TRY(hipMalloc((void**)&d_n, sizeof(uint32_t)));
  ShadowParams sp;
  std::memset(&sp, 0, sizeof sp);
  sp.tri = c->d_tri_prim;
  sp.nprim = c->nprim;
  sp.light = c->d_light;
  sp.nlight = c->nlight;
  sp.node = c->d_node;
  sp.nnode = (uint32_t)nn;
  sp.rec = c->d_tri;
  for (int a = 0; a < 3; a++) sp.c[a] = c->scene_c[a];
  sp.R = c->scene_r;
  // the walk computes eps(o) in float (host/rt_cull.h); the multipliers keep
  // a relative margin of 1e-6 and the +1 of the original slack on top
  sp.eps_rel = (double)(c->eps_ulps * 5.9604645e-8f);
  const double cmag = std::fmax(std::fabs(c->scene_c[0]), std::fmax(std::fabs(c->scene_c[1]),
                                                                  std::fabs(c->scene_c[2])));
  sp.plane_eps = (double)RT_CULL_PLANE * (cmag + c->scene_r) + 1e-6;
  // point lights: shadow rays leave hit points, which lie on the scene's
  // triangles up to the float error of their hit; origins beyond twice the
  // scene's extent are counted (rt_stats.shadow_unproven), never assumed
  sp.omax_assumed = 2.0 * c->scene_r + 1.0;
  sp.reach_cap = c->scene_r + 1.0;
  sp.prim_mu = c->d_prim_mu;
  sp.node_mu = c->d_node_mu;
  sp.global = c->d_sh_global;
  sp.nglobal = d_n;
  uint32_t n = 0;
  std::vector<float2> nm(1);
  hipError_t he = hipMemsetAsync(d_n, 0, sizeof(uint32_t), s);
  if (he == hipSuccess) he = rt_shadow_build(&sp, (int)c->info.max_depth + 2, s);
  if (he == hipSuccess) he = hipMemcpyAsync(&n, d_n, sizeof n, hipMemcpyDeviceToHost, s);
  if (he == hipSuccess) he = hipMemcpyAsync(nm.data(), c->d_node_mu, sizeof(float2), hipMemcpyDeviceToHost, s);
  if (he == hipSuccess) he = hipStreamSynchronize(s);
  (void)hipFree(d_n);
  if (he != hipSuccess) return rt_set_error(RT_EHIP, "shadow multipliers: %s", hipGetErrorString(he));
  c->n_sh_global = n;
  c->sh_omax = (float)(sp.omax_assumed * (1.0 - 1e-6));
  c->sh_mu_max = nm[0].x;  // the root's: the max over the scene
  c->sh_ulps = c->eps_ulps;
  c->info.shadow_global = n;
  c->info.shadow_mu_max = nm[0].x;
  return RT_OK;
}

// Light buffers of the scene's directional and point lights for the
// context's culling slack (csrc/rt_lightbuf.hip): once per scene and slack,
// synchronous (setup).  The shadow queries of the default walk then look up
// the cells their origins project to instead of walking the octree.
static void lbuf_release(rt_hip_ctx* c) {
  for (LBDevice*& d : c->lb_dev) {
    rt_lightbuf_free(d);
    d = nullptr;
  }
  (void)hipFree(c->d_lbuf);
  c->d_lbuf = nullptr;
  c->lb_ulps = -1.0f;
}

// The build parameters of one light's buffer for a scene of nprim triangles
// in the box (scene_c, scene_r) and the culling slack eps_ulps.
static void lb_fill(LBParams& lp, const float scene_c[3], float scene_r, const float aabb_lo[3],
                    const float aabb_hi[3], float eps_ulps, uint32_t type, const float lv[3], uint32_t nprim,
                    int proven) {
  std::memset(&lp, 0, sizeof lp);
  // a shadow ray leaves a hit point: inside the scene cube up to the float
  // error of the hit, so its slack eps(o) (host/rt_cull.h, float) is at most
  const double R = scene_r, eps_rel = (double)(eps_ulps * 5.9604645e-8f);
  const double cmag = std::fmax(std::fabs(scene_c[0]), std::fmax(std::fabs(scene_c[1]), std::fabs(scene_c[2])));
  const double slack = (eps_rel * (2.0 * R * 1.001 + 1e-3) + (double)RT_CULL_PLANE * (cmag + R) + 1e-6) * 1.01;
  double lo[3], hi[3], s1 = 0.0;
  for (int a = 0; a < 3; a++) {
    if (proven) {
      // the proof's origin box: the triangles' box grown by 1 + 1 % of the
      // scene (hit points off it -- float garbage hits beyond that -- are
      // counted by the shade pass, never assumed)
#ifndef RT_LB_PROOF_BOX
#define RT_LB_PROOF_BOX 1.0  // the proof box: the triangles' box grown by g = RT_LB_PROOF_BOX (1 + 0.02 R)
#endif
      const double g = RT_LB_PROOF_BOX * (1.0 + 0.02 * R);
      lo[a] = (double)aabb_lo[a] - g;
      hi[a] = (double)aabb_hi[a] + g;
    } else {
      lo[a] = scene_c[a] - R * 1.001 - 1e-3;
      hi[a] = scene_c[a] + R * 1.001 + 1e-3;
    }
    s1 += std::fmax(std::fabs(lo[a]), std::fabs(hi[a]));
  }
  lp.nprim = nprim;
  lp.kind = type == 1 ? RT_LB_DIR : RT_LB_POINT;
  double dmax = 0.0;
  for (int a = 0; a < 3; a++) {
    lp.lv[a] = lv[a];
    lp.box_lo[a] = lo[a];
    lp.box_hi[a] = hi[a];
  }
  for (int k = 0; k < 8; k++) {
    double d2 = 0.0;
    for (int a = 0; a < 3; a++) {
      const double x = ((k >> a) & 1 ? hi[a] : lo[a]) - lp.lv[a];
      d2 += x * x;
    }
    dmax = std::fmax(dmax, std::sqrt(d2));
  }
  lp.slack = slack;
  lp.s1 = s1;
  lp.dmax = dmax * 1.01 + 1.0;
  // two cells per triangle: C5 shade 1.97 -> 1.93 ms against one (half: 2.12,
  // four: 2.09; 117 M -> 172 M proven entries, 8 GB; profiles/r05x_tuning/)
  const uint64_t cells = 2ull * nprim;
  lp.target_cells = cells < 4096u ? 4096u : (cells > (1u << 25) ? (1u << 25) : (uint32_t)cells);
  lp.proven = proven ? 1u : 0u;
}

static int lbuf_prepare(rt_hip_ctx* c, hipStream_t s) {
  if (!c->light_buffers || c->accel != RT_ACCEL_OCTREE || !c->d_node || !c->nlight) return RT_OK;
  if (c->d_lbuf && c->lb_ulps == c->eps_ulps && c->lb_proven == c->exact_shadows) return RT_OK;
  lbuf_release(c);
  c->lb_dev.assign(c->nlight, nullptr);
  c->info.lightbuf_fail_reason[0] = 0;
  std::vector<RtLightBuf> hb(c->nlight);
  std::memset(hb.data(), 0, hb.size() * sizeof(RtLightBuf));
  char err[256] = {0};
  uint32_t failed = 0;
  for (uint32_t li = 0; li < c->nlight; li++) {
    const uint32_t t = c->light_type[li];
    if (t != 1 && t != 2) continue;
    LBParams lp;
    lb_fill(lp, c->scene_c, c->scene_r, c->scene_lo, c->scene_hi, c->eps_ulps, t, &c->light_v[3 * li], c->nprim,
            c->exact_shadows);
    lp.tri = c->d_tri_prim;
    lp.max_entries = c->lb_entry_cap;
    if (const char* e = std::getenv("RT_LB_CELLS")) {  // build tuning: cells per triangle
      const double k = std::atof(e);
      if (k > 0.0) lp.target_cells = (uint32_t)std::fmin((double)(1u << 26), std::fmax(4096.0, lp.target_cells * k));
    }
    const int br = rt_lightbuf_build(&lp, &hb[li], &c->lb_dev[li], s, err, sizeof err);
    if (br < 0) {  // not a capacity question: a failed launch or an inconsistent build
      (void)hipGetLastError();
      for (LBDevice*& d : c->lb_dev) {
        rt_lightbuf_free(d);
        d = nullptr;
      }
      return rt_set_error(RT_EHIP, "light buffer of light %u: %s", li, err);
    }
    if (br > 0) {
      // entry or cell cap, device memory, or a zero directional vector (no
      // grid): the light's queries walk the octree instead (hb[li] is zeroed:
      // RT_LB_NONE), as they did before light buffers -- a scene that fits the
      // walk still loads; in the exact-shadow mode that walk is the proven
      // per-node multiplier walk (shadow_prepare, built by the render)
      std::memset(&hb[li], 0, sizeof hb[li]);
      c->lb_dev[li] = nullptr;
      (void)hipGetLastError();  // an out-of-memory hipMalloc is not sticky; clear it anyway
      std::snprintf(c->info.lightbuf_fail_reason, sizeof c->info.lightbuf_fail_reason, "light %u: %s", li, err);
      failed++;
    }
  }
  c->info.lightbuf_failed = failed;
  HIP_TRY(hipMalloc((void**)&c->d_lbuf, hb.size() * sizeof(RtLightBuf)));
  HIP_TRY(hipMemcpy(c->d_lbuf, hb.data(), hb.size() * sizeof(RtLightBuf), hipMemcpyHostToDevice));
  c->lb_ulps = c->eps_ulps;
  c->lb_proven = c->exact_shadows;
  unsigned long long e = 0, n = 0, g = 0, te = 0, tg = 0, nv = 0, bd = 0, tnv = 0, tbd = 0;
  for (LBDevice* d : c->lb_dev) {
    rt_lightbuf_sizes(d, &e, &n, &g);
    rt_lightbuf_proof_counts(d, &nv, &bd);
    te += e;
    tg += g;
    tnv += nv;
    tbd += bd;
  }
  c->info.lightbuf_entries = te;
  c->info.lightbuf_global = tg;
  c->info.lightbuf_never = tnv;
  c->info.lightbuf_band = tbd;
  return RT_OK;
}

// Host-only survey of a light's buffer as rt_hip_create would build it for
// this scene (prim-order records, the scene's box, the default culling
// slack): rt_lightbuf_survey_host's counts (csrc/rt_lightbuf.h).
extern "C" int rt_lightbuf_survey(const rt_scene* scene, unsigned light, int exact, unsigned stride,
                                  unsigned long long out[12]) {
  if (!scene || !out) return rt_set_error(RT_EINVAL, "null argument");
  if (light >= scene->light_count || (scene->lights[light].type != 1 && scene->lights[light].type != 2))
    return rt_set_error(RT_EINVAL, "light %u is not a directional or point light", light);
  rt_flat_scene fs;
  int rc = rt_flatten(scene, RT_ACCEL_FLAT, &fs);
  if (rc) return rc;
  float sc[3], sr = 0.0f, blo[3], bhi[3];
  for (int a = 0; a < 3; a++) {
    const float lo = fs.ntri ? fs.scene_lo[a] : 0.0f, hi = fs.ntri ? fs.scene_hi[a] : 0.0f;
    sc[a] = 0.5f * (lo + hi);
    sr = std::fmax(sr, 0.5f * (hi - lo));
    blo[a] = lo;
    bhi[a] = hi;
  }
  const float lv[3] = {scene->lights[light].v.x, scene->lights[light].v.y, scene->lights[light].v.z};
  LBParams lp;
  lb_fill(lp, sc, sr, blo, bhi, (float)RT_EPS_ULPS_DEFAULT, (uint32_t)scene->lights[light].type, lv,
          (uint32_t)fs.ntri, exact);
  lp.tri = (const float4*)fs.tri;
  char err[256] = {0};
  if (rt_lightbuf_survey_host(&lp, stride, out, err, sizeof err)) rc = rt_set_error(RT_EINVAL, "%s", err);
  rt_flat_free(&fs);
  return rc;
}

extern "C" int rt_hip_set_light_buffers(rt_hip_ctx* c, int enable) {
  if (!c) return rt_set_error(RT_EINVAL, "null context");
  c->light_buffers = enable ? 1 : 0;
  if (!c->light_buffers) lbuf_release(c);
  return RT_OK;
}

extern "C" int rt_hip_set_lightbuf_entry_cap(rt_hip_ctx* c, unsigned long long cap) {
  if (!c) return rt_set_error(RT_EINVAL, "null context");
  c->lb_entry_cap = cap;
  lbuf_release(c);  // rebuilt (and the cap applied) by the next render
  HIP_TRY(hipSetDevice(c->device));
  return lbuf_prepare(c, c->stream);
}

extern "C" int rt_hip_create(int device, const rt_scene* scene, int accel, rt_hip_ctx** out) {
  if (!scene || !out) return rt_set_error(RT_EINVAL, "null argument");
  if (accel != RT_ACCEL_FLAT && accel != RT_ACCEL_OCTREE && accel != RT_ACCEL_OCTREE_GPU)
    return rt_set_error(RT_EINVAL, "unknown accel %d", accel);
  const bool dev_build = accel == RT_ACCEL_OCTREE_GPU;
  int ndev = 0;
  int rc = rt_hip_device_count(&ndev);
  if (rc) return rc;
  if (device < 0 || device >= ndev) return rt_set_error(RT_ENODEV, "device %d of %d", device, ndev);
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return rt_set_error(RT_ENODEV, "device %d is %s, kernels are built for gfx950", device,
                        prop.gcnArchName);
  HIP_TRY(hipSetDevice(device));

  auto t0 = std::chrono::steady_clock::now();
  rt_flat_scene fs;
  // device build: the host only flattens (prim-order records, normals,
  // materials, lights); the octree is built from the uploaded records
  rc = rt_flatten(scene, dev_build ? RT_ACCEL_FLAT : accel, &fs);
  if (rc) return rc;
  auto t1 = std::chrono::steady_clock::now();

  rt_hip_ctx* c = new rt_hip_ctx();
  if (const char* e = std::getenv("RT_CAND_REFINE")) c->cand_refine = std::atoi(e) != 0;  // A/B knob
  if (const char* e = std::getenv("RT_ASYNC_LISTS")) c->async_lists = std::atoi(e) != 0;  // A/B knob
  c->device = device;
  c->accel = dev_build ? (fs.ntri ? RT_ACCEL_OCTREE : RT_ACCEL_FLAT) : accel;
  c->nrec = (uint32_t)fs.nrec;
  c->nlight = (uint32_t)fs.nlight;
  size_t bytes_tri = fs.nrec * RT_TRI_FLOATS * sizeof(float);
  size_t bytes_nrm = fs.ntri * 9 * sizeof(float);
  size_t bytes_mat = fs.nobj * RT_MAT_FLOATS * sizeof(float);
  size_t bytes_light = fs.nlight * RT_LIGHT_FLOATS * sizeof(float);
  size_t bytes_node = fs.nnode * RT_NODE_FLOATS * sizeof(float);
  rc = upload(&c->d_tri, fs.tri, bytes_tri);
  if (!rc) rc = upload(&c->d_nrm, fs.nrm, bytes_nrm);
  if (!rc) rc = upload(&c->d_mat, fs.mat, bytes_mat);
  if (!rc) rc = upload(&c->d_light, fs.light, bytes_light);
  if (!rc && fs.nnode) rc = upload(&c->d_node, fs.node, bytes_node);
  // the per-frame counters in one allocation, zeroed by one memset per frame:
  // 8 item-stream counters (rt_render.hip), the stats, the hit-record and
  // shade-chunk counters
  if (!rc) rc = upload(&c->d_counter, nullptr, kFrameCounterBytes);
  if (!rc) {
    c->d_stats = (unsigned long long*)((char*)c->d_counter + kItemCounterBytes);
    c->d_hit_count = (uint32_t*)((char*)c->d_counter + kItemCounterBytes + kStatBytes);
  }
  if (!rc && hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
    rc = rt_set_error(RT_EHIP, "hipStreamCreate");
  rt_device_tree tree{};
  if (!rc && dev_build && fs.ntri) {
    // leaf cap 24 measured best on C5 with the trace / shade / fold split and
    // the candidate lists (12: 10.01-10.06 ms, 20 / 24: 9.89, 28: 9.99, 32: 10.01;
    // profiles/r05u_leaf_sweep/); clip level 7 (6 / 8 no better)
    rt_device_build_opts o{24, 7};
    if (const char* e = std::getenv("RT_DEV_LEAF")) o.leaf_cap = std::atoi(e);  // tuning knobs
    if (const char* e = std::getenv("RT_DEV_CLIP")) o.clip_level = std::atoi(e);
    hipError_t he = rt_device_build_octree(c->d_tri, (uint32_t)fs.ntri, fs.scene_lo, fs.scene_hi,
                                           &o, c->stream, &tree);
    if (he != hipSuccess) {
      rc = rt_set_error(RT_EHIP, "device octree build: %s", hipGetErrorString(he));
    } else {
      // leaf-order records for the walk; the prim-order ones stay for the
      // camera candidate lists
      c->d_tri_prim = c->d_tri;
      c->d_tri = tree.tri;
      c->d_node = tree.node;
      c->nrec = tree.nref;
      bytes_tri = (size_t)tree.nref * RT_TRI_FLOATS * sizeof(float);
      bytes_node = (size_t)tree.nnode * RT_NODE_FLOATS * sizeof(float);
      fs.nrec = tree.nref;
      fs.nnode = tree.nnode;
      fs.leaves = tree.leaves;
      fs.max_depth = tree.depth;
      fs.max_leaf = tree.max_leaf;
    }
  }
  auto t2 = std::chrono::steady_clock::now();
  c->nprim = (uint32_t)fs.ntri;
  if (!rc && !c->d_tri_prim) {
    if (c->accel == RT_ACCEL_FLAT) {
      c->d_tri_prim = c->d_tri;  // already prim order (no candidates needed)
    } else {
      rt_flat_scene fp;  // host octree: records are leaf order, with duplicates
      rc = rt_flatten(scene, RT_ACCEL_FLAT, &fp);
      if (!rc) {
        rc = upload(&c->d_tri_prim, fp.tri, fp.nrec * RT_TRI_FLOATS * sizeof(float));
        rt_flat_free(&fp);
      }
    }
  }
  for (int a = 0; a < 3; a++) {
    float lo = fs.ntri ? fs.scene_lo[a] : 0.0f, hi = fs.ntri ? fs.scene_hi[a] : 0.0f;
    c->scene_lo[a] = lo;
    c->scene_hi[a] = hi;
    c->scene_c[a] = 0.5f * (lo + hi);
    c->scene_r = std::fmax(c->scene_r, 0.5f * (hi - lo));
  }
  c->info.triangles = fs.ntri;
  c->info.tri_refs = fs.nrec;
  c->info.nodes = fs.nnode;
  c->info.leaves = fs.leaves;
  c->info.max_depth = fs.max_depth;
  c->info.max_leaf = fs.max_leaf;
  c->info.tri_record_bytes = RT_TRI_FLOATS * sizeof(float);
  c->info.node_record_bytes = RT_NODE_FLOATS * sizeof(float);
  c->info.device_bytes = bytes_tri + bytes_nrm + bytes_mat + bytes_light + bytes_node;
  c->info.build_seconds = std::chrono::duration<double>(dev_build ? t2 - t0 : t1 - t0).count();
  rt_flat_free(&fs);
  if (rc) {
    rt_hip_destroy(c);
    return rc;
  }
  // persistent grids: as many one-wave workgroups as each kernel's
  // registers and LDS let a CU hold (rt_render_grid); the compat kernel
  // keeps 16 per CU
  c->grid = prop.multiProcessorCount * 16;
  c->cus = prop.multiProcessorCount;
  for (size_t li = 0; li < scene->light_count; li++) {
    c->light_type.push_back((uint32_t)scene->lights[li].type);
    c->light_v.push_back(scene->lights[li].v.x);
    c->light_v.push_back(scene->lights[li].v.y);
    c->light_v.push_back(scene->lights[li].v.z);
  }
  int gmax = c->grid;
  const int dacc = c->accel == RT_ACCEL_FLAT ? RT_ACCEL_FLAT_D : RT_ACCEL_OCTREE_D;
  for (int tr = 0; tr < 2; tr++)
    for (int pol = 0; pol < RT_NPOLICIES; pol++)
      for (int cw = 0; cw < 2; cw++) {
        int g = 0;
        hipError_t he = rt_render_grid(tr, dacc, cw, pol, prop.multiProcessorCount, &g);
        if (he != hipSuccess) {
          rt_hip_destroy(c);
          return rt_set_error(RT_EHIP, "occupancy query: %s", hipGetErrorString(he));
        }
        c->grid_of[tr][pol][cw] = g;
        gmax = g > gmax ? g : gmax;
      }
  c->info.trace_grid = c->grid_of[1][RT_POLICY_DEFAULT][0];
  c->info.shade_grid = c->grid_of[0][RT_POLICY_LBUF][0];
  for (int a = 0; a < 3; a++) c->info.scene_center[a] = c->scene_c[a];
  c->info.scene_radius = c->scene_r;
  // per-lane traversal stack spill area, [entry][lane] for the largest grid
  if (c->accel == RT_ACCEL_OCTREE &&
      hipMalloc((void**)&c->d_spill, (size_t)gmax * 64 * RT_SPILL_STACK * sizeof(uint2)) != hipSuccess) {
    rt_hip_destroy(c);
    return rt_set_error(RT_EHIP, "hipMalloc traversal spill stack");
  }
  {  // light buffers: part of the scene's setup, like the octree
    const auto l0 = std::chrono::steady_clock::now();
    rc = lbuf_prepare(c, c->stream);
    c->info.lightbuf_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - l0).count();
    if (rc) {
      rt_hip_destroy(c);
      return rc;
    }
  }
  *out = c;
  return RT_OK;
}

extern "C" int rt_hip_accel_info(const rt_hip_ctx* c, rt_accel_info* out) {
  if (!c || !out) return rt_set_error(RT_EINVAL, "null argument");
  *out = c->info;
  return RT_OK;
}

extern "C" int rt_hip_accel_validate(const rt_hip_ctx* c) {
  if (!c) return rt_set_error(RT_EINVAL, "null context");
  HIP_TRY(hipSetDevice(c->device));
  rt_flat_scene f;
  std::memset(&f, 0, sizeof f);
  f.ntri = c->info.triangles;
  f.nrec = c->nrec;
  f.nnode = c->d_node ? c->info.nodes : 0;
  for (int a = 0; a < 3; a++) {
    f.scene_lo[a] = c->scene_c[a] - c->scene_r;
    f.scene_hi[a] = c->scene_c[a] + c->scene_r;
  }
  std::vector<float> tri(f.nrec * RT_TRI_FLOATS + 1), node(f.nnode * RT_NODE_FLOATS + 1);
  if (f.nrec)
    HIP_TRY(hipMemcpy(tri.data(), c->d_tri, f.nrec * RT_TRI_FLOATS * sizeof(float),
                      hipMemcpyDeviceToHost));
  if (f.nnode)
    HIP_TRY(hipMemcpy(node.data(), c->d_node, f.nnode * RT_NODE_FLOATS * sizeof(float),
                      hipMemcpyDeviceToHost));
  f.tri = tri.data();
  f.node = node.data();
  return rt_flat_validate(&f);
}

extern "C" int rt_hip_set_cull_slack(rt_hip_ctx* c, float ulps) {
  if (!c || !(ulps >= 0.0f)) return rt_set_error(RT_EINVAL, "bad slack");
  c->eps_ulps = ulps;
  c->cam_eps_ulps = ulps;
  c->known.valid = c->pknown.valid = c->kept_for.valid = 0;  // the lists change
  return RT_OK;
}

extern "C" int rt_hip_set_camera_slack(rt_hip_ctx* c, float ulps) {
  if (!c || !(ulps >= 0.0f)) return rt_set_error(RT_EINVAL, "bad slack");
  c->cam_eps_ulps = ulps;
  c->known.valid = c->pknown.valid = c->kept_for.valid = 0;  // the lists change
  return RT_OK;
}

extern "C" int rt_hip_set_exact_camera(rt_hip_ctx* c, int enable) {
  if (!c) return rt_set_error(RT_EINVAL, "null context");
  c->exact_camera = enable ? 1 : 0;
  return RT_OK;
}

extern "C" int rt_hip_set_exact_shadows(rt_hip_ctx* c, int enable) {
  if (!c) return rt_set_error(RT_EINVAL, "null context");
  c->exact_shadows = enable ? 1 : 0;
  // built now (setup), reported by rt_hip_accel_info: the light buffers in
  // the matching mode, and the walk's multipliers (policies that walk)
  HIP_TRY(hipSetDevice(c->device));
  int rc = lbuf_prepare(c, c->stream);
  if (rc) return rc;
  if (c->exact_shadows) return shadow_prepare(c, c->stream);
  return RT_OK;
}

// The exact reflection walk's per-node bounds (csrc/rt_reflect.hip): once
// per tree, synchronous (setup).
static int reflect_prepare(rt_hip_ctx* c, hipStream_t s) {
  if (c->d_node_rf || c->accel != RT_ACCEL_OCTREE || !c->d_node) return RT_OK;
  const size_t nn = c->info.nodes;
  float* phi = nullptr;
  uint32_t* d_u = nullptr;
  HIP_TRY(hipMalloc((void**)&c->d_node_rf, (3 * nn + 3) * sizeof(float4)));
  hipError_t he = hipMalloc((void**)&phi, (nn + 1) * sizeof(float));
  if (he == hipSuccess) he = hipMalloc((void**)&d_u, sizeof(uint32_t));
  ReflParams rp;
  std::memset(&rp, 0, sizeof rp);
  rp.node = c->d_node;
  rp.nnode = (uint32_t)nn;
  rp.rec = c->d_tri;
  rp.node_rf = c->d_node_rf;
  rp.node_phi = phi;
  rp.unbounded = d_u;
  uint32_t u = 0;
  if (he == hipSuccess) he = hipMemsetAsync(c->d_node_rf, 0, (3 * nn + 3) * sizeof(float4), s);
  if (he == hipSuccess) he = hipMemsetAsync(d_u, 0, sizeof(uint32_t), s);
  if (he == hipSuccess) he = rt_reflect_build(&rp, (int)c->info.max_depth + 2, s);
  if (he == hipSuccess) he = hipMemcpyAsync(&u, d_u, sizeof u, hipMemcpyDeviceToHost, s);
  if (he == hipSuccess) he = hipStreamSynchronize(s);
  (void)hipFree(phi);
  (void)hipFree(d_u);
  if (he != hipSuccess) {
    (void)hipFree(c->d_node_rf);
    c->d_node_rf = nullptr;
    return rt_set_error(RT_EHIP, "reflection bounds: %s", hipGetErrorString(he));
  }
  c->rf_unbounded = u;
  return RT_OK;
}

extern "C" int rt_hip_set_exact_reflections(rt_hip_ctx* c, int enable) {
  if (!c) return rt_set_error(RT_EINVAL, "null context");
  c->exact_refl = enable ? 1 : 0;
  if (!c->exact_refl) return RT_OK;
  HIP_TRY(hipSetDevice(c->device));
  return reflect_prepare(c, c->stream);
}

extern "C" int rt_hip_set_policy(rt_hip_ctx* c, int policy) {
  if (!c) return rt_set_error(RT_EINVAL, "null context");
  if (policy < RT_POLICY_DEFAULT || policy > RT_POLICY_DIR_STAGED)
    return rt_set_error(RT_EINVAL, "unknown traversal policy %d", policy);
  c->policy = policy;
  return RT_OK;
}

extern "C" int rt_hip_set_camera_refine(rt_hip_ctx* c, int enable) {
  if (!c) return rt_set_error(RT_EINVAL, "null context");
  c->cand_refine = enable ? 1 : 0;
  c->known.valid = c->pknown.valid = c->kept_for.valid = 0;  // the lists change
  return RT_OK;
}

extern "C" int rt_hip_set_camera_bound_scale(rt_hip_ctx* c, double scale) {
  if (!c || !(scale > 0.0)) return rt_set_error(RT_EINVAL, "bad bound scale");
  c->bound_scale = scale;
  c->known.valid = c->pknown.valid = c->kept_for.valid = 0;  // the lists change
  return RT_OK;
}

extern "C" int rt_cand_refine_sample(const rt_scene* scene, float eps_ulps, double bound_scale, unsigned stride,
                                     int compat, unsigned* out, size_t cap, size_t* n, size_t* total) {
  if (!scene || (!out && cap) || !n || !total) return rt_set_error(RT_EINVAL, "null argument");
  rt_frame f;
  rt_camera cam = scene->camera;
  if (compat) {  // gpu/rt's frame: the camera's width and height times 3 (gpu/rt.cpp:72-83)
    cam.width *= 3;
    cam.height *= 3;
  }
  int rc = compat ? rt_frame_from_camera_any(&cam, &f) : rt_frame_from_camera(&cam, &f);
  if (rc) return rc;
  rt_flat_scene fs;
  rc = rt_flatten(scene, RT_ACCEL_FLAT, &fs);
  if (rc) return rc;
  float sc[3], sr = 0;
  for (int a = 0; a < 3; a++) {  // as rt_hip_create
    float lo = fs.ntri ? fs.scene_lo[a] : 0.0f, hi = fs.ntri ? fs.scene_hi[a] : 0.0f;
    sc[a] = 0.5f * (lo + hi);
    sr = std::fmax(sr, 0.5f * (hi - lo));
  }
  CandParams cp;
  rc = cand_params(&f, sc, sr, eps_ulps, bound_scale, 0, 1, &cp, compat ? 1 : 0);
  if (!rc) {
    cp.nprim = (uint32_t)fs.ntri;
    *n = rt_cand_refine_sample_host(&cp, fs.tri, stride, out, cap, total);
  }
  rt_flat_free(&fs);
  return rc;
}

extern "C" int rt_cand_survey(const rt_scene* scene, float eps_ulps, double bound_scale, int threads,
                              int use_leaves, unsigned long long out[88]) {
  if (!scene || !out) return rt_set_error(RT_EINVAL, "null argument");
  rt_frame f;
  int rc = rt_frame_from_camera(&scene->camera, &f);
  if (rc) return rc;
  rt_flat_scene fs;
  rc = rt_flatten(scene, RT_ACCEL_FLAT, &fs);
  if (rc) return rc;
  float sc[3], sr = 0;
  for (int a = 0; a < 3; a++) {  // as rt_hip_create
    float lo = fs.ntri ? fs.scene_lo[a] : 0.0f, hi = fs.ntri ? fs.scene_hi[a] : 0.0f;
    sc[a] = 0.5f * (lo + hi);
    sr = std::fmax(sr, 0.5f * (hi - lo));
  }
  CandParams cp;
  rc = cand_params(&f, sc, sr, eps_ulps, bound_scale, 0, 1, &cp);
  rt_flat_scene ft;  // the host octree's leaves (use_leaves)
  std::memset(&ft, 0, sizeof ft);
  std::vector<uint32_t> pl;
  if (!rc && use_leaves) {
    rc = rt_flatten(scene, RT_ACCEL_OCTREE, &ft);
    if (!rc) {
      pl.assign(fs.ntri + 1, 0);
      for (size_t ni = 0; ni < ft.nnode; ni++) {
        uint32_t first, info;
        std::memcpy(&first, &ft.node[RT_NODE_FLOATS * ni + 3], 4);
        std::memcpy(&info, &ft.node[RT_NODE_FLOATS * ni + 7], 4);
        if (!(info & RT_NODE_LEAF)) continue;
        for (uint32_t k = 0; k < RT_LEAF_COUNT(info); k++) {
          uint32_t prim;
          std::memcpy(&prim, &ft.tri[RT_TRI_FLOATS * (size_t)(first + k) + 9], 4);
          pl[prim] = (uint32_t)ni;
        }
      }
    }
  }
  if (!rc) {
    cp.nprim = (uint32_t)fs.ntri;
    if (rt_cand_survey_host(&cp, fs.tri, use_leaves ? ft.node : nullptr,
                            use_leaves ? pl.data() : nullptr, threads, out))
      rc = rt_set_error(RT_EINVAL, "candidate survey: per-row tile count != rasterised tiles");
  }
  if (use_leaves) rt_flat_free(&ft);
  rt_flat_free(&fs);
  return rc;
}

static int cand_prepare(rt_hip_ctx* c, const rt_frame* f, KParams* kp, hipStream_t s, int compat = 0);

static int cand_verify(rt_hip_ctx* c, const rt_frame* f, KParams kp, int compat, unsigned long long out[7]);

extern "C" int rt_hip_cand_verify(rt_hip_ctx* c, const rt_frame* f, int rank, int nranks,
                                  unsigned long long out[7]) {
  if (!c || !f || !out) return rt_set_error(RT_EINVAL, "null argument");
  if (!c->d_cand_start || !c->d_cand || !c->d_cand_list)
    return rt_set_error(RT_EINVAL, "no candidate lists (render a frame with exact camera rays first)");
  if (c->last_p.rank != rank || c->last_p.nranks != nranks)
    return rt_set_error(RT_EINVAL, "the last render was rank %d of %d", c->last_p.rank, c->last_p.nranks);
  return cand_verify(c, f, c->last_p, 0, out);
}

// The same for the compatibility mode's lists (rt_hip_render_compat): the
// camera's 3x frame, one sample per pixel (CandParams::compat), one rank.
extern "C" int rt_hip_cand_verify_compat(rt_hip_ctx* c, const rt_camera* cam, unsigned long long out[7]) {
  if (!c || !cam || !out) return rt_set_error(RT_EINVAL, "null argument");
  if (!c->d_cand_start || !c->d_cand || !c->d_cand_list)
    return rt_set_error(RT_EINVAL, "no candidate lists (render a frame with exact camera rays first)");
  rt_camera big = *cam;
  big.width = 3 * cam->width;
  big.height = 3 * cam->height;
  rt_frame f;
  int rc = rt_frame_from_camera_any(&big, &f);
  if (rc) return rc;
  KParams kp;
  std::memset(&kp, 0, sizeof kp);
  kp.rank = 0;
  kp.nranks = 1;
  kp.ntiles_local = tiles_x_of(big.width) * tiles_y_of(big.height);
  return cand_verify(c, &f, kp, 1, out);
}

static int cand_verify(rt_hip_ctx* c, const rt_frame* f, KParams kp, int compat, unsigned long long out[7]) {
  const int rank = kp.rank, nranks = kp.nranks;
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = c->last_stream ? c->last_stream : c->stream;
  HIP_TRY(hipStreamSynchronize(s));
  // the render keeps only the big footprints: build the frame's lists again
  // (deterministic: the same entries at the same places) keeping every one
  {
    c->cand_store_fp = 1;
    const int rp = cand_prepare(c, f, &kp, s, compat);
    c->cand_store_fp = 0;
    if (rp) return rp;
    HIP_TRY(hipStreamSynchronize(s));
  }
  CandParams cp;
  int rc = cand_params(f, c->scene_c, c->scene_r, c->cam_eps_ulps, c->bound_scale, rank, nranks, &cp, compat);
  if (rc) return rc;
  cp.nprim = c->nprim;
  const uint32_t nt = (uint32_t)cp.ntiles_local;
  cp.refine = c->cand_refine ? 1u : 0u;
  cp.drop_key = nt;
  uint32_t ctr[4];
  HIP_TRY(hipMemcpy(ctr, c->d_cand_ctr, sizeof ctr, hipMemcpyDeviceToHost));
  const uint32_t nlist = ctr[3];
  std::vector<uint32_t> start(nt + 1), list(nlist + 1), pl;
  HIP_TRY(hipMemcpy(start.data(), c->d_cand_start, (nt + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost));
  std::vector<uint32_t> cand(start[nt] + 1);
  if (start[nt])
    HIP_TRY(hipMemcpy(cand.data(), c->d_cand, start[nt] * sizeof(uint32_t), hipMemcpyDeviceToHost));
  if (nlist) HIP_TRY(hipMemcpy(list.data(), c->d_cand_list, nlist * sizeof(uint32_t), hipMemcpyDeviceToHost));
  const size_t fpb = rt_cand_footprint_bytes();
  std::vector<unsigned char> fp((size_t)nlist * fpb + 1);
  if (nlist) HIP_TRY(hipMemcpy(fp.data(), c->d_cand_fp, (size_t)nlist * fpb, hipMemcpyDeviceToHost));
  std::vector<float> tri((size_t)c->nprim * RT_TRI_FLOATS + 1), node;
  HIP_TRY(hipMemcpy(tri.data(), c->d_tri_prim, (size_t)c->nprim * RT_TRI_FLOATS * sizeof(float),
                    hipMemcpyDeviceToHost));
  if (c->d_prim_leaf) {
    pl.resize(c->nprim + 1);
    HIP_TRY(hipMemcpy(pl.data(), c->d_prim_leaf, c->nprim * sizeof(uint32_t), hipMemcpyDeviceToHost));
    node.resize((size_t)c->info.nodes * RT_NODE_FLOATS + 1);
    HIP_TRY(hipMemcpy(node.data(), c->d_node, (size_t)c->info.nodes * RT_NODE_FLOATS * sizeof(float),
                      hipMemcpyDeviceToHost));
  }
  rt_cand_verify_host(&cp, tri.data(), c->d_prim_leaf ? node.data() : nullptr,
                      c->d_prim_leaf ? pl.data() : nullptr, list.data(), nlist, fp.data(),
                      start.data(), cand.data(), nt, out);
  return RT_OK;
}

extern "C" int rt_hip_cand_tile_entries(rt_hip_ctx* c, unsigned int* out, size_t n) {
  if (!c || !out) return rt_set_error(RT_EINVAL, "null argument");
  if (!c->d_cand_start) return rt_set_error(RT_EINVAL, "no candidate lists (render a frame first)");
  if (n > (size_t)c->last_p.ntiles_local)
    return rt_set_error(RT_EINVAL, "%zu tiles asked, the last render had %d", n, c->last_p.ntiles_local);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = c->last_stream ? c->last_stream : c->stream;
  HIP_TRY(hipStreamSynchronize(s));
  std::vector<uint32_t> st(n + 1);
  HIP_TRY(hipMemcpy(st.data(), c->d_cand_start, (n + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost));
  for (size_t t = 0; t < n; t++) out[t] = st[t + 1] - st[t];
  return RT_OK;
}

extern "C" int rt_hip_set_timing(rt_hip_ctx* c, int enable) {
  if (!c) return rt_set_error(RT_EINVAL, "null context");
  HIP_TRY(hipSetDevice(c->device));
  for (auto& f : c->ev)
    for (hipEvent_t& e : f)
      if (!e) HIP_TRY(hipEventCreate(&e));
  c->timing = enable ? 1 : 0;
  c->frames = 0;
  return RT_OK;
}

extern "C" int rt_hip_frame_times(rt_hip_ctx* c, int n, float* lists_ms, float* render_ms) {
  if (!c || !lists_ms || !render_ms) return rt_set_error(RT_EINVAL, "null argument");
  if (n <= 0 || n > RT_TIMED_FRAMES || (unsigned long long)n > c->frames)
    return rt_set_error(RT_EINVAL, "%d timed frames asked, %llu recorded (ring of %d)", n,
                        c->frames, RT_TIMED_FRAMES);
  HIP_TRY(hipSetDevice(c->device));
  for (int i = 0; i < n; i++) {
    hipEvent_t* e = c->ev[(c->frames - (unsigned long long)n + (unsigned long long)i) % RT_TIMED_FRAMES];
    HIP_TRY(hipEventSynchronize(e[4]));
    HIP_TRY(hipEventElapsedTime(lists_ms + i, e[0], e[1]));
    HIP_TRY(hipEventElapsedTime(render_ms + i, e[1], e[4]));
  }
  return RT_OK;
}

extern "C" int rt_hip_frame_kernel_times(rt_hip_ctx* c, int n, float* trace_ms, float* shade_ms,
                                         float* fold_ms) {
  if (!c || !trace_ms || !shade_ms || !fold_ms) return rt_set_error(RT_EINVAL, "null argument");
  if (n <= 0 || n > RT_TIMED_FRAMES || (unsigned long long)n > c->frames)
    return rt_set_error(RT_EINVAL, "%d timed frames asked, %llu recorded (ring of %d)", n,
                        c->frames, RT_TIMED_FRAMES);
  HIP_TRY(hipSetDevice(c->device));
  for (int i = 0; i < n; i++) {
    hipEvent_t* e = c->ev[(c->frames - (unsigned long long)n + (unsigned long long)i) % RT_TIMED_FRAMES];
    HIP_TRY(hipEventSynchronize(e[4]));
    HIP_TRY(hipEventElapsedTime(trace_ms + i, e[1], e[2]));
    HIP_TRY(hipEventElapsedTime(shade_ms + i, e[2], e[3]));
    HIP_TRY(hipEventElapsedTime(fold_ms + i, e[3], e[4]));
  }
  return RT_OK;
}

extern "C" int rt_hip_tile_cycles(rt_hip_ctx* c, unsigned long long* out, size_t n) {
  if (!c || !out) return rt_set_error(RT_EINVAL, "null argument");
  if (!c->d_tile_cycles || n > c->tile_cycles_n)
    return rt_set_error(RT_EINVAL, "%zu tile clocks asked, %zu recorded (rt_hip_set_count_work)", n,
                        c->tile_cycles_n);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = c->last_stream ? c->last_stream : c->stream;
  HIP_TRY(hipStreamSynchronize(s));
  HIP_TRY(hipMemcpy(out, c->d_tile_cycles, n * sizeof *out, hipMemcpyDeviceToHost));
  return RT_OK;
}

extern "C" int rt_hip_tile_phase_cycles(rt_hip_ctx* c, int phase, unsigned long long* out, size_t n) {
  if (!c || !out || phase < 0 || phase > 5) return rt_set_error(RT_EINVAL, "bad argument");
  if (!c->d_tile_cycles || n > c->tile_cycles_n)
    return rt_set_error(RT_EINVAL, "%zu item clocks asked, %zu recorded (rt_hip_set_count_work)", n,
                        c->tile_cycles_n);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = c->last_stream ? c->last_stream : c->stream;
  HIP_TRY(hipStreamSynchronize(s));
  HIP_TRY(hipMemcpy(out, c->d_tile_cycles + (size_t)phase * c->tile_cycles_n, n * sizeof *out,
                    hipMemcpyDeviceToHost));
  return RT_OK;
}

extern "C" int rt_hip_set_count_work(rt_hip_ctx* c, int enable) {
  if (!c) return rt_set_error(RT_EINVAL, "null context");
  c->count_work = enable ? 1 : 0;
  return RT_OK;
}

// ---------------------------------------------------- exact camera rays
// Frame constants of the candidate lists (csrc/rt_cand.hip) and the three
// launches: count -> scan -> (one small read-back for the list sizes) ->
// fill.  Everything is derived from the frame in double, rounded so that
// each bound stays conservative.
template <class T>
static int grow_dev(T** p, size_t* cap, size_t need) {
  if (need <= *cap && *p) return RT_OK;
  (void)hipFree(*p);
  *p = nullptr;
  size_t n = need + need / 4 + 64;
  HIP_TRY(hipMalloc((void**)p, n * sizeof(T)));
  *cap = n;
  return RT_OK;
}

static double d3dot(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// big footprints whose per-lane row counts big_count_kernel keeps for
// big_kernel (C5: ~5e4 per frame; beyond this big_kernel recounts)
static constexpr uint32_t kBigLaneCap = 1u << 17;
// (big footprint, chunk) work items of the entry-parallel big emission (C5:
// ~5e4 per frame; beyond this the frame's big footprints go to big_kernel)
#ifndef RT_CAND_ITEM_CAP
#define RT_CAND_ITEM_CAP (1u << 20)
#endif
static constexpr uint32_t kItemCap = RT_CAND_ITEM_CAP;
// the lists' two prim-length scans: the device-length scan of rt_cand.hip
// (1; the classification's over the listed prims only, no zeroing pass) or
// rocPRIM's over every prim (0)
#ifndef RT_DEV_SCAN
#define RT_DEV_SCAN 1
#endif

extern "C" int rt_hip_set_cand_item_cap(rt_hip_ctx* c, unsigned cap) {
  if (!c) return rt_set_error(RT_EINVAL, "null context");
  c->cand_item_cap = cap;
  c->known.valid = c->pknown.valid = c->kept_for.valid = 0;  // the lists change
  return RT_OK;
}

// the trace's item-clock sum in the frame counters (KParams::cost_sum)
static unsigned long long* cost_sum_of(rt_hip_ctx* c) {
  return (unsigned long long*)((char*)c->d_counter + kItemCounterBytes + kStatBytes + kHitCounterBytes);
}

// Frame constants of the candidate lists for rank/nranks (no device work).
static int cand_params(const rt_frame* f, const float scene_c[3], float scene_r, float eps_ulps,
                       double bound_scale, int rank, int nranks, CandParams* out, int compat) {
  const double eps = 0x1p-24;
  CandParams& cp = *out;
  std::memset(&cp, 0, sizeof cp);
  const double pos[3] = {f->position.x, f->position.y, f->position.z};
  const double u[3] = {f->u.x, f->u.y, f->u.z}, v[3] = {f->v.x, f->v.y, f->v.z};
  const double C[3] = {f->C.x, f->C.y, f->C.z};
  double n[3] = {u[1] * v[2] - u[2] * v[1], u[2] * v[0] - u[0] * v[2], u[0] * v[1] - u[1] * v[0]};
  const double nn = std::sqrt(d3dot(n, n));
  if (!(nn > 1e-6)) return rt_set_error(RT_EINVAL, "degenerate camera (u parallel to v)");
  for (int a = 0; a < 3; a++) {
    cp.pos[a] = pos[a];
    cp.u[a] = u[a];
    cp.v[a] = v[a];
    cp.C[a] = C[a];
    cp.n[a] = n[a] / nn;
  }
  const double cpos[3] = {C[0] - pos[0], C[1] - pos[1], C[2] - pos[2]};
  cp.plane = d3dot(cpos, cp.n);
  if (!(std::fabs(cp.plane) > 1e-6)) return rt_set_error(RT_EINVAL, "degenerate camera (L = 0)");
  const double g00 = d3dot(u, u), g01 = d3dot(u, v), g11 = d3dot(v, v);
  const double det = g00 * g11 - g01 * g01;
  cp.ginv[0] = g11 / det;
  cp.ginv[1] = -g01 / det;
  cp.ginv[2] = g00 / det;
  cp.gscale = std::sqrt(cp.ginv[0] * cp.ginv[0] + 2 * cp.ginv[1] * cp.ginv[1] + cp.ginv[2] * cp.ginv[2]);
  {
    const double pc[3] = {-cpos[0], -cpos[1], -cpos[2]};
    const double pu = d3dot(pc, u), pv = d3dot(pc, v);
    cp.k0 = cp.ginv[0] * pu + cp.ginv[1] * pv;
    cp.l0 = cp.ginv[1] * pu + cp.ginv[2] * pv;
  }
  // a tile's sample rectangle (rt_cand.hip tile_keep): cpu/rt's samples k in
  // [W/2 - c, W/2 - c + 1/2] for the tile's columns c = 8 tx .. 8 tx + 7, so
  // centre W/2 - 8 tx - 3.25 and half side 3.75 (likewise l); compatibility
  // mode: k = c - W/2, centre 8 tx + 3.5 - W/2, half side 3.5
  {
    const double hw = (double)(f->width / 2), hh = (double)(f->height / 2);
    cp.tile_hk = cp.tile_hl = compat ? 3.5 : 3.75;
    cp.tile_k00 = compat ? 3.5 - hw : hw - 3.25;
    cp.tile_l00 = compat ? 3.5 - hh : hh - 3.25;
    cp.tile_dk = cp.tile_dl = compat ? 8.0 : -8.0;
    for (int a = 0; a < 3; a++) {
      cp.tile_p00[a] = pos[a] - (C[a] + cp.tile_k00 * u[a] + cp.tile_l00 * v[a]);
      cp.tile_du[a] = cp.tile_dk * u[a];
      cp.tile_dv[a] = cp.tile_dl * v[a];
      cp.tile_w[a] = std::fabs(u[a]) * cp.tile_hk + std::fabs(v[a]) * cp.tile_hl;
    }
    cp.tile_hd = (cp.tile_hk * std::sqrt(d3dot(u, u)) + cp.tile_hl * std::sqrt(d3dot(v, v))) * (1.0 + 1e-12);
  }
  const int W = f->width, H = f->height;
  cp.compat = compat;
  if (compat) {
    // gpu/rt: one sample per pixel of the 3x frame, k = px - W/2, px in
    // [0, W - 1] (gpu/raytracer.cu:97-103), likewise l
    cp.kmin = -(double)(W / 2);
    cp.kmax = (double)(W - 1 - W / 2);
    cp.lmin = -(double)(H / 2);
    cp.lmax_ = (double)(H - 1 - H / 2);
  } else {
    // samples: k = i + {0, 1/2}, i in [1 - W/2, W/2] (cpu/raytracer.c:50-58)
    cp.kmin = 1.0 - W / 2;
    cp.kmax = W / 2 + 0.5;
    cp.lmin = 1.0 - H / 2;
    cp.lmax_ = H / 2 + 0.5;
  }
  double lmax = 0, omax = 0;
  for (int ci = 0; ci < 4; ci++) {  // |o - pos| and |o| are convex: corners bound them
    const double k = (ci & 1) ? cp.kmax : cp.kmin, l = (ci & 2) ? cp.lmax_ : cp.lmin;
    double o[3], d[3];
    for (int a = 0; a < 3; a++) {
      o[a] = C[a] + u[a] * k + v[a] * l;
      d[a] = o[a] - pos[a];
    }
    lmax = std::fmax(lmax, std::sqrt(d3dot(d, d)));
    omax = std::fmax(omax, std::sqrt(d3dot(o, o)));
  }
  cp.lmax = lmax * (1 + 1e-9) + 1e-9;
  cp.omax = omax * (1 + 1e-9) + 1e-9;
  // float camera line (o_f, normalize(pos - o_f)): within 2.5 eps rad of the
  // direction towards pos, so within dline of pos; o_f within dorig of o
  cp.dline = 6.0 * eps * cp.lmax + 1e-12;
  cp.dorig = 8.0 * eps * (std::sqrt(d3dot(C, C)) + std::fabs(cp.kmin) + cp.kmax + std::fabs(cp.lmin) +
                          cp.lmax_) * 1.8;
  // smallest culling slack of a camera ray: rt_cull_eps with the max-norm
  // |o - c| bounded below per axis over the sample rectangle
  double mlb = 0;
  for (int a = 0; a < 3; a++) {
    double lo = 1e300, hi = -1e300;
    for (int ci = 0; ci < 4; ci++) {
      const double k = (ci & 1) ? cp.kmax : cp.kmin, l = (ci & 2) ? cp.lmax_ : cp.lmin;
      const double x = C[a] + u[a] * k + v[a] * l - scene_c[a];
      lo = std::fmin(lo, x);
      hi = std::fmax(hi, x);
    }
    const double m = (lo <= 0 && hi >= 0) ? 0.0 : std::fmin(std::fabs(lo), std::fabs(hi));
    mlb = std::fmax(mlb, m);
  }
  const double R = scene_r;
  const double cmag = std::fmax(std::fabs(scene_c[0]), std::fmax(std::fabs(scene_c[1]),
                                                                std::fabs(scene_c[2])));
  const double eps_rel = (double)(eps_ulps * 5.9604645e-8f);
  const double eps_min = (eps_rel * (std::fmax(mlb - cp.dorig, 0.0) + R) +
                          (double)RT_CULL_PLANE * (cmag + R) + 1e-6) * (1.0 - 1e-5);
  // the slab test's own rounding (rt_cull.h: a few ulps of |o| and of |t d|)
  // takes 4 ulps of |o| + the scene's extent out of that slack
  cp.eps_avail = eps_min - 8.0 * eps * (cp.omax + 2.0 * (cmag + R));
  // tools/mt_bound.py: C_DOT = 6 sqrt 2 -> 8.6, C_A = 5 sqrt 2 -> 7.2 (scale 1 = the proven bound)
  cp.c_dot = 8.6 * bound_scale;
  cp.c_a = 7.2 * bound_scale;
  cp.W = W;
  cp.H = H;
  cp.tiles_x = tiles_x_of(W);
  cp.tiles_y = tiles_y_of(H);
  cp.rank = rank;
  cp.nranks = nranks;
  cp.tb = rt_block_side(nranks);
  cp.blocks_x = rt_blocks_x(cp.tiles_x, cp.tb);
  cp.ntiles_local = rank_tile_count(W, H, rank, nranks);
  return RT_OK;
}

static int ensure_tmp(rt_hip_ctx* c, size_t bytes) {
  // never null once ensured: rt_cand_scan takes a null temp for a size query,
  // also on its one-workgroup path, which needs none
  if (bytes < 256) bytes = 256;
  if (bytes <= c->scan_tmp_bytes && c->d_scan_tmp) return RT_OK;
  (void)hipFree(c->d_scan_tmp);
  c->d_scan_tmp = nullptr;
  HIP_TRY(hipMalloc(&c->d_scan_tmp, bytes));
  c->scan_tmp_bytes = bytes;
  return RT_OK;
}

// The last render's kept-entry count (rt_hip_stats reads it) outlives a list
// build that overwrites the offsets it points into: saved in stream order to
// a word no build writes (d_cand_ctr[8]).
static int save_valid(rt_hip_ctx* c, hipStream_t s) {
  if (!c->d_cand_valid || !c->d_cand_ctr || c->d_cand_valid == c->d_cand_ctr + 8) return RT_OK;
  HIP_TRY(hipMemcpyAsync(c->d_cand_ctr + 8, c->d_cand_valid, sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  c->d_cand_valid = c->d_cand_ctr + 8;
  return RT_OK;
}

// The entry buffers (keys, vals, keys2, cand) for n entries.
static int cand_entry_buffers(rt_hip_ctx* c, size_t n) {
  if (n + 1 <= c->cand_cap) return RT_OK;
  c->ext_ready = 0;  // consumed lists (ext) point into these
  for (uint32_t** b : {&c->d_cand_keys, &c->d_cand_vals, &c->d_cand_keys2, &c->d_cand}) {
    (void)hipFree(*b);
    *b = nullptr;
  }
  c->cand_cap = 0;  // set only once all four entry buffers exist
  size_t cap = 0;
  int rc = grow_dev(&c->d_cand_keys, &cap, n + 1);
  if (rc) return rc;
  for (uint32_t** b : {&c->d_cand_vals, &c->d_cand_keys2, &c->d_cand})
    HIP_TRY(hipMalloc((void**)b, cap * sizeof(uint32_t)));
  c->cand_cap = cap;
  return RT_OK;
}

// The per-tile offsets and work-order buffers for nt tiles.
static int cand_tile_buffers(rt_hip_ctx* c, size_t nt) {
  if (nt + 1 > c->cand_tiles_cap || nt + 1 > c->order_cap) {
    c->ext_ready = 0;  // the consumed lists' offsets and work order live here
    if (c->d_cand_valid && c->d_cand_valid != c->d_cand_ctr + 8) c->d_cand_valid = nullptr;
  }
  if (nt + 1 > c->cand_tiles_cap) {
    size_t cap = c->cand_tiles_cap;
    int rc = grow_dev(&c->d_cand_start, &cap, nt + 1);
    if (rc) return rc;
    c->cand_tiles_cap = cap;
  }
  if (nt + 1 > c->order_cap) {
    (void)hipFree(c->d_order);
    c->d_order = nullptr;
    c->order_cap = 0;
    HIP_TRY(hipMalloc((void**)&c->d_order, 3 * (nt + 1) * sizeof(uint32_t)));
    c->order_cap = nt + 1;
  }
  return RT_OK;
}

// The longest-first work order of the nt tiles from their offsets, and the
// lists' kernel parameters common to both builds.
static int cand_order(rt_hip_ctx* c, KParams* kp, size_t nt, uint32_t total, hipStream_t s, const rt_frame* f,
                      int rank, int nranks) {
  size_t tb = 0;
  // the item clocks of this frame's last trace on this context (its counters
  // are zeroed only by the render that follows this order)
  // -- or of the last frame of the same size and rank split: a new camera
  // (an animation's next frame) moves the costly tiles little, and the order
  // is a schedule only (any order renders the same image)
  const bool hist = c->cost_hist.same_grid(f, rank, nranks) && c->d_item_cost && c->item_cost_cap >= 4 * nt;
  const uint32_t* ic = hist ? c->d_item_cost : nullptr;
  const unsigned long long* cs = hist ? cost_sum_of(c) : nullptr;
  HIP_TRY(rt_cand_order(c->d_cand_start, (uint32_t)nt, total, c->d_order, c->d_order + nt + 1,
                        c->d_order + 2 * (nt + 1), ic, cs, c->cost_waves, nullptr, &tb, s));
  int rc = ensure_tmp(c, tb);
  if (rc) return rc;
  tb = c->scan_tmp_bytes;
  HIP_TRY(rt_cand_order(c->d_cand_start, (uint32_t)nt, total, c->d_order, c->d_order + nt + 1,
                        c->d_order + 2 * (nt + 1), ic, cs, c->cost_waves, c->d_scan_tmp, &tb, s));
  kp->tile_order = c->d_order + 2 * (nt + 1);
  kp->n_heavy = c->d_order + (nt + 1) + nt;  // the scan of the heavy flags: its total
  kp->cand_start = c->d_cand_start;
  kp->tri_prim = c->d_tri_prim;
  return RT_OK;
}

// Radix sort bits of keys below n_keys.
static int key_bits(size_t n_keys) {
  int bits = 1;
  while ((1ull << bits) < n_keys) bits++;
  return bits;
}

// Passes 0-2 of the lists of cp (the prims [cp.prim0, cp.prim1)): the
// unsorted (tile, prim) entries in d_cand_keys / d_cand_vals, each listed
// prim's depth-skip bound in d_cand_skip and the global prims in
// d_cand_global; count -> scan -> (read back the entry total: the build's
// only host sync) -> emit.  The entry buffers are sized for total +
// glob_copies x globals (the triangle-parallel build routes each global to
// every rank).  No contended atomics; deterministic.
// Entries per big emission item for a build of 1/split of a frame's work (a
// rank's lists of an N-rank frame, a producer's slice of N): 1024 for a whole
// frame, halved per doubling of split down to 128, so the items stay many
// enough to overlap (rt_cand.hip).  RT_CAND_CHUNK_SHIFT: A/B knob.
static uint32_t cand_chunk_shift(uint32_t split) {
  if (const char* e = std::getenv("RT_CAND_CHUNK_SHIFT")) {
    const int v = std::atoi(e);
    if (v >= 6 && v <= 14) return (uint32_t)v;
  }
  uint32_t sh = 10;
  for (uint32_t q = split; q > 1 && sh > 7; q >>= 1) sh--;
  return sh;
}

static int cand_build(rt_hip_ctx* c, CandParams& cp, hipStream_t s, uint32_t glob_copies, uint32_t* total_out,
                      uint32_t* nglobal_out, const ListShape* known = nullptr, ListShape* shape = nullptr) {
  int rc = RT_OK;
  // every build overwrites the entry, offset and order buffers: lists that
  // rt_hip_cand_consume left for a render (ext) are gone from here on, so
  // that render builds its own (produce -> consume -> produce ->
  // render must not render from clobbered buffers)
  c->ext_ready = 0;
  rc = save_valid(c, s);
  if (rc) return rc;
  cp.tri = c->d_tri_prim;
  cp.nprim = c->nprim;
  const size_t np = c->nprim;
  if (!c->d_prim_leaf && c->d_node) {  // once per scene: which leaf holds each prim
    HIP_TRY(hipMalloc((void**)&c->d_prim_leaf, (np + 1) * sizeof(uint32_t)));
    HIP_TRY(hipMemsetAsync(c->d_prim_leaf, 0xff, (np + 1) * sizeof(uint32_t), s));  // atomicMin's start
    HIP_TRY(rt_cand_prim_leaf(c->d_node, (uint32_t)c->info.nodes, c->d_tri, c->d_prim_leaf, s));
  }
  cp.node = c->d_node;
  cp.prim_leaf = c->d_prim_leaf;
  if (!c->h_cand) {
    // h_cand is allocated last: a partial set left by an earlier failure is
    // freed here, never allocated over
    for (void** b : {(void**)&c->d_cand_list, &c->d_cand_fp, (void**)&c->d_cand_sfp, (void**)&c->d_cand_visits,
                     (void**)&c->d_cand_off,
                     (void**)&c->d_cand_global, (void**)&c->d_cand_big, (void**)&c->d_cand_ctr,
                     (void**)&c->d_cand_skip, (void**)&c->d_cand_big_lane, (void**)&c->d_cand_items,
                     (void**)&c->d_cand_wave_items, (void**)&c->d_cand_wave_base, (void**)&c->d_scan_bsum}) {
      (void)hipFree(*b);
      *b = nullptr;
    }
    HIP_TRY(hipMalloc((void**)&c->d_cand_list, (np + 1) * sizeof(uint32_t)));
    HIP_TRY(hipMalloc(&c->d_cand_fp, (np + 1) * rt_cand_footprint_bytes()));
    HIP_TRY(hipMalloc((void**)&c->d_cand_sfp, 2 * (np + 1) * sizeof(uint4)));
    HIP_TRY(hipMalloc((void**)&c->d_cand_visits, (np + 1) * sizeof(uint32_t)));
    HIP_TRY(hipMalloc((void**)&c->d_cand_off, (np + 1) * sizeof(uint32_t)));
    HIP_TRY(hipMalloc((void**)&c->d_cand_global, (np + 1) * sizeof(uint32_t)));
    HIP_TRY(hipMalloc((void**)&c->d_cand_big, (np + 1) * sizeof(uint32_t)));
    // [8]: a saved valid count; [16..23]: the last asynchronous build's ctr[0..7]
    HIP_TRY(hipMalloc((void**)&c->d_cand_ctr, 32 * sizeof(uint32_t)));
    HIP_TRY(hipMalloc((void**)&c->d_cand_skip, (np + 1) * sizeof(float)));
    HIP_TRY(hipMalloc((void**)&c->d_cand_big_lane, (size_t)kBigLaneCap * 64 * sizeof(uint32_t)));
    HIP_TRY(hipMalloc((void**)&c->d_cand_items, ((size_t)kItemCap + 1) * sizeof(uint2)));
    const size_t nw = (size_t)rt_cand_big_waves() + 1;
    HIP_TRY(hipMalloc((void**)&c->d_cand_wave_items, nw * sizeof(uint32_t)));
    HIP_TRY(hipMemset(c->d_cand_wave_items, 0, nw * sizeof(uint32_t)));  // [last] stays 0
    HIP_TRY(hipMalloc((void**)&c->d_cand_wave_base, nw * sizeof(uint32_t)));
    HIP_TRY(hipMalloc((void**)&c->d_scan_bsum, (size_t)rt_cand_scan_dev_tiles((uint32_t)np) * sizeof(uint32_t)));
    HIP_TRY(hipHostMalloc((void**)&c->h_cand, 8 * sizeof(uint32_t), hipHostMallocDefault));
  }
  cp.list = c->d_cand_list;
  cp.fp = (rtc::Footprint*)c->d_cand_fp;
  // compact small footprints while tile columns fit their 16-bit intervals
  cp.sfp = cp.tiles_x < 32767 ? c->d_cand_sfp : nullptr;
  cp.store_fp = (c->cand_store_fp || !cp.sfp) ? 1u : 0u;
  cp.visits = c->d_cand_visits;
  cp.off = c->d_cand_off;
  cp.global = c->d_cand_global;
  cp.big = c->d_cand_big;
  cp.ctr = c->d_cand_ctr;
  cp.skip = c->d_cand_skip;
  cp.big_lane = c->d_cand_big_lane;
  cp.big_cap = kBigLaneCap;
  cp.items = c->d_cand_items;
  cp.item_cap = c->cand_item_cap < kItemCap ? c->cand_item_cap : kItemCap;
  cp.chunk_shift = cand_chunk_shift(glob_copies ? glob_copies : (uint32_t)cp.nranks);
  cp.wave_items = c->d_cand_wave_items;
  cp.wave_base = c->d_cand_wave_base;
  cp.refine = c->cand_refine ? 1u : 0u;
  cp.drop_key = (uint32_t)cp.ntiles_local;  // sorts after the tiles (their keys are < ntiles_local)
  // (ctr[0 .. 7] and visits[np] are zeroed by quick_kernel)
  size_t tb = 0;
  HIP_TRY(rt_cand_scan(c->d_cand_visits, c->d_cand_off, (uint32_t)np, nullptr, &tb, s));
  rc = ensure_tmp(c, tb);
  if (rc) return rc;
  tb = 0;
  HIP_TRY(rt_cand_scan(c->d_cand_wave_items, c->d_cand_wave_base, rt_cand_big_waves(), nullptr, &tb, s));
  rc = ensure_tmp(c, tb);
  if (rc) return rc;
  // pass 0: flags -> compact list of the prims the float fast path leaves
  // (over this build's slice of the prims only)
  if (cp.prim1 > cp.nprim || cp.prim0 > cp.prim1) return rt_set_error(RT_EINVAL, "prim slice");
  const uint32_t slice = cp.prim1 - cp.prim0;
  HIP_TRY(rt_cand_quick(&cp, s));
#if RT_DEV_SCAN
  (void)slice;
  HIP_TRY(rt_cand_scan_scatter(&cp, c->d_scan_bsum, s));
#else
  tb = c->scan_tmp_bytes;
  HIP_TRY(rt_cand_scan(c->d_cand_visits, c->d_cand_off, slice, c->d_scan_tmp, &tb, s));
  HIP_TRY(rt_cand_scatter(&cp, s));
  HIP_TRY(hipMemsetAsync(c->d_cand_visits, 0, (np + 1) * sizeof(uint32_t), s));
#endif
  // pass 1: footprints and tile counts of the listed prims
  HIP_TRY(rt_cand_count(&cp, s));
  HIP_TRY(rt_cand_big_count(&cp, s));
  // the big footprints' emission items (a scan over the big_count waves)
  tb = c->scan_tmp_bytes;
  HIP_TRY(rt_cand_scan(c->d_cand_wave_items, c->d_cand_wave_base, rt_cand_big_waves(), c->d_scan_tmp, &tb, s));
  HIP_TRY(rt_cand_items(&cp, s));
#if RT_DEV_SCAN
  // over the list's length only (ctr[3], on the device); the entry total -> ctr[6]
  HIP_TRY(rt_cand_scan_dev(c->d_cand_visits, c->d_cand_off, (uint32_t)np, c->d_cand_ctr + 3, c->d_cand_ctr + 6,
                           c->d_scan_bsum, s));
  if (known) {
    // no read-back: the frame's lists were built before with a read-back of
    // their sizes (deterministic for the same frame), so the buffers hold
    // them; an entry past known->total would not be written and would set
    // ctr[7] (rt_hip_stats then reports the frame, rt_hip_cand_produce
    // builds again: never silent).  The emission kernels read the item
    // count and the over-cap flag on the device and the render reads the
    // global prims' count there
    rc = cand_entry_buffers(c, (size_t)known->total + (size_t)glob_copies * known->nglobal);
    if (rc) return rc;
    cp.keys = c->d_cand_keys;
    cp.vals = c->d_cand_vals;
    cp.key_cap = known->total;
    HIP_TRY(rt_cand_emit(&cp, s));
    // the same launch shape as the read-back build (the kernels read the
    // counts on the device and loop over whatever they find)
    if (known->over)
      HIP_TRY(rt_cand_big(&cp, known->nbig, s));
    else
      HIP_TRY(rt_cand_big_items(&cp, known->nitems, 1, s));
    // (entries past the build's own total, ctr[6] -- never expected -- are
    // left to the caller: cand_prepare drops them before the sort, a
    // produce's partition routes them as dropped; and cand_prepare's
    // bounds_kernel snapshots the counters for rt_hip_stats)
    *total_out = known->total;  // the sort's length
    *nglobal_out = known->nglobal;  // (the render reads the count on the device, ctr[1])
    return RT_OK;
  }
  // one read-back of the build's sizes: ctr[1..6] (the total in [6], the
  // items in [4])
  HIP_TRY(hipMemcpyAsync(c->h_cand, c->d_cand_ctr, 8 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
#else
  tb = c->scan_tmp_bytes;
  HIP_TRY(rt_cand_scan(c->d_cand_visits, c->d_cand_off, (uint32_t)np, c->d_scan_tmp, &tb, s));
  HIP_TRY(hipMemcpyAsync(c->h_cand, c->d_cand_ctr, 8 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(c->h_cand + 6, c->d_cand_off + np, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
#endif
  HIP_TRY(hipStreamSynchronize(s));
  const uint32_t total = c->h_cand[6], nglobal = c->h_cand[1], nbig = c->h_cand[2];
  const uint32_t nitems = c->h_cand[4], items_over = c->h_cand[5];
  rc = cand_entry_buffers(c, (size_t)total + (size_t)glob_copies * nglobal);
  if (rc) return rc;
  cp.key_cap = 0;
  cp.keys = c->d_cand_keys;
  cp.vals = c->d_cand_vals;
  HIP_TRY(rt_cand_emit(&cp, s));
  if (items_over)
    HIP_TRY(rt_cand_big(&cp, nbig, s));
  else
    HIP_TRY(rt_cand_big_items(&cp, nitems, 0, s));
  if (shape) {
    shape->total = total;
    shape->nglobal = nglobal;
    shape->nbig = nbig;
    shape->nitems = nitems;
    shape->over = items_over;
  }
  *total_out = total;
  *nglobal_out = nglobal;
  return RT_OK;
}

// Sorts n (key < n_keys, value) pairs keys/vals -> keys2/vals2 on the key
// bits from begin_bit up (rocPRIM radix sort, stable, temporary storage in
// d_scan_tmp).
static int cand_sort(rt_hip_ctx* c, uint32_t* keys, uint32_t* keys2, uint32_t* vals, uint32_t* vals2, uint32_t n,
                     size_t n_keys, hipStream_t s, int begin_bit = 0) {
  const int bits = key_bits(n_keys);
  size_t tb = 0;
  HIP_TRY(rt_cand_sort(keys, keys2, vals, vals2, n, begin_bit, bits, nullptr, &tb, s));
  int rc = ensure_tmp(c, tb);
  if (rc) return rc;
  tb = c->scan_tmp_bytes;
  if (n) HIP_TRY(rt_cand_sort(keys, keys2, vals, vals2, n, begin_bit, bits, c->d_scan_tmp, &tb, s));
  return RT_OK;
}

// This rank's lists, built on this rank: cand_build for the rank's tiles
// (every prim) -> radix sort by tile -> per-tile offsets -> per-entry skip
// bounds -> work order.
static int cand_prepare(rt_hip_ctx* c, const rt_frame* f, KParams* kp, hipStream_t s, int compat) {
  CandParams cp;
  int rc = cand_params(f, c->scene_c, c->scene_r, c->cam_eps_ulps, c->bound_scale, kp->rank, kp->nranks,
                       &cp, compat);
  if (rc) return rc;
  cp.prim0 = 0;
  cp.prim1 = c->nprim;
  const size_t nt = (size_t)kp->ntiles_local;
  uint32_t total = 0, nglobal = 0;
  // The last build's counters, read back without waiting after an
  // estimated-shape build below: the next estimate starts from them
  if (c->snap_pending && c->ev_kept && hipEventQuery(c->ev_kept) == hipSuccess) {
    const uint32_t* h = c->h_kept + 1;  // ctr[0..7]
    if (h[7]) {  // that frame outgrew its estimate (reported): the next build reads back
      c->known.valid = c->kept_for.valid = 0;
    } else if (c->known.valid) {
      c->known.total = h[6];
      c->known.nglobal = h[1];
      c->known.nbig = h[2];
      c->known.nitems = h[4];
      c->known.over = h[5];
    }
    c->snap_pending = 0;
  }
  // Asynchronous (no host wait) for a frame whose lists were built before
  // with a read-back -- its sizes are deterministic -- and, with headroom,
  // for a new camera of the same size and rank split (an animation's next
  // frame, a panned view): the last build's sizes + 1/4 size the buffers and
  // launches, every kernel checks its counts on the device, and a frame past
  // them is reported (RT_EHITBUF via ctr[7], rt_hip_stats / the frame check)
  // and built again with a read-back.  The first frame of a size or split,
  // the compatibility mode and cand_verify's rebuild (every footprint kept)
  // read their sizes back.
  const bool exact_shape = c->known.same(f, kp->rank, kp->nranks);
  const bool est_shape = !exact_shape && RT_ASYNC_NEW_CAMERA && c->known.same_grid(f, kp->rank, kp->nranks);
  const bool async = RT_DEV_SCAN && c->async_lists && !c->cand_store_fp && !compat && (exact_shape || est_shape);
  ListShape est = c->known;
  if (est_shape) {
    est.total = c->known.total + c->known.total / 4 + 4096;
    est.nglobal = c->known.nglobal + c->known.nglobal / 4 + 64;
    est.nbig = c->known.nbig + c->known.nbig / 4 + 64;
    est.nitems = c->known.nitems + c->known.nitems / 4 + 64;
  }
  rc = cand_build(c, cp, s, 0, &total, &nglobal, async ? &est : nullptr, async ? nullptr : &c->known);
  if (rc) return rc;
  c->last_async = async ? 1 : 0;
  if (async) nglobal = 0;  // on the device (ctr[1])
  if (!async && !compat) {  // the sizes just read back size this frame's later builds
    c->known.set(f, kp->rank, kp->nranks);
  } else if (!async) {
    c->known.valid = 0;
  }
  rc = cand_tile_buffers(c, nt);
  if (rc) return rc;
  // the kept count of the last build of this size and split, once its
  // read-back is done
  if (!c->kept_ready && c->kept_for.valid && c->ev_kept && hipEventQuery(c->ev_kept) == hipSuccess) {
    c->kept = *c->h_kept;
    c->kept_ready = 1;
  }
  // the kept entries compacted before the sort (the refinement drops ~55 %
  // of them on C5): an asynchronous build takes the kept count of the same
  // frame's earlier build; a fresh frame (a new camera: the build read its
  // total back anyway) reads its own back after the compaction's scan -- one
  // more short host wait instead of sorting the dropped entries
  // (for a new camera the last frame's kept count + 1/8: the scatter writes
  // the unused tail as dropped, and a count past it sets ctr[7])
  const bool kept_same = c->kept_for.same(f, kp->rank, kp->nranks);
  const bool compact_known = RT_COMPACT_LISTS && async && c->cand_refine && c->kept_ready &&
                             (kept_same || (RT_ASYNC_NEW_CAMERA && c->kept_for.same_grid(f, kp->rank, kp->nranks))) &&
                             c->kept <= total && total > 0;
  const bool compact_fresh = RT_COMPACT_LISTS && RT_COMPACT_FRESH && !async && !compat && !c->cand_store_fp &&
                             c->cand_refine && total > 0;
  bool kept_now = false;
  if (compact_known || compact_fresh) {
    // the kept entries (stable) -> keys2 / d_cand, sorted back into keys /
    // vals, and the buffer pairs swapped so that the sorted ones are where
    // the uncompacted path leaves them
    const uint32_t nw = rt_cand_part_waves(total);
    if ((size_t)2 * nw + 4 > c->part_cap) {
      (void)hipFree(c->d_part);
      c->d_part = nullptr;
      c->part_cap = 0;
      const size_t cap = 2 * ((size_t)nw + nw / 4) + 1024;
      HIP_TRY(hipMalloc((void**)&c->d_part, cap * sizeof(uint32_t)));
      c->part_cap = cap;
    }
    uint32_t* cnt = c->d_part;
    uint32_t* off = c->d_part + nw + 1;
    size_t tmpb = 0;
    // (only the build's own entries, ctr[6]; fewer kept than last time --
    // never expected -- leave a tail the scatter writes as dropped)
    uint32_t cap = total;
    if (compact_known) {
      cap = kept_same ? c->kept : c->kept + c->kept / 8 + 4096;
      if (cap > total) cap = total;
    }
    HIP_TRY(rt_cand_compact(c->d_cand_keys, c->d_cand_vals, total, c->d_cand_ctr + 6, (uint32_t)nt, cap, cnt, off,
                            nullptr, &tmpb, c->d_cand_keys2, c->d_cand, c->d_cand_ctr + 7, s));
    rc = ensure_tmp(c, tmpb);
    if (rc) return rc;
    tmpb = c->scan_tmp_bytes;
    HIP_TRY(rt_cand_compact(c->d_cand_keys, c->d_cand_vals, total, c->d_cand_ctr + 6, (uint32_t)nt, cap, cnt, off,
                            c->d_scan_tmp, &tmpb, c->d_cand_keys2, c->d_cand, c->d_cand_ctr + 7, s));
    uint32_t kept = cap;
    if (compact_fresh) {  // off[nw] = the kept entries
      if (!c->h_kept) HIP_TRY(hipHostMalloc((void**)&c->h_kept, 9 * sizeof(uint32_t), hipHostMallocDefault));
      HIP_TRY(hipMemcpyAsync(c->h_kept, off + nw, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));
      kept = *c->h_kept;
      if (kept > total) return rt_set_error(RT_EHIP, "compaction kept %u of %u entries", kept, total);
      c->kept = kept;
      c->kept_ready = 1;
      c->kept_for.set(f, kp->rank, kp->nranks);
      kept_now = true;
    }
    rc = cand_sort(c, c->d_cand_keys2, c->d_cand_keys, c->d_cand, c->d_cand_vals, kept, nt + 1, s);
    if (rc) return rc;
    std::swap(c->d_cand_keys, c->d_cand_keys2);
    std::swap(c->d_cand_vals, c->d_cand);
    total = kept;
  } else {
    // an asynchronous build's entries past its own total (never expected): dropped
    if (async) HIP_TRY(rt_cand_fill_tail(c->d_cand_keys, c->d_cand_ctr + 6, total, (uint32_t)nt, s));
    // keys are tiles < nt, or nt for an entry the refinement dropped: nt + 1 keys
    rc = cand_sort(c, c->d_cand_keys, c->d_cand_keys2, c->d_cand_vals, c->d_cand, total, nt + 1, s);
    if (rc) return rc;
  }
  // start[nt] = the entries with a tile (the dropped ones sort after them)
  // (an asynchronous build's counters snapshot for rt_hip_stats, where no build writes)
  HIP_TRY(rt_cand_bounds(c->d_cand_keys2, total, c->d_cand_start, (uint32_t)nt, async ? c->d_cand_ctr : nullptr, s));
  if (RT_COMPACT_LISTS && c->cand_refine && !compat && !kept_now && (!kept_same || est_shape)) {
    // this frame's kept count -- and after an estimated-shape build its
    // counters (bounds_kernel's snapshot) -- for the later builds, read back
    // without waiting
    if (!c->h_kept) HIP_TRY(hipHostMalloc((void**)&c->h_kept, 9 * sizeof(uint32_t), hipHostMallocDefault));
    if (!c->ev_kept) HIP_TRY(hipEventCreateWithFlags(&c->ev_kept, hipEventDisableTiming));
    HIP_TRY(hipMemcpyAsync(c->h_kept, c->d_cand_start + nt, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    if (est_shape) HIP_TRY(hipMemcpyAsync(c->h_kept + 1, c->d_cand_ctr + 16, 8 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipEventRecord(c->ev_kept, s));
    c->kept_for.set(f, kp->rank, kp->nranks);
    c->kept_ready = 0;
    c->snap_pending = est_shape ? 1 : 0;
  }
  // the sorted keys are spent: their buffer takes the per-entry skip bounds
  float* entry_skip = (float*)c->d_cand_keys2;
  HIP_TRY(rt_cand_entry_skip(c->d_cand, c->d_cand_skip, entry_skip, total, c->d_cand_start + nt, s));
  // longest-first work order of the rank's tiles (heavy lists first)
  rc = cand_order(c, kp, nt, total, s, f, kp->rank, kp->nranks);
  if (rc) return rc;
  kp->cand = c->d_cand;
  kp->cand_global = c->d_cand_global;
  kp->n_cand_global = nglobal;
  kp->n_cand_global_dev = async ? c->d_cand_ctr + 1 : nullptr;
  kp->cand_skip = entry_skip;
  c->cand_entries = total;  // until rt_hip_stats reads start[nt]
  c->d_cand_valid = (c->cand_refine || async) ? c->d_cand_start + nt : nullptr;
  c->cand_global = nglobal;
  c->cand_prims = 0;  // not counted separately (entries and globals are)
  return RT_OK;
}

// Triangle-parallel lists of an N-rank frame:
// rank r builds the whole frame's entries of prims [r P / N, (r + 1) P / N)
// -- the float fast path, classification and emission each run once per
// prim over the N GPUs instead of once per prim on every GPU -- and routes
// them to the ranks owning their tiles; one all-to-all exchange gives each
// rank its own lists (rt_hip_cand_consume).
extern "C" int rt_hip_cand_produce(rt_hip_ctx* c, const rt_frame* f, int rank, int nranks, unsigned* counts,
                                   unsigned* nglobal_out, void* stream) {
  if (!c || !f || !counts || !nglobal_out) return rt_set_error(RT_EINVAL, "null argument");
  if (nranks <= 0 || rank < 0 || rank >= nranks) return rt_set_error(RT_EINVAL, "rank %d of %d", rank, nranks);
  if (c->accel != RT_ACCEL_OCTREE || !c->d_node || !c->exact_camera)
    return rt_set_error(RT_EINVAL, "no camera candidate lists in this configuration (octree, exact camera rays)");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  CandParams cp;
  int rc = cand_params(f, c->scene_c, c->scene_r, c->cam_eps_ulps, c->bound_scale, 0, 1, &cp, 0);
  if (rc) return rc;
  const uint64_t np = c->nprim;
  // this producer's slice: the blocks of RT_SLICE_BLOCK prims b = rank mod
  // nranks (prims near each other in the scene -- one sphere, one region --
  // are near each other in prim order: contiguous slices loaded the producer
  // of the nearest objects ~20 % above the mean on C5, blocks spread it)
  const uint64_t nb = (np + RT_SLICE_BLOCK - 1) / RT_SLICE_BLOCK;
  uint64_t len = 0;
  for (uint64_t b = (uint64_t)rank; b < nb; b += (uint64_t)nranks)
    len += std::min<uint64_t>(RT_SLICE_BLOCK, np - b * RT_SLICE_BLOCK);
  cp.prim0 = 0;
  cp.prim1 = (uint32_t)len;
  cp.sl_stride = (uint32_t)nranks;
  cp.sl_rank = (uint32_t)rank;
  // a slice produced before for this frame is built without the mid-build
  // read-back (its sizes are deterministic); the read-back of the counts at
  // the end checks them, and a mismatch -- never expected -- builds again
  const bool async = RT_DEV_SCAN && c->async_lists && !c->cand_store_fp && c->pknown.same(f, rank, nranks);
  uint32_t total = 0, nglobal = 0;
  rc = cand_build(c, cp, s, (uint32_t)nranks, &total, &nglobal, async ? &c->pknown : nullptr,
                  async ? nullptr : &c->pknown);
  if (rc) return rc;
  if (!async) c->pknown.set(f, rank, nranks);
  const uint32_t tpr = (uint32_t)rt_hip_tiles_per_rank(f->width, f->height, nranks);
  const int tb = rt_block_side(nranks);
  // key = rank << tbits | local tile (tpr: a global), rank nranks for an
  // entry the refinement dropped (or, in an asynchronous build, past the
  // build's own total); then a stable partition by rank: each rank's entries
  // keep their emission order, which the consumer's stable sort by tile
  // turns into the per-tile order of the rank's own build
  const int tbits = key_bits((size_t)tpr + 1);
  if (nranks > 256 || tbits + key_bits((size_t)nranks + 1) > 32)
    return rt_set_error(RT_EINVAL, "%d ranks x %u tiles per rank: routed keys exceed 32 bits", nranks, tpr);
  // (the entries' routing is fused into the partition's count pass)
  HIP_TRY(rt_cand_route_globals(c->d_cand_global, nglobal, nranks, tpr, (uint32_t)tbits, c->d_cand_keys + total,
                                c->d_cand_vals + total, s));
  const uint32_t n = total + nglobal * (uint32_t)nranks;
  if ((size_t)nranks + 9 > c->rstart_cap) {  // the starts, then the build's counters
    (void)hipFree(c->d_rstart);
    (void)hipHostFree(c->h_rstart);
    c->d_rstart = nullptr;
    c->h_rstart = nullptr;
    c->rstart_cap = 0;
    HIP_TRY(hipMalloc((void**)&c->d_rstart, ((size_t)nranks + 9) * sizeof(uint32_t)));
    HIP_TRY(hipHostMalloc((void**)&c->h_rstart, ((size_t)nranks + 9) * sizeof(uint32_t), hipHostMallocDefault));
    c->rstart_cap = (size_t)nranks + 9;
  }
  if (3 * (size_t)n + 1 > c->send_cap) {
    (void)hipFree(c->d_send);
    c->d_send = nullptr;
    c->send_cap = 0;
    const size_t cap = 3 * ((size_t)n + n / 4 + 1024);
    HIP_TRY(hipMalloc((void**)&c->d_send, cap * sizeof(uint32_t)));
    c->send_cap = cap;
  }
  // per-wave rank counts (rank-major) -> exclusive scan -> stable scatter
  const size_t nh = ((size_t)nranks + 1) * rt_cand_part_waves(n);
  if (2 * nh + 2 > c->part_cap) {
    (void)hipFree(c->d_part);
    c->d_part = nullptr;
    c->part_cap = 0;
    const size_t cap = 2 * (nh + nh / 4) + 1024;
    HIP_TRY(hipMalloc((void**)&c->d_part, cap * sizeof(uint32_t)));
    c->part_cap = cap;
  }
  uint32_t* hist = c->d_part;
  uint32_t* hoff = c->d_part + nh + 1;
  if (nh) {
    size_t tmpb = 0;
    HIP_TRY(rt_cand_scan(hist, hoff, (uint32_t)(nh - 1), nullptr, &tmpb, s));
    rc = ensure_tmp(c, tmpb);
    if (rc) return rc;
    tmpb = c->scan_tmp_bytes;
    HIP_TRY(rt_cand_part_count(c->d_cand_keys, n, (uint32_t)tbits, nranks, hist, total, cp.tiles_x,
                               rt_blocks_x(cp.tiles_x, tb), tb, cp.drop_key, async ? c->d_cand_ctr + 6 : nullptr, s));
    HIP_TRY(rt_cand_scan(hist, hoff, (uint32_t)(nh - 1), c->d_scan_tmp, &tmpb, s));
  }
  HIP_TRY(rt_cand_part_scatter(c->d_cand_keys, c->d_cand_vals, c->d_cand_skip, n, (uint32_t)tbits, nranks, hoff,
                               c->d_rstart, c->d_send, c->d_cand_ctr, s));
  // the per-rank starts and the build's counters in one read-back
  HIP_TRY(hipMemcpyAsync(c->h_rstart, c->d_rstart, ((size_t)nranks + 9) * sizeof(uint32_t), hipMemcpyDeviceToHost,
                         s));
  HIP_TRY(hipStreamSynchronize(s));
  const uint32_t* hc = c->h_rstart + nranks + 1;  // ctr[0 .. 7]
  if (async && (hc[7] || hc[6] != c->pknown.total || hc[1] != c->pknown.nglobal || hc[2] != c->pknown.nbig ||
                hc[4] != c->pknown.nitems || hc[5] != c->pknown.over)) {
    c->pknown.valid = 0;  // not this slice's sizes after all: build it with the read-back
    return rt_hip_cand_produce(c, f, rank, nranks, counts, nglobal_out, stream);
  }
  for (int d = 0; d < nranks; d++) counts[d] = c->h_rstart[d + 1] - c->h_rstart[d];
  *nglobal_out = nglobal;
  c->send_n = c->h_rstart[nranks];  // the routed entries (the refinement's dropped ones sort after them)
  return RT_OK;
}

extern "C" int rt_hip_cand_send_buffer(const rt_hip_ctx* c, const void** d_entries, size_t* n) {
  if (!c || !d_entries || !n) return rt_set_error(RT_EINVAL, "null argument");
  *d_entries = c->d_send;
  *n = c->send_n;
  return RT_OK;
}

// This rank's lists from the entries the producers routed to it (any order
// of sources; 3 words each: rank-local tile or tpr for a global, prim, skip
// bits): sort by tile -> gather prims and skip bounds -> offsets -> work
// order.  The next rt_hip_render of (frame, rank, nranks) uses them.
extern "C" int rt_hip_cand_consume(rt_hip_ctx* c, const rt_frame* f, int rank, int nranks, const void* d_entries,
                                   size_t n, unsigned nglobal, void* stream) {
  if (!c || !f || (!d_entries && n)) return rt_set_error(RT_EINVAL, "null argument");
  if (nranks <= 0 || rank < 0 || rank >= nranks) return rt_set_error(RT_EINVAL, "rank %d of %d", rank, nranks);
  if (n >= (1ull << 31) || nglobal > n) return rt_set_error(RT_EINVAL, "%zu entries, %u globals", n, nglobal);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  const size_t nt = (size_t)rank_tile_count(f->width, f->height, rank, nranks);
  const uint32_t tpr = (uint32_t)rt_hip_tiles_per_rank(f->width, f->height, nranks);
  c->ext_ready = 0;  // set again once this consume's lists are complete
  int rc = save_valid(c, s);
  if (rc) return rc;
  rc = cand_entry_buffers(c, n);
  if (rc) return rc;
  rc = cand_tile_buffers(c, nt);
  if (rc) return rc;
  const uint32_t* in = (const uint32_t*)d_entries;
  HIP_TRY(rt_cand_unpack(in, (uint32_t)n, (uint32_t)nt, tpr, c->d_cand_keys, c->d_cand_vals, s));
  // keys are tiles < nt, or nt for the globals: nt + 1 keys
  rc = cand_sort(c, c->d_cand_keys, c->d_cand_keys2, c->d_cand_vals, c->d_cand, (uint32_t)n, nt + 1, s);
  if (rc) return rc;
  const uint32_t total = (uint32_t)(n - nglobal);
  HIP_TRY(rt_cand_bounds(c->d_cand_keys2, total, c->d_cand_start, (uint32_t)nt, nullptr, s));
  // the spent unsorted keys take the skip bounds, the spent indices the prims
  HIP_TRY(rt_cand_gather(in, c->d_cand, (uint32_t)n, c->d_cand_vals, (float*)c->d_cand_keys, s));
  KParams kp;
  std::memset(&kp, 0, sizeof kp);
  rc = cand_order(c, &kp, nt, total, s, f, rank, nranks);
  if (rc) return rc;
  c->ext = kp;
  c->ext.cand = c->d_cand_vals;
  c->ext.cand_skip = (const float*)c->d_cand_keys;
  c->ext.cand_global = c->d_cand_vals + total;
  c->ext.n_cand_global = nglobal;
  c->ext_ready = 1;
  c->ext_rank = rank;
  c->ext_nranks = nranks;
  std::memcpy(&c->ext_frame, f, sizeof *f);
  c->ext_total = total;
  return RT_OK;
}

// Hit-record buffers for a rank of ntiles tiles: first sized for 2 hits per
// camera ray (the reference scenes make 0.5-1.3; C5 0.48), then for what an
// overflowing frame needed (rt_hip_stats -> RT_EHITBUF); `last` for every
// (item, lane).
static int hit_buffers(rt_hip_ctx* c, size_t ntiles) {
  const size_t items = 4 * ntiles;
  if (items > c->last_cap) {
    (void)hipFree(c->d_last);
    c->d_last = nullptr;
    c->last_cap = 0;
    HIP_TRY(hipMalloc((void**)&c->d_last, items * 64 * sizeof(uint32_t)));
    c->last_cap = items;
  }
  size_t want = (2 * items * 64 + RT_HIT_REGIONS - 1) / RT_HIT_REGIONS + 1024;
  if (c->hit_need > want) want = c->hit_need;
  if (want > (1ull << 29) - 1) want = (1ull << 29) - 1;  // slot field of a record index
  if (want <= c->hit_cap && c->d_hit) return RT_OK;
  (void)hipFree(c->d_hit);
  (void)hipFree(c->d_hit_prev);
  (void)hipFree(c->d_hit_term);
  c->d_hit = nullptr;
  c->d_hit_prev = nullptr;
  c->d_hit_term = nullptr;
  c->hit_cap = 0;
  const size_t n = want * RT_HIT_REGIONS;
  HIP_TRY(hipMalloc((void**)&c->d_hit, n * 2 * sizeof(float4)));
  HIP_TRY(hipMalloc((void**)&c->d_hit_prev, n * sizeof(uint32_t)));
  HIP_TRY(hipMalloc((void**)&c->d_hit_term, n * sizeof(float4)));
  c->hit_cap = want;  // only once every buffer exists
  return RT_OK;
}

extern "C" int rt_hip_render(rt_hip_ctx* c, const rt_frame* f, int rank, int nranks,
                             float* d_tiles, void* stream) {
  if (!c || !f || !d_tiles) return rt_set_error(RT_EINVAL, "null argument");
  if (nranks <= 0 || rank < 0 || rank >= nranks)
    return rt_set_error(RT_EINVAL, "rank %d of %d", rank, nranks);
  if (f->width <= 0 || f->height <= 0) return rt_set_error(RT_EINVAL, "empty frame");
  // cpu/rt's frame is even-sized (rt_frame_from_camera; its output for odd
  // sizes is undefined, cpu/raytracer.c:89-91,128-134); the camera sample
  // model of the candidate lists assumes it (rt_cand.hip pixel_range)
  if ((f->width | f->height) & 1)
    return rt_set_error(RT_EINVAL, "frame %dx%d: cpu/rt renders even sizes only", f->width, f->height);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  // lists rt_hip_cand_consume built for exactly this frame and rank: used once
  const bool use_ext = c->ext_ready && c->ext_rank == rank && c->ext_nranks == nranks &&
                       std::memcmp(&c->ext_frame, f, sizeof *f) == 0;
  c->ext_ready = 0;
  KParams p;
  std::memset(&p, 0, sizeof p);
  p.tri = c->d_tri;
  p.nrm = c->d_nrm;
  p.mat = c->d_mat;
  p.light = c->d_light;
  p.node = c->d_node;
  p.nrec = c->nrec;
  p.nlight = c->nlight;
  p.u = rt::f3{f->u.x, f->u.y, f->u.z};
  p.v = rt::f3{f->v.x, f->v.y, f->v.z};
  p.C = rt::f3{f->C.x, f->C.y, f->C.z};
  p.pos = rt::f3{f->position.x, f->position.y, f->position.z};
  p.W = f->width;
  p.H = f->height;
  p.tiles_x = tiles_x_of(f->width);
  p.ntiles_total = tiles_x_of(f->width) * tiles_y_of(f->height);
  p.rank = rank;
  p.nranks = nranks;
  p.ntiles_local = rank_tile_count(f->width, f->height, rank, nranks);
  p.out = d_tiles;
  p.tile_counter = c->d_counter;
  p.stats = c->d_stats;
  p.scene_c = rt::f3{c->scene_c[0], c->scene_c[1], c->scene_c[2]};
  p.scene_r = c->scene_r;
  p.scene_cmag = std::fmax(std::fabs(c->scene_c[0]), std::fmax(std::fabs(c->scene_c[1]),
                                                               std::fabs(c->scene_c[2])));
  p.spill = c->d_spill;
  // prim-order records: camera candidates, light buffers and the exact
  // shadow mode's global list all index them (set with or without lists)
  p.tri_prim = c->d_tri_prim;
  // culling slack: eps_ulps ulps of the origin-to-geometry distance
  // (DESIGN.md "Conservative culling")
  p.eps_rel = c->eps_ulps * 5.9604645e-8f;
  p.eps_rel_cam = c->cam_eps_ulps * 5.9604645e-8f;
  if (p.ntiles_local == 0) {
    // a rank past the frame's last block (e.g. 96x54 over 8 ranks: 6 blocks)
    // renders nothing; its tile buffer (sized by rank 0) stays as it is and
    // gathers as padding.  Its stats read 0.
    c->cand_prims = c->cand_entries = c->cand_global = 0;
    c->d_cand_valid = nullptr;
    c->last_async = 0;
    hipEvent_t* ev = c->ev[c->frames % RT_TIMED_FRAMES];
    if (c->timing) HIP_TRY(hipEventRecord(ev[0], s));
    HIP_TRY(hipMemsetAsync(c->d_counter, 0, kFrameCounterBytes, s));
    c->cost_hist.valid = 0;  // (the counters hold no trace's clocks now)
    if (c->timing) {
      for (int k = 1; k < 5; k++) HIP_TRY(hipEventRecord(ev[k], s));
      c->frames++;
    }
    c->last_p = p;
    c->last_stream = s;
    return RT_OK;
  }
  {
    int rc = hit_buffers(c, (size_t)p.ntiles_local);
    if (rc) return rc;
  }
  p.hit = c->d_hit;
  p.hit_prev = c->d_hit_prev;
  p.hit_term = c->d_hit_term;
  p.hit_count = c->d_hit_count;
  p.shade_counter = c->d_hit_count + RT_HIT_REGIONS * 32;
  p.hit_cap = (uint32_t)c->hit_cap;
  p.last = c->d_last;
  if (c->count_work) {  // per-item clocks of the instrumented pass (rt_hip_tile_cycles)
    const size_t items = 4 * (size_t)p.ntiles_local;
    if (items > c->tile_cycles_cap) {
      (void)hipFree(c->d_tile_cycles);
      c->d_tile_cycles = nullptr;
      c->tile_cycles_cap = 0;
      HIP_TRY(hipMalloc((void**)&c->d_tile_cycles, 6 * items * sizeof(unsigned long long)));
      c->tile_cycles_cap = items;
    }
    c->tile_cycles_n = items;
    p.tile_cycles = c->d_tile_cycles;
  }
  {
    // light buffers, proven in exact-shadow mode (no-op unless the slack or
    // the mode changed); the staged policies walk
    int rc = lbuf_prepare(c, s);
    if (rc) return rc;
    if (c->policy == RT_POLICY_DEFAULT || c->policy == RT_POLICY_LANE) p.lbuf = c->d_lbuf;
  }
  // the proven walk's multipliers: only where some light's queries walk
  const bool walks = !p.lbuf || c->info.lightbuf_failed;
  if (walks) {
    int rc = shadow_prepare(c, s);  // no-op unless the culling slack changed
    if (rc) return rc;
  }
  // proven buffers: the off-box queries' queue.  An entry carries the
  // decided bits of lights 0..31 only, so with more lights the off-box
  // queries are counted instead (shadow_unproven -> RT_EINEXACT), never
  // re-shaded without the lights past the 32nd
  if (p.lbuf && c->exact_shadows && c->nlight <= 32) {
    if (!c->d_oob) {
      HIP_TRY(hipMalloc((void**)&c->d_oob_count, sizeof(uint32_t)));
      HIP_TRY(hipMalloc((void**)&c->d_oob, (size_t)RT_OOB_CAP * sizeof(uint4)));
    }
    p.oob = c->d_oob;
    p.oob_count = c->d_oob_count;
    p.oob_cap = RT_OOB_CAP;
    HIP_TRY(hipMemsetAsync(c->d_oob_count, 0, sizeof(uint32_t), s));
  }
  if (c->exact_shadows && walks) {  // the proven walk
    p.node_mu = c->d_node_mu;
    p.sh_global = c->d_sh_global;
    p.n_sh_global = c->n_sh_global;
    p.sh_omax = c->sh_omax;
  }
  c->cand_prims = c->cand_entries = c->cand_global = 0;
  c->d_cand_valid = nullptr;
  hipEvent_t* ev = c->ev[c->frames % RT_TIMED_FRAMES];
  if (c->timing) HIP_TRY(hipEventRecord(ev[0], s));
  if (c->accel == RT_ACCEL_OCTREE && c->d_node && c->exact_camera) {
    if (use_ext) {  // the lists rt_hip_cand_consume built from the producers' entries
      p.cand_start = c->ext.cand_start;
      p.cand = c->ext.cand;
      p.cand_global = c->ext.cand_global;
      p.n_cand_global = c->ext.n_cand_global;
      p.cand_skip = c->ext.cand_skip;
      p.tile_order = c->ext.tile_order;
      p.n_heavy = c->ext.n_heavy;
      p.tri_prim = c->ext.tri_prim;
      c->cand_entries = c->ext_total;
      c->d_cand_valid = nullptr;
      c->cand_global = c->ext.n_cand_global;
      c->cand_prims = 0;
    } else {
      int rc = cand_prepare(c, f, &p, s);
      if (rc) return rc;
    }
  }
  if (!(c->accel == RT_ACCEL_OCTREE && c->d_node && c->exact_camera && !use_ext)) c->last_async = 0;
  // an empty octree scene has nothing to traverse: the FLAT kernels with 0
  // records are exact (their grids are the FLAT instantiation's own)
  const bool empty = c->accel == RT_ACCEL_OCTREE && !c->d_node;
  const int dacc = (c->accel == RT_ACCEL_FLAT || empty) ? RT_ACCEL_FLAT_D : RT_ACCEL_OCTREE_D;
  const int pol = dacc == RT_ACCEL_FLAT_D ? 0 : c->policy, cw = c->count_work ? 1 : 0;
  // the shade kernel without the walk when every directional / point light
  // queries its buffer (the default and per-lane policies use buffers)
  int spol = pol;
  if (dacc == RT_ACCEL_OCTREE_D && p.lbuf && !p.node_mu && !p.n_sh_global &&
      (pol == RT_POLICY_DEFAULT || pol == RT_POLICY_LANE)) {
    bool all = true;
    for (uint32_t li = 0; li < c->nlight && all; li++)
      if (c->light_type[li] == 1 || c->light_type[li] == 2) all = c->lb_dev[li] != nullptr;
    if (all) spol = RT_POLICY_LBUF;
  }
  // exact reflection rays: the default policy's trace kernel with the proven
  // reflection walk (its own instantiation: the default has no switch)
  int tpol = pol;
  if (dacc == RT_ACCEL_OCTREE_D && c->exact_refl) {
    if (pol != RT_POLICY_DEFAULT)
      return rt_set_error(RT_EINVAL, "exact reflections need the default traversal policy (have %d)", pol);
    int rc = reflect_prepare(c, s);
    if (rc) return rc;
    p.node_rf = c->d_node_rf;
    tpol = RT_POLICY_EXACT_REFL;
  }
  int gt = empty ? c->grid : c->grid_of[1][tpol][cw], gs = empty ? c->grid : c->grid_of[0][spol][cw];
  // small frames: no more persistent waves than work items (every wave pulls
  // items until all 8 streams drain, so any grid covers the frame; the
  // surplus waves of a full grid only cost dispatch on a frame of a few
  // thousand items -- C1 has 4,096).  The shade kernel's records are not
  // known before the trace, at least one 64-record chunk per item is assumed
  {
    const long long items = 4ll * p.ntiles_local;
    if (items < gt) gt = (int)items;
    if (items < gs) gs = (int)items;
  }
  // every device pointer the kernels will follow must exist (a null one
  // would fault the card, not fail the call)
  if (!p.tri_prim && (p.lbuf || p.n_sh_global || p.cand_start))
    return rt_set_error(RT_EHIP, "render: prim-order records missing");
  if (!p.hit || !p.last || !p.out || (p.nrec && (!p.tri || !p.nrm)))
    return rt_set_error(RT_EHIP, "render: device buffers missing");
  // item clocks for the same frame's next work order (only the candidate
  // lists' order uses them)
  if (p.tile_order && RT_COST_ORDER) {
    const size_t items = 4 * (size_t)p.ntiles_local;
    if (items > c->item_cost_cap) {
      (void)hipFree(c->d_item_cost);
      c->d_item_cost = nullptr;
      c->item_cost_cap = 0;
      c->cost_hist.valid = 0;
      HIP_TRY(hipMalloc((void**)&c->d_item_cost, items * sizeof(uint32_t)));
      c->item_cost_cap = items;
    }
    p.item_cost = c->d_item_cost;
    p.cost_sum = cost_sum_of(c);
  }
  if (!c->d_frame_check) {
    HIP_TRY(hipMalloc((void**)&c->d_frame_check, 4 * sizeof(unsigned long long)));
    HIP_TRY(hipMemsetAsync(c->d_frame_check, 0, 4 * sizeof(unsigned long long), s));
  }
  p.frame_check = c->d_frame_check;
  p.list_flag = c->last_async ? c->d_cand_ctr + 16 + 7 : nullptr;  // bounds_kernel's snapshot of ctr[7]
  HIP_TRY(hipMemsetAsync(c->d_counter, 0, kFrameCounterBytes, s));  // item streams, stats, record counters
  if (c->timing) HIP_TRY(hipEventRecord(ev[1], s));
  HIP_TRY(rt_launch_trace(&p, dacc, c->count_work, tpol, gt, s));
  if (p.item_cost) {
    c->cost_hist.set(f, rank, nranks);
    c->cost_waves = (uint32_t)gt;
  } else {
    c->cost_hist.valid = 0;
  }
  if (c->timing) HIP_TRY(hipEventRecord(ev[2], s));
  HIP_TRY(rt_launch_shade(&p, dacc, c->count_work, spol, gs, s));
  HIP_TRY(rt_launch_shade_fixup(&p, c->nprim, s));
  if (c->timing) HIP_TRY(hipEventRecord(ev[3], s));
  HIP_TRY(rt_launch_fold(&p, s));
  c->last_p = p;
  if (c->timing) {
    HIP_TRY(hipEventRecord(ev[4], s));
    c->frames++;
  }
  c->last_stream = s;
  return RT_OK;
}

// Shadow verification (tests, tools): the last render's hit records shaded
// again, every stride-th record of each region, once through the context's
// walk (octree) and once by brute force over every triangle (the FLAT any-hit
// of cpu/hit.c:93-109 over the prim-order records), and the two unshadowed-
// light masks compared record by record.  The render's image, terms and stats
// are left as they were.  out = {records compared, shadow queries compared,
// records whose masks differ, queries the walk called lit and brute force
// shadowed}.
extern "C" int rt_hip_verify_shadows_from(rt_hip_ctx* c, unsigned stride, unsigned first,
                                          unsigned long long out[4]);
extern "C" int rt_hip_verify_shadows(rt_hip_ctx* c, unsigned stride, unsigned long long out[4]) {
  return rt_hip_verify_shadows_from(c, stride, 0, out);
}

extern "C" int rt_hip_verify_shadows_from(rt_hip_ctx* c, unsigned stride, unsigned first,
                                          unsigned long long out[4]) {
  if (!c || !out) return rt_set_error(RT_EINVAL, "null argument");
  if (!c->d_hit || !c->last_p.hit) return rt_set_error(RT_EINVAL, "no hit records (render a frame first)");
  if (c->nlight > 32) return rt_set_error(RT_EINVAL, "shadow verification covers at most 32 lights");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = c->last_stream ? c->last_stream : c->stream;
  HIP_TRY(hipStreamSynchronize(s));
  const size_t n = c->hit_cap * RT_HIT_REGIONS;
  uint32_t *lit[2] = {nullptr, nullptr}, *ctr = nullptr;
  float4* term = nullptr;
  unsigned long long* st = nullptr;
  int rc = RT_OK;
  uint32_t hc[RT_HIT_REGIONS * 32];
  std::vector<uint32_t> la, lb;
  unsigned long long nsh = 0;
  for (uint32_t li = 0; li < c->nlight; li++) nsh += c->light_type[li] == 1 || c->light_type[li] == 2;
  if (hipMalloc((void**)&lit[0], n * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc((void**)&lit[1], n * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc((void**)&term, n * sizeof(float4)) != hipSuccess ||
      hipMalloc((void**)&ctr, RT_HIT_REGIONS * 32 * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc((void**)&st, kStatBytes) != hipSuccess) {
    rc = rt_set_error(RT_EHIP, "hipMalloc shadow verification buffers");
    goto done;
  }
  for (int pass = 0; pass < 2 && !rc; pass++) {
    KParams p = c->last_p;
    p.hit_term = term;
    p.hit_lit = lit[pass];
    p.shade_stride = stride ? stride : 1;
    p.shade_first = first;
    p.shade_counter = ctr;
    p.stats = st;
    int dacc = c->accel == RT_ACCEL_FLAT || !c->d_node ? RT_ACCEL_FLAT_D : RT_ACCEL_OCTREE_D;
    int g = c->grid_of[0][0][0];
    if (pass == 1) {  // brute force over the prim-order records
      p.tri = c->d_tri_prim;
      p.nrec = c->nprim;
      p.node = nullptr;
      dacc = RT_ACCEL_FLAT_D;
      if (rt_render_grid(0, RT_ACCEL_FLAT_D, 0, 0, c->cus, &g) != hipSuccess) g = c->grid;
    }
    if (pass == 1) p.oob = nullptr;
    if (hipMemsetAsync(lit[pass], 0xff, n * sizeof(uint32_t), s) != hipSuccess ||
        hipMemsetAsync(ctr, 0, RT_HIT_REGIONS * 32 * sizeof(uint32_t), s) != hipSuccess ||
        (p.oob && hipMemsetAsync(p.oob_count, 0, sizeof(uint32_t), s) != hipSuccess) ||
        rt_launch_shade(&p, dacc, 0, dacc == RT_ACCEL_FLAT_D ? 0 : c->policy, g, s) != hipSuccess ||
        rt_launch_shade_fixup(&p, c->nprim, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      rc = rt_set_error(RT_EHIP, "shadow verification pass %d: %s", pass,
                        hipGetErrorString(hipGetLastError()));
  }
  if (rc) goto done;
  la.resize(n);
  lb.resize(n);
  if (hipMemcpy(la.data(), lit[0], n * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(lb.data(), lit[1], n * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(hc, c->d_hit_count, sizeof hc, hipMemcpyDeviceToHost) != hipSuccess) {
    rc = rt_set_error(RT_EHIP, "shadow verification read-back");
    goto done;
  }
  std::memset(out, 0, 4 * sizeof *out);
  for (int x = 0; x < RT_HIT_REGIONS; x++) {
    const size_t cnt = hc[32 * x] < c->hit_cap ? hc[32 * x] : c->hit_cap;
    for (size_t k = first; k < cnt; k += (stride ? stride : 1)) {
      const size_t a = (size_t)x * c->hit_cap + k;
      out[0]++;
      if (la[a] != lb[a]) {
        out[2]++;
        out[3] += (unsigned long long)__builtin_popcount(la[a] & ~lb[a]);
      }
    }
  }
  out[1] = out[0] * nsh;
done:
  (void)hipFree(lit[0]);
  (void)hipFree(lit[1]);
  (void)hipFree(term);
  (void)hipFree(ctr);
  (void)hipFree(st);
  return rc;
}

// Shadow-query probe (tests, tools): light `light`'s shadow ray from each
// of n host origins (x, y, z), through the context's light buffer (brute =
// 0; built as the context's mode -- slack-grown or proven -- says) or by brute
// force over every triangle (brute = 1).  hit[i] = 1: shadowed.
extern "C" int rt_hip_probe_closest(rt_hip_ctx* c, const float* origins, const float* dirs, size_t n, int brute,
                                    unsigned* prim, float* dist) {
  if (!c || (n && (!origins || !dirs || !prim || !dist))) return rt_set_error(RT_EINVAL, "null argument");
  if (!brute && (c->accel != RT_ACCEL_OCTREE || !c->d_node || !c->d_spill))
    return rt_set_error(RT_EINVAL, "the walk probe needs an octree context");
  if (!c->d_tri_prim) return rt_set_error(RT_EINVAL, "no triangles");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  KParams p;
  std::memset(&p, 0, sizeof p);
  p.tri = c->d_tri;
  p.node = c->d_node;
  p.nrec = c->nrec;
  p.tri_prim = c->d_tri_prim;
  p.spill = c->d_spill;
  p.scene_c = rt::f3{c->scene_c[0], c->scene_c[1], c->scene_c[2]};
  p.scene_r = c->scene_r;
  p.scene_cmag = std::fmax(std::fabs(c->scene_c[0]), std::fmax(std::fabs(c->scene_c[1]),
                                                               std::fabs(c->scene_c[2])));
  p.eps_rel = c->eps_ulps * 5.9604645e-8f;  // the secondary rays' slack (make_ray at depth > 0)
  if (!brute && c->exact_refl) {  // the exact reflection mode's walk
    int rc0 = reflect_prepare(c, s);
    if (rc0) return rc0;
    p.node_rf = c->d_node_rf;
  }
  int gmax = 0;  // waves the spill area holds (rt_hip_create: the largest persistent grid)
  for (auto& a : c->grid_of)
    for (auto& b2 : a)
      for (int g : b2) gmax = g > gmax ? g : gmax;
  if (gmax < c->grid) gmax = c->grid;
  const size_t chunk = (size_t)gmax * 64;
  float *d_o = nullptr, *d_d = nullptr;
  uint32_t* d_h = nullptr;
  const size_t m = n < chunk ? n : chunk;
  std::vector<uint32_t> h(2 * m + 2);
  int rc = RT_OK;
  if (hipMalloc((void**)&d_o, (m * 3 + 1) * sizeof(float)) != hipSuccess ||
      hipMalloc((void**)&d_d, (m * 3 + 1) * sizeof(float)) != hipSuccess ||
      hipMalloc((void**)&d_h, (2 * m + 2) * sizeof(uint32_t)) != hipSuccess)
    rc = rt_set_error(RT_EHIP, "hipMalloc probe buffers");
  for (size_t at = 0; rc == RT_OK && at < n; at += chunk) {  // the walk's spill area holds `chunk` rays
    const size_t k = n - at < chunk ? n - at : chunk;
    if (hipMemcpy(d_o, origins + 3 * at, k * 3 * sizeof(float), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_d, dirs + 3 * at, k * 3 * sizeof(float), hipMemcpyHostToDevice) != hipSuccess ||
        rt_launch_probe_closest(&p, d_o, d_d, (uint32_t)k, c->nprim, brute, d_h, gmax, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess ||
        hipMemcpy(h.data(), d_h, 2 * k * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess) {
      rc = rt_set_error(RT_EHIP, "closest probe: %s", hipGetErrorString(hipGetLastError()));
      break;
    }
    for (size_t i = 0; i < k; i++) {
      prim[at + i] = h[2 * i];
      std::memcpy(&dist[at + i], &h[2 * i + 1], sizeof(float));
    }
  }
  (void)hipFree(d_o);
  (void)hipFree(d_d);
  (void)hipFree(d_h);
  return rc;
}

extern "C" int rt_hip_probe_shadows(rt_hip_ctx* c, unsigned light, const float* origins, size_t n, int brute,
                                    unsigned char* hit) {
  if (!c || (!origins && n) || (!hit && n)) return rt_set_error(RT_EINVAL, "null argument");
  if (light >= c->nlight || (c->light_type[light] != 1 && c->light_type[light] != 2))
    return rt_set_error(RT_EINVAL, "light %u is not a directional or point light", light);
  if (n > (1u << 26)) return rt_set_error(RT_EINVAL, "%zu origins (at most 2^26 per call)", n);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  if (!brute) {
    int rc = lbuf_prepare(c, s);
    if (rc) return rc;
    if (!c->d_lbuf) return rt_set_error(RT_EINVAL, "no light buffers (octree contexts with light buffers on)");
  }
  if (!c->d_tri_prim) return rt_set_error(RT_EINVAL, "no triangles");
  KParams p;
  std::memset(&p, 0, sizeof p);
  p.light = c->d_light;
  p.nlight = c->nlight;
  p.tri_prim = c->d_tri_prim;
  p.lbuf = brute ? nullptr : c->d_lbuf;
  p.scene_c = rt::f3{c->scene_c[0], c->scene_c[1], c->scene_c[2]};
  p.scene_r = c->scene_r;
  p.scene_cmag = std::fmax(std::fabs(c->scene_c[0]), std::fmax(std::fabs(c->scene_c[1]),
                                                               std::fabs(c->scene_c[2])));
  p.eps_rel = c->eps_ulps * 5.9604645e-8f;
  float* d_o = nullptr;
  uint32_t* d_h = nullptr;
  std::vector<uint32_t> h(n);
  int rc = RT_OK;
  if (hipMalloc((void**)&d_o, (n * 3 + 1) * sizeof(float)) != hipSuccess ||
      hipMalloc((void**)&d_h, (n + 1) * sizeof(uint32_t)) != hipSuccess) {
    rc = rt_set_error(RT_EHIP, "hipMalloc probe buffers");
  } else if (hipMemcpy(d_o, origins, n * 3 * sizeof(float), hipMemcpyHostToDevice) != hipSuccess ||
             rt_launch_probe_shadow(&p, d_o, (uint32_t)n, light, (uint32_t)c->nprim, brute, d_h, s) != hipSuccess ||
             hipStreamSynchronize(s) != hipSuccess ||
             hipMemcpy(h.data(), d_h, n * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess) {
    rc = rt_set_error(RT_EHIP, "shadow probe: %s", hipGetErrorString(hipGetLastError()));
  } else {
    for (size_t i = 0; i < n; i++) hit[i] = (unsigned char)h[i];
  }
  (void)hipFree(d_o);
  (void)hipFree(d_h);
  return rc;
}

// The per-frame checks of every render since the last call (fold_kernel):
// *flags = OR of RT_FRAME_* (0: every frame complete and exact by the
// conditions rt_hip_stats checks), *frames = renders checked, queries[0] /
// [1] = their closest-hit / shadow queries summed; all reset.  Lets a caller
// that renders many frames without rt_hip_stats (bench.py's timed loops)
// refuse a result with an incomplete frame in it, and count every frame's
// own queries.
extern "C" int rt_hip_frame_check(rt_hip_ctx* c, unsigned* flags, unsigned* frames, unsigned long long* queries) {
  if (!c || !flags || !frames || !queries) return rt_set_error(RT_EINVAL, "null argument");
  *flags = *frames = 0;
  queries[0] = queries[1] = 0;
  if (!c->d_frame_check) return RT_OK;
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = c->last_stream ? c->last_stream : c->stream;
  unsigned long long h[4] = {0, 0, 0, 0};
  HIP_TRY(hipMemcpyAsync(h, c->d_frame_check, sizeof h, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemsetAsync(c->d_frame_check, 0, sizeof h, s));
  HIP_TRY(hipStreamSynchronize(s));
  *flags = (unsigned)h[0];
  *frames = (unsigned)h[1];
  queries[0] = h[2];
  queries[1] = h[3];
  return RT_OK;
}

extern "C" int rt_hip_stats(rt_hip_ctx* c, rt_stats* out) {
  if (!c || !out) return rt_set_error(RT_EINVAL, "null argument");
  HIP_TRY(hipSetDevice(c->device));
  unsigned long long hs[RT_STAT_SETS * RT_STAT_STRIDE], h[RT_NSTATS];
  uint32_t hc[RT_HIT_REGIONS * 32];
  hipStream_t s = c->last_stream ? c->last_stream : c->stream;
  HIP_TRY(hipMemcpyAsync(hs, c->d_stats, sizeof hs, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(hc, c->d_hit_count, sizeof hc, hipMemcpyDeviceToHost, s));
  uint32_t valid = 0, actr[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c->d_cand_valid) HIP_TRY(hipMemcpyAsync(&valid, c->d_cand_valid, sizeof valid, hipMemcpyDeviceToHost, s));
  const int was_async = c->last_async;
  if (was_async) HIP_TRY(hipMemcpyAsync(actr, c->d_cand_ctr + 16, sizeof actr, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (c->d_cand_valid) {
    c->cand_entries = valid;
    c->d_cand_valid = nullptr;
  }
  if (was_async) {
    c->last_async = 0;
    c->cand_global = actr[1];
    if (actr[7]) {  // never expected (the same frame's lists): reported, and the next build reads back
      c->known.valid = c->kept_for.valid = 0;
      return rt_set_error(RT_EHITBUF, "%u candidate-list entries, %u expected: render again", actr[6],
                          c->known.total);
    }
  }
  for (int k = 0; k < RT_NSTATS; k++) {  // the copies of each counter (RT_STAT_SETS)
    h[k] = 0;
    for (int set = 0; set < RT_STAT_SETS; set++) h[k] += hs[set * RT_STAT_STRIDE + k];
  }
  size_t need = 0;
  unsigned long long records = 0;
  for (int x = 0; x < RT_HIT_REGIONS; x++) {
    need = hc[32 * x] > need ? hc[32 * x] : need;
    records += hc[32 * x];
  }
  std::memset(out, 0, sizeof *out);
  out->closest = h[0];
  out->shadow = h[1];
  out->pixels = h[2];
  out->camera = 4 * h[2];
  out->node_visits = h[3];
  out->tri_tests = h[4];
  out->depth_overflow = h[5];
  out->zero_normal = h[6];
  out->hits = h[7];
  out->closest_node_lanes = h[8];
  out->closest_tri_lanes = h[9];
  out->shadow_node_lanes = h[10];
  out->shadow_tri_lanes = h[11];
  out->cycles_camera = h[12];
  out->cycles_cand = h[13];
  out->cycles_secondary = h[14];
  out->cycles_shadow = h[15];
  out->cycles_shadow_directional = h[16];
  out->stack_spills = h[17];
  out->shadow_zero_risk = h[18];
  out->shadow_node_visits = h[19];
  out->shadow_tri_tests = h[20];
  out->shadow_unproven = h[21];
  out->closest_unproven = h[22];
  out->hit_records = records;
  out->cand_prims = c->cand_prims;
  out->cand_entries = c->cand_entries;
  out->cand_global = c->cand_global;
  if (need > c->hit_cap) {  // the frame is incomplete: grow for the next render
    c->hit_need = need + need / 4 + 1024;
    return rt_set_error(RT_EHITBUF, "%llu hit records, %zu per region held (grown to %zu: render again)",
                        records, c->hit_cap, c->hit_need);
  }
  if (out->depth_overflow)
    return rt_set_error(RT_EDEPTH, "%llu paths overflowed the bounce limit or a traversal stack",
                        out->depth_overflow);
  // never silent: the image may differ from cpu/rt's there
  if (out->zero_normal)
    return rt_set_error(RT_EZERONORMAL,
                        "%llu closest hits had an exactly zero interpolated normal (cpu/hit.c:79 "
                        "would skip those objects)",
                        out->zero_normal);
  if (out->shadow_zero_risk)
    return rt_set_error(RT_EZERONORMAL,
                        "%llu shadow rays hit an object whose interpolated normal can vanish "
                        "(cpu/hit.c:99 may skip it; early any-hit exit not proven exact)",
                        out->shadow_zero_risk);
  if (c->last_p.oob) {
    uint32_t q = 0;
    HIP_TRY(hipMemcpy(&q, c->d_oob_count, sizeof q, hipMemcpyDeviceToHost));
    out->shadow_deferred = q;
    if (q > RT_OOB_CAP)
      return rt_set_error(RT_EINEXACT, "%u shadow queries from off the exact mode's proof box, %u decided",
                          q, RT_OOB_CAP);
  }
  if (out->closest_unproven)
    return rt_set_error(RT_EINEXACT,
                        "%llu reflection rays with |d| past the exact reflection walk's bound "
                        "(csrc/rt_reflect.h RT_RF_DLMAX)", out->closest_unproven);
  if (out->shadow_unproven)
    return rt_set_error(RT_EINEXACT,
                        "%llu shadow rays left from beyond the extent the exact shadow mode's "
                        "bound assumes (csrc/rt_shadow.hip, csrc/rt_lightbuf.hip)",
                        out->shadow_unproven);
  // tuning knobs that give up the parity guarantee (A/B measurements only):
  // the image is complete, but not promised to equal cpu/rt's
  if (c->accel == RT_ACCEL_OCTREE && c->d_node &&
      (!c->exact_camera || c->bound_scale < 1.0 || c->eps_ulps < RT_EPS_ULPS_DEFAULT))
    return rt_set_error(RT_EINEXACT,
                        "rendered with exact_camera=%d, camera bound scale %g, culling slack %g ulps "
                        "(defaults 1, 1, %d): cpu/rt parity not guaranteed",
                        c->exact_camera, c->bound_scale, (double)c->eps_ulps, RT_EPS_ULPS_DEFAULT);
  return RT_OK;
}

extern "C" int rt_hip_assemble(rt_hip_ctx* c, const rt_frame* f, const float* d_gathered,
                               int nranks, float* d_rgb, void* stream) {
  if (!c || !f || !d_gathered || !d_rgb || nranks <= 0)
    return rt_set_error(RT_EINVAL, "bad argument");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  int tx = tiles_x_of(f->width);
  int nt = tx * tiles_y_of(f->height);
  HIP_TRY(rt_launch_assemble(d_gathered, d_rgb, f->width, f->height, tx, nt, nranks,
                             rt_hip_tiles_per_rank(f->width, f->height, nranks), s));
  return RT_OK;
}

extern "C" int rt_hip_render_image(rt_hip_ctx* c, const rt_frame* f, float* h_rgb, rt_stats* st) {
  if (!c || !f || !h_rgb) return rt_set_error(RT_EINVAL, "null argument");
  HIP_TRY(hipSetDevice(c->device));
  size_t nt = rt_hip_tile_buffer_floats(f->width, f->height, 1);
  size_t npx = (size_t)f->width * f->height;
  float *d_tiles = nullptr, *d_rgb = nullptr;
  HIP_TRY(hipMalloc((void**)&d_tiles, nt * sizeof(float)));
  if (hipMalloc((void**)&d_rgb, npx * 3 * sizeof(float)) != hipSuccess) {
    (void)hipFree(d_tiles);
    return rt_set_error(RT_EHIP, "hipMalloc image");
  }
  rt_stats tmp;
  int rc = RT_OK;
  for (int attempt = 0; attempt < 3; attempt++) {  // again after the hit or list buffers grew
    rc = rt_hip_render(c, f, 0, 1, d_tiles, nullptr);
    if (!rc) rc = rt_hip_assemble(c, f, d_tiles, 1, d_rgb, nullptr);
    if (!rc && hipMemcpyAsync(h_rgb, d_rgb, npx * 3 * sizeof(float), hipMemcpyDeviceToHost,
                              c->stream) != hipSuccess)
      rc = rt_set_error(RT_EHIP, "D2H image");
    if (!rc) rc = rt_hip_stats(c, st ? st : &tmp);
    if (rc != RT_EHITBUF) break;
  }
  (void)hipFree(d_tiles);
  (void)hipFree(d_rgb);
  return rc;
}

static int choose_accel(const rt_scene* s);

// gpu/rt compatibility mode (csrc/rt_render.hip compat_kernel): the frame
// of the camera at 3x its size (gpu/rt.cpp:72-83: width and height scaled,
// so L and C follow), one ray per high-resolution pixel, then the 3x3
// downscale; h_rgba = width x height RGBA8 in gpu/rt's PNG row order.
extern "C" int rt_hip_render_compat(rt_hip_ctx* c, const rt_camera* cam, unsigned char* h_rgba,
                                    rt_stats* st) {
  if (!c || !cam || !h_rgba) return rt_set_error(RT_EINVAL, "null argument");
  if (cam->width <= 0 || cam->height <= 0) return rt_set_error(RT_EINVAL, "empty frame");
  if ((long long)cam->width * cam->height > (1ll << 28) / 9)
    return rt_set_error(RT_EINVAL, "frame too large for the 3x render");
  HIP_TRY(hipSetDevice(c->device));
  rt_camera big = *cam;
  big.width = 3 * cam->width;
  big.height = 3 * cam->height;
  rt_frame f;
  int rc = rt_frame_from_camera_any(&big, &f);
  if (rc) return rc;
  const size_t nhi = (size_t)big.width * big.height, nlo = (size_t)cam->width * cam->height;
  uint32_t *d_hi = nullptr, *d_lo = nullptr;
  HIP_TRY(hipMalloc((void**)&d_hi, nhi * sizeof(uint32_t)));
  if (hipMalloc((void**)&d_lo, nlo * sizeof(uint32_t)) != hipSuccess) {
    (void)hipFree(d_hi);
    return rt_set_error(RT_EHIP, "hipMalloc image");
  }
  hipStream_t s = c->stream;
  KParams p;
  std::memset(&p, 0, sizeof p);
  p.tri = c->d_tri;
  p.nrm = c->d_nrm;
  p.mat = c->d_mat;
  p.light = c->d_light;
  p.node = c->d_node;
  p.nrec = c->nrec;
  p.nlight = c->nlight;
  p.u = rt::f3{f.u.x, f.u.y, f.u.z};
  p.v = rt::f3{f.v.x, f.v.y, f.v.z};
  p.C = rt::f3{f.C.x, f.C.y, f.C.z};
  p.pos = rt::f3{f.position.x, f.position.y, f.position.z};
  p.W = big.width;
  p.H = big.height;
  p.tiles_x = tiles_x_of(big.width);
  p.ntiles_total = tiles_x_of(big.width) * tiles_y_of(big.height);
  p.nranks = 1;
  p.ntiles_local = p.ntiles_total;
  p.out = (float*)d_hi;
  p.tile_counter = c->d_counter;
  p.stats = c->d_stats;
  p.scene_c = rt::f3{c->scene_c[0], c->scene_c[1], c->scene_c[2]};
  p.scene_r = c->scene_r;
  p.scene_cmag = std::fmax(std::fabs(c->scene_c[0]), std::fmax(std::fabs(c->scene_c[1]),
                                                               std::fabs(c->scene_c[2])));
  p.spill = c->d_spill;
  p.eps_rel = c->eps_ulps * 5.9604645e-8f;
  p.eps_rel_cam = c->cam_eps_ulps * 5.9604645e-8f;
  const int accel = (c->accel == RT_ACCEL_FLAT || !c->d_node) ? RT_ACCEL_FLAT_D : RT_ACCEL_OCTREE_D;
  rc = shadow_prepare(c, s);
  if (rc) {
    (void)hipFree(d_hi);
    (void)hipFree(d_lo);
    return rc;
  }
  if (c->exact_shadows) {
    p.node_mu = c->d_node_mu;
    p.sh_global = c->d_sh_global;
    p.n_sh_global = c->n_sh_global;
    p.sh_omax = c->sh_omax;
  }
  p.tri_prim = c->d_tri_prim;
  // exact camera rays in this mode too: the candidate lists of the 3x frame's
  // one-sample-per-pixel camera (csrc/rt_cand.hip CandParams::compat)
  c->cand_prims = c->cand_entries = c->cand_global = 0;
  c->d_cand_valid = nullptr;
  if (c->accel == RT_ACCEL_OCTREE && c->d_node && c->exact_camera) {
    rc = cand_prepare(c, &f, &p, s, 1);
    if (rc) {
      (void)hipFree(d_hi);
      (void)hipFree(d_lo);
      return rc;
    }
  }
  c->cost_hist.valid = 0;  // the counters are the compat render's
  if (hipMemsetAsync(c->d_counter, 0, kFrameCounterBytes, s) != hipSuccess ||
      rt_launch_compat(&p, accel, c->grid, s) != hipSuccess ||
      rt_launch_downscale(d_hi, d_lo, cam->width, cam->height, s) != hipSuccess ||
      hipMemcpyAsync(h_rgba, d_lo, nlo * sizeof(uint32_t), hipMemcpyDeviceToHost, s) != hipSuccess)
    rc = rt_set_error(RT_EHIP, "compat render: %s", hipGetErrorString(hipGetLastError()));
  c->last_stream = s;
  rt_stats tmp;
  if (!rc) rc = rt_hip_stats(c, st ? st : &tmp);
  if (st) st->camera = st->pixels;  // one camera ray per high-resolution pixel
  (void)hipFree(d_hi);
  (void)hipFree(d_lo);
  return rc;
}

// gpu/rt.cpp:56-97: `rt file.svati output.png` with gpu/rt's semantics
extern "C" int rt_raytrace_gpu(const char* input, const char* output, int accel) {
  rt_scene* scene = nullptr;
  int rc = rt_scene_load_svati(input, &scene);
  if (rc) return rc;
  if (accel < 0) accel = choose_accel(scene);
  rt_hip_ctx* ctx = nullptr;
  std::vector<unsigned char> img((size_t)4 * (scene->camera.width > 0 ? scene->camera.width : 0) *
                                 (scene->camera.height > 0 ? scene->camera.height : 0) + 4);
  rc = rt_hip_create(0, scene, accel, &ctx);
  if (!rc) rc = rt_hip_render_compat(ctx, &scene->camera, img.data(), nullptr);
  if (!rc) rc = rt_png_write_rgba(output, scene->camera.width, scene->camera.height, img.data());
  if (ctx) rt_hip_destroy(ctx);
  rt_scene_free(scene);
  return rc;
}

extern "C" int rt_hip_malloc(int device, size_t bytes, void** d_ptr) {
  if (!d_ptr) return rt_set_error(RT_EINVAL, "null argument");
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipMalloc(d_ptr, bytes ? bytes : 16));
  return RT_OK;
}
extern "C" int rt_hip_free(void* d_ptr) {
  HIP_TRY(hipFree(d_ptr));
  return RT_OK;
}
extern "C" int rt_hip_memcpy_d2h(void* dst, const void* src, size_t bytes) {
  HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return RT_OK;
}
extern "C" int rt_hip_memcpy_h2d(void* dst, const void* src, size_t bytes) {
  HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return RT_OK;
}

extern "C" int rt_hip_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream) {
  if (!bytes) return RT_OK;
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return RT_OK;
}

// ------------------------------------------------------------ drop-in entry

static int choose_accel(const rt_scene* s) {
  // brute force is exact and cheapest for tiny scenes; the host SAH octree
  // renders the reference's small scenes fastest (C3/C4); from ~10^5
  // triangles the device-built octree both builds (0.7 s vs 6 s) and renders
  // (C5: 19.0 vs 29.0 ms) faster
  size_t n = rt_scene_triangle_count(s);
  return n <= 64 ? RT_ACCEL_FLAT : (n < 100000 ? RT_ACCEL_OCTREE : RT_ACCEL_OCTREE_GPU);
}

extern "C" int rt_raytrace(const char* input, const char* output) {
  return rt_raytrace_multi(input, output, 1, -1, nullptr, nullptr);
}

#define NCCL_TRY(expr)                                                                 \
  do {                                                                                 \
    ncclResult_t r_ = (expr);                                                          \
    if (r_ != ncclSuccess) {                                                           \
      rc = rt_set_error(RT_ERCCL, "%s: %s", #expr, ncclGetErrorString(r_));            \
      goto out;                                                                        \
    }                                                                                  \
  } while (0)

// fn(g) for every GPU g on its own host thread (device setup and the render
// calls -- whose candidate lists wait on their device once -- proceed on all
// GPUs at once); the first failure's message is re-raised on this thread
// (the detail message is per thread, rt_error.c).
template <class F>
static int per_gpu(int ngpus, F fn) {
  std::vector<int> rcs(ngpus, RT_OK);
  std::vector<std::string> msgs(ngpus);
  std::vector<std::thread> th;
  for (int g = 0; g < ngpus; g++)
    th.emplace_back([&, g]() {
      rcs[g] = fn(g);
      if (rcs[g]) msgs[g] = rt_last_error();
    });
  for (auto& t : th) t.join();
  for (int g = 0; g < ngpus; g++)
    if (rcs[g]) return rt_set_error(rcs[g], "GPU %d: %s", g, msgs[g].c_str());
  return RT_OK;
}

// Triangle-parallel candidate lists of an n-rank frame over n contexts in
// this process (rt_raytrace_multi, and tests on one GPU): every rank produces
// the whole frame's entries of its 1/n of the triangles (rt_hip_cand_produce,
// one thread per rank), the blocks are exchanged -- one grouped RCCL
// send/recv all-to-all over the ranks' communicators (comms != NULL: one
// device per rank, xGMI), or device memcpys (comms == NULL: any devices, e.g.
// every context on GPU 0 in a test) -- and every rank consumes its own
// (rt_hip_cand_consume); each context's next rt_hip_render(f, rank, n) uses
// them.  The same three library calls bench.py makes around
// torch.distributed's all_to_all_single.
static int cand_exchange(rt_hip_ctx* const* ctx, int n, const rt_frame* f, ncclComm_t* comms) {
  std::vector<std::vector<unsigned>> counts(n, std::vector<unsigned>(n, 0));
  std::vector<unsigned> ng(n, 0);
  int rc = per_gpu(n, [&](int r) {
    return rt_hip_cand_produce(ctx[r], f, r, n, counts[r].data(), &ng[r], nullptr);
  });
  if (rc) return rc;
  unsigned nglobal = 0;
  for (unsigned x : ng) nglobal += x;
  // rank d receives counts[r][d] entries from each r, in source order
  std::vector<size_t> recv_n(n, 0);
  for (int d = 0; d < n; d++)
    for (int r = 0; r < n; r++) recv_n[d] += counts[r][d];
  std::vector<uint32_t*> recv(n, nullptr);
  bool in_group = false;
  for (int d = 0; d < n && !rc; d++)
    rc = rt_hip_malloc(ctx[d]->device, (recv_n[d] + 1) * 12, (void**)&recv[d]);
  if (!rc && comms) {
    NCCL_TRY(ncclGroupStart());
    in_group = true;
    for (int r = 0; r < n; r++) {
      (void)hipSetDevice(ctx[r]->device);
      size_t so = 0, ro = 0;
      for (int d = 0; d < n; d++) {  // what r sends to d, and receives from d
        if (counts[r][d]) NCCL_TRY(ncclSend(ctx[r]->d_send + 3 * so, 3 * (size_t)counts[r][d], ncclUint32, d,
                                            comms[r], ctx[r]->stream));
        if (counts[d][r]) NCCL_TRY(ncclRecv(recv[r] + 3 * ro, 3 * (size_t)counts[d][r], ncclUint32, d,
                                            comms[r], ctx[r]->stream));
        so += counts[r][d];
        ro += counts[d][r];
      }
    }
    in_group = false;
    NCCL_TRY(ncclGroupEnd());
  } else if (!rc) {
    for (int r = 0; r < n && !rc; r++) {
      if (hipSetDevice(ctx[r]->device) != hipSuccess || hipStreamSynchronize(ctx[r]->stream) != hipSuccess) {
        rc = rt_set_error(RT_EHIP, "exchange: producer %d", r);
        break;
      }
    }
    for (int d = 0; d < n && !rc; d++) {
      size_t ro = 0;
      for (int r = 0; r < n && !rc; r++) {
        size_t so = 0;
        for (int k = 0; k < d; k++) so += counts[r][k];
        // on the receiver's stream, so its consume is ordered after the copy
        // (a device-to-device hipMemcpyPeer may return before it completes)
        if (counts[r][d] &&
            hipMemcpyPeerAsync(recv[d] + 3 * ro, ctx[d]->device, ctx[r]->d_send + 3 * so, ctx[r]->device,
                               (size_t)counts[r][d] * 12, ctx[d]->stream) != hipSuccess)
          rc = rt_set_error(RT_EHIP, "exchange: %d -> %d", r, d);
        ro += counts[r][d];
      }
    }
  }
  if (!rc)
    rc = per_gpu(n, [&](int d) {
      return rt_hip_cand_consume(ctx[d], f, d, n, recv[d], recv_n[d], nglobal, nullptr);
    });
  // the consumes read the received blocks on their streams: wait, then free
  for (int d = 0; d < n; d++) {
    if (recv[d]) {
      (void)hipSetDevice(ctx[d]->device);
      (void)hipStreamSynchronize(ctx[d]->stream);
      rt_hip_free(recv[d]);
    }
  }
  return rc;
out:
  if (in_group) (void)ncclGroupEnd();
  for (int d = 0; d < n; d++)
    if (recv[d]) rt_hip_free(recv[d]);
  return rc;
}

extern "C" int rt_hip_cand_exchange_local(rt_hip_ctx** ctx, int n, const rt_frame* f) {
  if (!ctx || !f || n < 1 || n > 256) return rt_set_error(RT_EINVAL, "bad argument");
  for (int r = 0; r < n; r++)
    if (!ctx[r]) return rt_set_error(RT_EINVAL, "null context %d", r);
  return cand_exchange(ctx, n, f, nullptr);
}

// rt_raytrace_multi's candidate lists: triangle-parallel from this many GPUs
// up (as bench.py: below it the second sort and the exchange cost more than
// the per-rank build's shared part)
#ifndef RT_MULTI_PARTITION_MIN
#define RT_MULTI_PARTITION_MIN 4
#endif

extern "C" int rt_raytrace_multi_dev(const char* input, const char* output, int ngpus, const int* devices,
                                     int accel, rt_stats* stats, double* render_ms);

extern "C" int rt_raytrace_multi(const char* input, const char* output, int ngpus, int accel,
                                 rt_stats* stats, double* render_ms) {
  if (ngpus < 1 || ngpus > 64) return rt_set_error(RT_EINVAL, "bad argument");
  std::vector<int> devs(ngpus);
  for (int g = 0; g < ngpus; g++) devs[g] = g;
  return rt_raytrace_multi_dev(input, output, ngpus, devs.data(), accel, stats, render_ms);
}

// Rank g on device devices[g].  Distinct devices: RCCL (the gather, and the
// candidate lists' all-to-all from 4 ranks up).  A device used by several
// ranks (a test running N ranks on one GPU): the same steps with device
// memcpys (rt_hip_cand_exchange_local's transport, and a copy of each
// rank's tile buffer into the gathered one).
extern "C" int rt_raytrace_multi_dev(const char* input, const char* output, int ngpus, const int* devices,
                                     int accel, rt_stats* stats, double* render_ms) {
  if (!input || !output || !devices || ngpus < 1 || ngpus > 64) return rt_set_error(RT_EINVAL, "bad argument");
  rt_scene* scene = nullptr;
  int rc = rt_scene_load_svati(input, &scene);
  if (rc) return rc;
  // the reference opens (truncates) the output right after parsing, before
  // rendering, and fails there with strerror (cpu/raytracer.c:88,
  // cpu/printer.c:5-7); the P3 text itself is written after the render
  if (FILE* fo = std::fopen(output, "w+")) {
    std::fclose(fo);
  } else {
    rc = rt_set_error(RT_EIO, "%s", std::strerror(errno));
    rt_scene_free(scene);
    return rc;
  }
  rt_frame f;
  rc = rt_frame_from_camera(&scene->camera, &f);
  if (rc) {
    rt_scene_free(scene);
    return rc;
  }
  if (accel < 0) accel = choose_accel(scene);
  int ndev = 0;
  rc = rt_hip_device_count(&ndev);
  bool shared = false;  // some device holds several ranks: memcpy transport, no RCCL
  for (int g = 0; g < ngpus && !rc; g++) {
    if (devices[g] < 0 || devices[g] >= ndev)
      rc = rt_set_error(RT_ENODEV, "rank %d: device %d of %d present", g, devices[g], ndev);
    for (int h = 0; h < g; h++) shared = shared || devices[h] == devices[g];
  }
  std::vector<rt_hip_ctx*> ctx(ngpus, nullptr);
  std::vector<float*> d_tiles(ngpus, nullptr);
  std::vector<ncclComm_t> comms(ngpus, nullptr);
  float* d_gather = nullptr;
  float* d_rgb = nullptr;
  std::vector<float> h_rgb;
  size_t tile_floats = rt_hip_tile_buffer_floats(f.width, f.height, ngpus);
  size_t npx = (size_t)f.width * f.height;
  std::chrono::steady_clock::time_point t0, t1;
  rt_stats sum{};
  bool in_group = false;
  // every GPU builds its own scene image and octree at once
  if (!rc)
    rc = per_gpu(ngpus, [&](int g) {
      int r = rt_hip_create(devices[g], scene, accel, &ctx[g]);
      if (!r) r = rt_hip_malloc(devices[g], tile_floats * sizeof(float), (void**)&d_tiles[g]);
      return r;
    });
  if (!rc) rc = rt_hip_malloc(devices[0], tile_floats * ngpus * sizeof(float), (void**)&d_gather);
  if (!rc) rc = rt_hip_malloc(devices[0], npx * 3 * sizeof(float), (void**)&d_rgb);
  if (rc) goto out;
  if (ngpus > 1 && !shared) NCCL_TRY(ncclCommInitAll(comms.data(), ngpus, devices));
  for (int g = 0; g < ngpus; g++) {
    (void)hipSetDevice(devices[g]);
    (void)hipDeviceSynchronize();
  }
  t0 = std::chrono::steady_clock::now();
  if (ngpus >= RT_MULTI_PARTITION_MIN && ctx[0]->accel == RT_ACCEL_OCTREE && ctx[0]->d_node &&
      ctx[0]->exact_camera) {
    // each rank 1/N of the triangles, one all-to-all
    rc = cand_exchange(ctx.data(), ngpus, &f, shared ? nullptr : comms.data());
    if (rc) goto out;
  }
  rc = per_gpu(ngpus, [&](int g) {
    int r = rt_hip_render(ctx[g], &f, g, ngpus, d_tiles[g], nullptr);
    rt_stats st;
    if (!r && (r = rt_hip_stats(ctx[g], &st)) == RT_EHITBUF)  // the buffer grew: once more
      r = rt_hip_render(ctx[g], &f, g, ngpus, d_tiles[g], nullptr);
    else if (r == RT_EDEPTH || r == RT_EZERONORMAL)
      r = RT_OK;  // reported by the stats pass below
    return r;
  });
  if (rc) goto out;
  if (ngpus > 1 && shared) {
    // the ranks' tile buffers into the gathered one, rank-major (as ncclGather)
    for (int g = 0; g < ngpus && !rc; g++) {
      // (on rank 0's stream: the assemble that follows waits for the copies)
      if (hipSetDevice(devices[g]) != hipSuccess || hipStreamSynchronize(ctx[g]->stream) != hipSuccess ||
          hipMemcpyPeerAsync(d_gather + (size_t)g * tile_floats, devices[0], d_tiles[g], devices[g],
                             tile_floats * sizeof(float), ctx[0]->stream) != hipSuccess)
        rc = rt_set_error(RT_EHIP, "gather: rank %d", g);
    }
    if (!rc) rc = rt_hip_assemble(ctx[0], &f, d_gather, ngpus, d_rgb, nullptr);
  } else if (ngpus > 1) {
    // one gather of every rank's tile buffer to device 0 over xGMI
    NCCL_TRY(ncclGroupStart());
    in_group = true;
    for (int g = 0; g < ngpus; g++) {
      (void)hipSetDevice(devices[g]);
      NCCL_TRY(ncclGather(d_tiles[g], g == 0 ? d_gather : nullptr, tile_floats, ncclFloat, 0,
                          comms[g], ctx[g]->stream));
    }
    in_group = false;
    NCCL_TRY(ncclGroupEnd());
    rc = rt_hip_assemble(ctx[0], &f, d_gather, ngpus, d_rgb, nullptr);
  } else {
    rc = rt_hip_assemble(ctx[0], &f, d_tiles[0], 1, d_rgb, nullptr);
  }
  if (rc) goto out;
  for (int g = 0; !rc && g < ngpus; g++) {
    rt_stats st;
    rc = rt_hip_stats(ctx[g], &st);
    sum.closest += st.closest;
    sum.shadow += st.shadow;
    sum.camera += st.camera;
    sum.pixels += st.pixels;
    sum.node_visits += st.node_visits;
    sum.tri_tests += st.tri_tests;
    sum.depth_overflow += st.depth_overflow;
    sum.zero_normal += st.zero_normal;
    sum.hits += st.hits;
    sum.cand_prims += st.cand_prims;
    sum.cand_entries += st.cand_entries;
    sum.cand_global += st.cand_global;
    sum.closest_node_lanes += st.closest_node_lanes;
    sum.closest_tri_lanes += st.closest_tri_lanes;
    sum.shadow_node_lanes += st.shadow_node_lanes;
    sum.shadow_tri_lanes += st.shadow_tri_lanes;
  }
  t1 = std::chrono::steady_clock::now();
  if (rc) goto out;
  h_rgb.resize(npx * 3);
  rc = rt_hip_memcpy_d2h(h_rgb.data(), d_rgb, npx * 3 * sizeof(float));
  if (!rc) rc = rt_ppm_write(output, f.width, f.height, h_rgb.data());
  if (stats) *stats = sum;
  if (render_ms) *render_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
out:
  if (in_group) (void)ncclGroupEnd();  // close the group a failed enqueue left open
  for (int g = 0; g < ngpus; g++) {
    if (comms[g]) ncclCommDestroy(comms[g]);
    if (d_tiles[g]) rt_hip_free(d_tiles[g]);
    rt_hip_destroy(ctx[g]);
  }
  if (d_gather) rt_hip_free(d_gather);
  if (d_rgb) rt_hip_free(d_rgb);
  rt_scene_free(scene);
  return rc;
}
