// rt_lists.cpp -- the camera rays' candidate lists on the host side
// (DESIGN.md §2 "Exact camera rays", §4 "Candidate-list kernels"): frame
// constants, the per-rank build (cand_prepare: fast path -> classification ->
// emission -> refinement -> compaction -> sort -> offsets -> work order), the
// triangle-parallel produce / consume of an N-rank frame, the host
// re-derivation that verifies them, and the host surveys.
#include "rt_ctx.h"

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
  // headroom past a new camera's estimate (the last build's size + 1/4 +
  // 4096, cand_prepare): growing a buffer frees the old one, and hipFree
  // waits for the device -- a whole frame's host lead lost mid-build
  size_t n = need + need / 2 + 8192;
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
  lists_changed(c);  // the lists change
  return RT_OK;
}

// the trace's item-clock sum in the frame counters (KParams::cost_sum)
unsigned long long* cost_sum_of(rt_hip_ctx* c) {
  return (unsigned long long*)((char*)c->d_counter + kItemCounterBytes + kStatBytes + kHitCounterBytes);
}

// Frame constants of the candidate lists for rank/nranks (no device work).
int cand_params(const rt_frame* f, const float scene_c[3], float scene_r, float eps_ulps,
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
  bytes += bytes / 2 + 65536;  // headroom (as grow_dev): a new camera's sort is a little longer
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
int cand_prepare(rt_hip_ctx* c, const rt_frame* f, KParams* kp, hipStream_t s, int compat) {
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
      c->kept_pending = 0;
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
  if (c->kept_pending && c->ev_kept && hipEventQuery(c->ev_kept) == hipSuccess) {
    c->kept = *c->h_kept;
    c->kept_for = c->kept_pend;
    c->kept_ready = 1;
    c->kept_pending = 0;
  }
  // the kept entries compacted before the sort (the refinement drops ~55 %
  // of them on C5): an asynchronous build takes the kept count of the same
  // frame's earlier build; a fresh frame (a new camera: the build read its
  // total back anyway) reads its own back after the compaction's scan -- one
  // more short host wait instead of sorting the dropped entries
  // (for a new camera the last frame's kept count + 1/16: the scatter writes
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
      const size_t cap = 2 * ((size_t)nw + nw / 2) + 1024;  // headroom (as grow_dev)
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
      cap = kept_same ? c->kept : c->kept + c->kept / 16 + 4096;
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
  if (RT_COMPACT_LISTS && c->cand_refine && !compat && !kept_now && (!kept_same || est_shape) &&
      !(c->kept_pending && c->kept_pend.same(f, kp->rank, kp->nranks))) {
    // this frame's kept count -- and after an estimated-shape build its
    // counters (bounds_kernel's snapshot) -- for the later builds, read back
    // without waiting
    if (!c->h_kept) HIP_TRY(hipHostMalloc((void**)&c->h_kept, 9 * sizeof(uint32_t), hipHostMallocDefault));
    if (!c->ev_kept) HIP_TRY(hipEventCreateWithFlags(&c->ev_kept, hipEventDisableTiming));
    HIP_TRY(hipMemcpyAsync(c->h_kept, c->d_cand_start + nt, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    if (est_shape) HIP_TRY(hipMemcpyAsync(c->h_kept + 1, c->d_cand_ctr + 16, 8 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipEventRecord(c->ev_kept, s));
    // (the count in hand, if any, stays usable -- for this size and split --
    // until this one arrives: the host runs frames ahead of the device)
    c->kept_pend.set(f, kp->rank, kp->nranks);
    c->kept_pending = 1;
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
  // build's own total); then a stable partition by rank.  The consumer's
  // stable sort by tile gives each tile the same entries as the rank's own
  // build -- in the producers' interleaved slice order, not necessarily the
  // same order within a tile, which the render does not depend on (the
  // winner is the lexicographic (new_dist, prim) minimum, rt_render.hip
  // consider_exact)
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
