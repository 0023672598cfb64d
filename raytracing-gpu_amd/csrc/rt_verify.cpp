// rt_verify.cpp -- test, measurement and verification hooks of
// include/rt_hip_test.h: the tile map's self-check, the device tree's
// validator, phase timing and per-item clocks, the shadow re-shading check,
// the closest-hit and shadow probes, the per-frame device checks, the light
// buffers' host survey.
#include "rt_ctx.h"

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
