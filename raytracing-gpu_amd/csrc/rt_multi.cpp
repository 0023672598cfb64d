// rt_multi.cpp -- rt_raytrace_multi / rt_raytrace_multi_dev: the frame's
// tiles over N GPUs of this node, one host thread per GPU, the triangle-
// parallel candidate lists' all-to-all (grouped ncclSend / ncclRecv, or
// device memcpys when ranks share a device) and one RCCL gather to rank 0.
#include "rt_ctx.h"

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

