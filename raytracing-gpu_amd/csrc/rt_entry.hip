// rt_entry.hip -- per-tile entry nodes of the camera rays' packet walk
// (DESIGN.md §4 "Camera walks from per-tile entry nodes").
//
// Every camera ray of an 8x8 tile starts on the tile's patch of the film and
// passes (within the rounding of normalize(pos - point), cpu/raytracer.c:55-60)
// through the eye, so the rays of a tile lie in one thin pyramid.  Per frame,
// one thread per tile walks the octree's top levels against that pyramid and
// keeps the nodes at depth `depth` (and the leaves above it) that the pyramid
// reaches; the trace kernel's camera packet walk then starts from them --
// sorted near to far -- instead of the root, skipping the top levels' pops
// and their dependent payload fetches (every tile's walk used to start with
// the same few root-level rounds).
//
// Exactness: a node the root-started walk would enter has every ancestor's
// grown box hit by some lane's ray, so its depth-`depth` ancestor is hit and
// -- the pyramid test being conservative -- kept here; the packet walk tests
// each entry's box for every lane before pushing it (the lanes that want it,
// as for a child), and order only changes which nodes the distance pruning
// skips, never the lexicographic (new_dist, prim) winner.  The test: the
// node's box, grown by twice the camera rays' largest culling slack (the
// walk's slab test is exact up to that slack, host/rt_cull.h) plus 1e-5 of
// the eye-to-box distance (the rays' direction and origin rounding), is
// projected through the eye onto the film; the node is kept when the
// corners' bounding rectangle meets the tile's sample rectangle (grown by
// 0.02 film units + 1e-5 relative).  A box reaching the plane through the eye
// parallel to the film is always kept (the projection is not defined there).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "rt_entry.h"
#include "rt_tiles.h"
#include "../host/rt_cull.h"

namespace rte {

struct V3 {
  float x, y, z;
};
__device__ inline float dotv(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

// Can a camera ray of the tile (film rectangle [k0, k1] x [l0, l1]) reach the
// box [lo - g, hi + g]?  Conservative.
__device__ inline bool reaches(const EntryParams& p, const float4& lo, const float4& hi, float k0, float k1,
                               float l0, float l1) {
  const V3 pos{p.pos[0], p.pos[1], p.pos[2]}, w{p.w[0], p.w[1], p.w[2]};
  const V3 ku{p.ku[0], p.ku[1], p.ku[2]}, kv{p.kv[0], p.kv[1], p.kv[2]};
  // the box's farthest corner from the eye bounds the rounding allowance
  const float dx = fmaxf(fabsf(lo.x - pos.x), fabsf(hi.x - pos.x));
  const float dy = fmaxf(fabsf(lo.y - pos.y), fabsf(hi.y - pos.y));
  const float dz = fmaxf(fabsf(lo.z - pos.z), fabsf(hi.z - pos.z));
  const float g = p.grow + 1e-5f * (dx + dy + dz + p.L);
  float kmin = __builtin_inff(), kmax = -__builtin_inff(), lmin = __builtin_inff(), lmax = -__builtin_inff();
  for (int c = 0; c < 8; c++) {
    const V3 y{((c & 1) ? hi.x + g : lo.x - g) - pos.x, ((c & 2) ? hi.y + g : lo.y - g) - pos.y,
               ((c & 4) ? hi.z + g : lo.z - g) - pos.z};
    const float yw = dotv(y, w);
    // in front of the eye: y.w < 0 (the film lies at pos + w L); a corner
    // at or behind that plane -- keep the node
    if (!(yw < -1e-6f * (dx + dy + dz + 1.0f))) return true;
    const float k = p.L * dotv(y, ku) / yw, l = p.L * dotv(y, kv) / yw;
    kmin = fminf(kmin, k);
    kmax = fmaxf(kmax, k);
    lmin = fminf(lmin, l);
    lmax = fmaxf(lmax, l);
  }
  const float mk = 0.02f + 1e-5f * (fabsf(k0) + fabsf(k1)), ml = 0.02f + 1e-5f * (fabsf(l0) + fabsf(l1));
  return !(kmax < k0 - mk || kmin > k1 + mk || lmax < l0 - ml || lmin > l1 + ml);
}

__global__ __launch_bounds__(256) void entry_kernel(EntryParams p) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= p.ntiles) return;
  const int tb = rt_block_side(p.nranks);
  int tx, ty;
  rt_tile_xy(t, (uint32_t)p.rank, (uint32_t)p.nranks, (uint32_t)rt_blocks_x(p.tiles_x, tb), (uint32_t)tb, &tx, &ty);
  // the tile's samples: PPM (row, col) -> i = W - col - W/2, j = H - row - H/2,
  // samples k in {i, i + .5}, l in {j, j + .5} (rt_render.hip camera_sample)
  const float k0 = (float)(p.W - (8 * tx + 7) - p.W / 2), k1 = (float)(p.W - 8 * tx - p.W / 2) + 0.5f;
  const float l0 = (float)(p.H - (8 * ty + 7) - p.H / 2), l1 = (float)(p.H - 8 * ty - p.H / 2) + 0.5f;
  uint32_t stk[RT_ENTRY_STACK];
  uint8_t sd[RT_ENTRY_STACK];
  int sp = 0;
  uint32_t out[RT_ENTRY_MAX];
  float key[RT_ENTRY_MAX];
  uint32_t n = 0;
  bool over = false;
  stk[sp] = 0;
  sd[sp++] = 0;
  while (sp > 0 && !over) {
    --sp;
    const uint32_t ni = stk[sp];
    const int d = sd[sp];
    const float4 lo = p.node[2 * (size_t)ni], hi = p.node[2 * (size_t)ni + 1];
    if (!reaches(p, lo, hi, k0, k1, l0, l1)) continue;
    const uint32_t first = __float_as_uint(lo.w), info = __float_as_uint(hi.w);
    if ((info & RT_NODE_LEAF) || d >= p.depth) {
      if (n == RT_ENTRY_MAX) {
        over = true;
        break;
      }
      // near to far by the box centre's distance from the eye
      const float cx = 0.5f * (lo.x + hi.x) - p.pos[0], cy = 0.5f * (lo.y + hi.y) - p.pos[1],
                  cz = 0.5f * (lo.z + hi.z) - p.pos[2];
      const float k2 = cx * cx + cy * cy + cz * cz;
      uint32_t j = n++;
      while (j > 0 && key[j - 1] > k2) {
        key[j] = key[j - 1];
        out[j] = out[j - 1];
        j--;
      }
      key[j] = k2;
      out[j] = ni;
      continue;
    }
    const uint32_t cnt = RT_NODE_COUNT(info);
    if (sp + (int)cnt > RT_ENTRY_STACK) {
      over = true;
      break;
    }
    for (uint32_t c = 0; c < cnt; c++) {
      stk[sp] = first + c;
      sd[sp++] = (uint8_t)(d + 1);
    }
  }
  if (over) {  // too many: the walk starts at the root
    p.entry_n[t] = RT_ENTRY_ROOT;
    return;
  }
  p.entry_n[t] = n;
  for (uint32_t k = 0; k < n; k++) p.entry[(size_t)t * RT_ENTRY_MAX + k] = out[k];
}

}  // namespace rte

extern "C" hipError_t rt_entry_build(const EntryParams* p, hipStream_t s) {
  if (p->ntiles == 0) return hipSuccess;
  hipLaunchKernelGGL(rte::entry_kernel, dim3((p->ntiles + 255) / 256), dim3(256), 0, s, *p);
  return hipGetLastError();
}
