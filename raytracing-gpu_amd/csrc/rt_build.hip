// rt_build.hip -- octree build on the GPU.
//
// The reference builds its object-level octree on the GPU as
//   per-object Morton-style cell code (gpu/partitioning/octree.cu:140-197)
//   -> LSD radix sort (sort.tuh:137-220) -> node diff + prefix scan
//   (prefix_sum.cu:50-184) -> parallel link-up (octree.cu:245-360, 362-411).
// This is the same pipeline shape, re-designed for the per-triangle tree the
// render kernel walks (host/rt_cull.h node format):
//
//   1. count   one thread per triangle: how many references it gets.  A
//              triangle whose box fits a cell of the clip level Lc gets one
//              reference keyed by its centroid; a bigger one (ground planes,
//              long thin triangles) gets one reference per Lc cell that its
//              box overlaps and its plane crosses, with the box clipped to
//              that cell -- so its references sit deep in the tree instead of
//              inflating every ancestor box (the reference's own rule leaves
//              42-51 % of triangles near the root).
//   2. scan    rocPRIM exclusive scan of the counts -> reference offsets.
//   3. emit    63-bit Morton key (21 levels x 3 bits, octant bit a = upper
//              half of axis a, as rt_cull.h), triangle id and clipped box per
//              reference.
//   4. sort    rocPRIM radix sort of (key, reference) pairs, stable.
//   5. split   breadth-first, one thread per pending node: a node whose
//              range holds <= leaf_cap references (or is at level 21) is a
//              leaf, otherwise levels where the whole range shares one octant
//              are skipped and the range is cut into its non-empty octants
//              by binary search on the sorted keys; a scan of the child
//              counts gives every node's contiguous child block.
//   6. boxes   leaves: union of their references' boxes; interiors bottom-up,
//              level by level: union of the children.
//   7. gather  triangle records in leaf order (duplicated per reference).
//
// Correctness does not depend on the tree (culling is conservative w.r.t.
// node boxes that contain their triangles); every point of a triangle lies in
// some Lc cell it is referenced in, inside that reference's clipped box,
// inside every ancestor's box.  Deterministic: stable sort, scans, no atomics.
#include <hip/hip_runtime.h>
#include <cstring>  // before rocPRIM (its texture-cache iterator uses memset)
#include <rocprim/rocprim.hpp>

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <vector>

#include "rt_build.h"

extern "C" {
#include "../host/rt_cull.h"
}

namespace rtb {

constexpr int kLevels = 21;  // 63-bit keys

struct BuildParams {
  const float4* rec;  // ntri records, 3 float4 each (host/rt_internal.h)
  uint32_t ntri;
  float root_lo[3];
  float ext;          // root cube edge
  float pad;          // cell padding (absolute)
  int clip_level;     // Lc
};

__device__ __forceinline__ void tri_box(const float4* rec, uint32_t i, float lo[3], float hi[3],
                                        float v0[3], float n[3], float e1[3], float e2[3]) {
  float4 q0 = rec[3 * (size_t)i], q1 = rec[3 * (size_t)i + 1], q2 = rec[3 * (size_t)i + 2];
  float a[3] = {q0.x, q0.y, q0.z};
  e1[0] = q0.w; e1[1] = q1.x; e1[2] = q1.y;
  e2[0] = q1.z; e2[1] = q1.w; e2[2] = q2.x;
  for (int k = 0; k < 3; k++) {
    float c1 = a[k] + e1[k], c2 = a[k] + e2[k];
    lo[k] = fminf(a[k], fminf(c1, c2));
    hi[k] = fmaxf(a[k], fmaxf(c1, c2));
    v0[k] = a[k];
  }
  n[0] = e1[1] * e2[2] - e1[2] * e2[1];
  n[1] = e1[2] * e2[0] - e1[0] * e2[2];
  n[2] = e1[0] * e2[1] - e1[1] * e2[0];
}

__device__ __forceinline__ uint64_t spread3(uint32_t v) {
  uint64_t x = v & 0x1fffffu;
  x = (x | (x << 32)) & 0x001f00000000ffffull;
  x = (x | (x << 16)) & 0x001f0000ff0000ffull;
  x = (x | (x << 8)) & 0x100f00f00f00f00full;
  x = (x | (x << 4)) & 0x10c30c30c30c30c3ull;
  x = (x | (x << 2)) & 0x1249249249249249ull;
  return x;
}
// octant bit a = upper half of axis a: x in bit 0 of each 3-bit digit
__device__ __forceinline__ uint64_t morton(uint32_t ix, uint32_t iy, uint32_t iz) {
  return spread3(ix) | (spread3(iy) << 1) | (spread3(iz) << 2);
}

__device__ __forceinline__ int cell_of(float x, float lo, float cs, int n) {
  float f = floorf((x - lo) / cs);
  int i = f < 0.0f ? 0 : (f > (float)(n - 1) ? n - 1 : (int)f);
  return i;
}

// Cells of level Lc the triangle is referenced in; calls f(ix, iy, iz, clo, chi)
// for each (cell box padded by pad).  Returns the count.
template <class F>
__device__ uint32_t for_cells(const BuildParams& p, const float lo[3], const float hi[3],
                              const float v0[3], const float n[3], const float e1[3],
                              const float e2[3], F&& f) {
  const int nc = 1 << p.clip_level;
  const float cs = p.ext / (float)nc;
  int i0[3], i1[3];
  for (int k = 0; k < 3; k++) {
    i0[k] = cell_of(lo[k] - p.pad, p.root_lo[k], cs, nc);
    i1[k] = cell_of(hi[k] + p.pad, p.root_lo[k], cs, nc);
  }
  float an = fabsf(n[0]) + fabsf(n[1]) + fabsf(n[2]);
  // rounding bound of the float cross product, per component (a skinny
  // triangle's n can be off by far more than ulps of |n|)
  float ne[3] = {1e-6f * (fabsf(e1[1] * e2[2]) + fabsf(e1[2] * e2[1])),
                 1e-6f * (fabsf(e1[2] * e2[0]) + fabsf(e1[0] * e2[2])),
                 1e-6f * (fabsf(e1[0] * e2[1]) + fabsf(e1[1] * e2[0]))};
  uint32_t cnt = 0;
  for (int z = i0[2]; z <= i1[2]; z++)
    for (int y = i0[1]; y <= i1[1]; y++)
      for (int x = i0[0]; x <= i1[0]; x++) {
        int ix[3] = {x, y, z};
        float clo[3], chi[3], cc[3];
        for (int k = 0; k < 3; k++) {
          clo[k] = p.root_lo[k] + cs * (float)ix[k] - p.pad;
          chi[k] = p.root_lo[k] + cs * (float)(ix[k] + 1) + p.pad;
          cc[k] = 0.5f * (clo[k] + chi[k]);
        }
        // plane test, conservative: a point X of the triangle inside the cell
        // has n.(X - v0) = 0, so |n.(c - v0)| <= h |n|_1; plus the rounding
        // of n and of the dot product
        float h = 0.5f * (chi[0] - clo[0]);
        float d = n[0] * (cc[0] - v0[0]) + n[1] * (cc[1] - v0[1]) + n[2] * (cc[2] - v0[2]);
        float slack = 0.0f;
        for (int k = 0; k < 3; k++) slack += ne[k] * (fabsf(cc[k] - v0[k]) + h);
        if (fabsf(d) > (h * an + slack) * 1.001f) continue;
        cnt++;
        f(x, y, z, clo, chi);
      }
  return cnt;
}

__device__ __forceinline__ bool is_big(const BuildParams& p, const float lo[3], const float hi[3]) {
  float cs = p.ext / (float)(1 << p.clip_level);
  float e = fmaxf(hi[0] - lo[0], fmaxf(hi[1] - lo[1], hi[2] - lo[2]));
  return e > cs;
}

__global__ void k_count(BuildParams p, uint32_t* __restrict__ cnt) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.ntri) return;
  float lo[3], hi[3], v0[3], n[3], e1[3], e2[3];
  tri_box(p.rec, i, lo, hi, v0, n, e1, e2);
  uint32_t c = 1;
  if (is_big(p, lo, hi)) {
    c = for_cells(p, lo, hi, v0, n, e1, e2, [](int, int, int, const float*, const float*) {});
    if (c == 0) c = 1;  // degenerate (zero-area): keep one whole-box reference
  }
  cnt[i] = c;
}

__global__ void k_emit(BuildParams p, const uint32_t* __restrict__ off, uint64_t* __restrict__ key,
                       uint32_t* __restrict__ ref_idx, uint32_t* __restrict__ ref_prim,
                       float* __restrict__ ref_box) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.ntri) return;
  float lo[3], hi[3], v0[3], n[3], e1[3], e2[3];
  tri_box(p.rec, i, lo, hi, v0, n, e1, e2);
  uint32_t o = off[i];
  auto put = [&](uint32_t r, uint64_t k, const float* bl, const float* bh) {
    key[r] = k;
    ref_idx[r] = r;
    ref_prim[r] = i;
    for (int a = 0; a < 3; a++) {
      ref_box[6 * (size_t)r + a] = bl[a];
      ref_box[6 * (size_t)r + 3 + a] = bh[a];
    }
  };
  const int nf = 1 << kLevels;
  const float csf = p.ext / (float)nf;
  uint32_t c = 0;
  if (is_big(p, lo, hi)) {
    const int sh = kLevels - p.clip_level;
    c = for_cells(p, lo, hi, v0, n, e1, e2, [&](int x, int y, int z, const float* clo, const float* chi) {
      float bl[3], bh[3];
      for (int a = 0; a < 3; a++) {
        bl[a] = fmaxf(lo[a], clo[a]);
        bh[a] = fminf(hi[a], chi[a]);
        if (bl[a] > bh[a]) bl[a] = bh[a] = 0.5f * (clo[a] + chi[a]);  // rounding guard
      }
      // key: the cell's code, lower levels at the cell's centre
      uint32_t mid = sh > 0 ? (1u << (sh - 1)) : 0u;
      uint64_t k = morton(((uint32_t)x << sh) | mid, ((uint32_t)y << sh) | mid,
                          ((uint32_t)z << sh) | mid);
      put(o + c, k, bl, bh);
      c++;
    });
  }
  if (c == 0) {
    uint32_t ix[3];
    for (int a = 0; a < 3; a++)
      ix[a] = (uint32_t)cell_of(0.5f * (lo[a] + hi[a]), p.root_lo[a], csf, nf);
    put(o, morton(ix[0], ix[1], ix[2]), lo, hi);
  }
}

// pending node of the breadth-first split
struct Pending {
  uint32_t s, e, level;
};

__device__ __forceinline__ uint32_t digit(uint64_t k, uint32_t level) {
  return (uint32_t)(k >> (3 * (kLevels - 1 - level))) & 7u;
}

// first index in [s, e) whose digit at `level` is >= o (keys share the prefix)
__device__ __forceinline__ uint32_t lower(const uint64_t* key, uint32_t s, uint32_t e,
                                         uint32_t level, uint32_t o) {
  while (s < e) {
    uint32_t m = s + (e - s) / 2;
    if (digit(key[m], level) < o)
      s = m + 1;
    else
      e = m;
  }
  return s;
}

// 5a: classify each pending node; split[j*9 + o] = child boundaries
__global__ void k_split(const Pending* __restrict__ pend, uint32_t np, const uint64_t* __restrict__ key,
                        uint32_t leaf_cap, uint32_t* __restrict__ split,
                        uint32_t* __restrict__ level_out, uint32_t* __restrict__ nchild) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= np) return;
  Pending pd = pend[j];
  uint32_t s = pd.s, e = pd.e, L = pd.level;
  uint32_t c = 0;
  if (e - s > leaf_cap) {
    while (L < (uint32_t)kLevels && digit(key[s], L) == digit(key[e - 1], L)) L++;
    if (L < (uint32_t)kLevels) {
      uint32_t b = s;
      for (uint32_t o = 0; o < 8; o++) {
        split[9 * (size_t)j + o] = b;
        uint32_t nb = o == 7 ? e : lower(key, b, e, L, o + 1);
        if (nb > b) c++;
        b = nb;
      }
      split[9 * (size_t)j + 8] = e;
    }
  }
  level_out[j] = L;
  nchild[j] = c;
}

// 5b: write the node records' link fields and the next pending list
__global__ void k_link(const Pending* __restrict__ pend, uint32_t np, const uint32_t* __restrict__ split,
                       const uint32_t* __restrict__ level, const uint32_t* __restrict__ nchild,
                       const uint32_t* __restrict__ coff, uint32_t node_base, uint32_t next_base,
                       float4* __restrict__ node, Pending* __restrict__ next,
                       uint32_t* __restrict__ leaf_stats) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= np) return;
  Pending pd = pend[j];
  uint32_t c = nchild[j];
  float4 lo = make_float4(0, 0, 0, 0), hi = lo;
  if (c == 0) {
    lo.w = __uint_as_float(pd.s);
    hi.w = __uint_as_float(RT_NODE_LEAF | (pd.e - pd.s));
    atomicAdd(&leaf_stats[0], 1u);
    atomicMax(&leaf_stats[1], pd.e - pd.s);
  } else {
    uint32_t first = next_base + coff[j], mask = 0, k = 0;
    for (uint32_t o = 0; o < 8; o++) {
      uint32_t b = split[9 * (size_t)j + o], nb = split[9 * (size_t)j + o + 1];
      if (nb > b) {
        mask |= 1u << o;
        next[coff[j] + k] = Pending{b, nb, level[j] + 1};
        k++;
      }
    }
    lo.w = __uint_as_float(first);
    hi.w = __uint_as_float(c | (mask << 8));
  }
  node[2 * (size_t)(node_base + j)] = lo;
  node[2 * (size_t)(node_base + j) + 1] = hi;
}

// 6: node boxes of one breadth-first level [base, base + n)
__global__ void k_boxes(float4* __restrict__ node, uint32_t base, uint32_t n,
                        const uint32_t* __restrict__ sorted_ref, const float* __restrict__ ref_box) {
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  size_t ni = base + j;
  float4 lo = node[2 * ni], hi = node[2 * ni + 1];
  uint32_t first = __float_as_uint(lo.w), info = __float_as_uint(hi.w);
  float bl[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, bh[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  if (info & RT_NODE_LEAF) {
    uint32_t cnt = RT_LEAF_COUNT(info);
    for (uint32_t k = 0; k < cnt; k++) {
      const float* b = ref_box + 6 * (size_t)sorted_ref[first + k];
      for (int a = 0; a < 3; a++) {
        bl[a] = fminf(bl[a], b[a]);
        bh[a] = fmaxf(bh[a], b[3 + a]);
      }
    }
  } else {
    uint32_t cnt = RT_NODE_COUNT(info);
    for (uint32_t k = 0; k < cnt; k++) {
      float4 cl = node[2 * (size_t)(first + k)], ch = node[2 * (size_t)(first + k) + 1];
      bl[0] = fminf(bl[0], cl.x); bl[1] = fminf(bl[1], cl.y); bl[2] = fminf(bl[2], cl.z);
      bh[0] = fmaxf(bh[0], ch.x); bh[1] = fmaxf(bh[1], ch.y); bh[2] = fmaxf(bh[2], ch.z);
    }
  }
  node[2 * ni] = make_float4(bl[0], bl[1], bl[2], lo.w);
  node[2 * ni + 1] = make_float4(bh[0], bh[1], bh[2], hi.w);
}

// 7: records in leaf order
__global__ void k_gather(const float4* __restrict__ rec, const uint32_t* __restrict__ sorted_ref,
                         const uint32_t* __restrict__ ref_prim, uint32_t nref,
                         float4* __restrict__ out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nref) return;
  uint32_t p = ref_prim[sorted_ref[i]];
  out[3 * (size_t)i] = rec[3 * (size_t)p];
  out[3 * (size_t)i + 1] = rec[3 * (size_t)p + 1];
  out[3 * (size_t)i + 2] = rec[3 * (size_t)p + 2];
}

}  // namespace rtb

#define BTRY(expr)                       \
  do {                                   \
    hipError_t e_ = (expr);              \
    if (e_ != hipSuccess) {              \
      err = e_;                          \
      goto done;                         \
    }                                    \
  } while (0)

static unsigned blocks(size_t n) { return (unsigned)((n + 255) / 256); }

extern "C" hipError_t rt_device_build_octree(const float4* d_rec, uint32_t ntri,
                                             const float scene_lo[3], const float scene_hi[3],
                                             const rt_device_build_opts* opts, hipStream_t s,
                                             rt_device_tree* out) {
  using namespace rtb;
  hipError_t err = hipSuccess;
  *out = rt_device_tree{};
  uint64_t *key = nullptr, *key2 = nullptr;
  uint32_t *cnt = nullptr, *off = nullptr, *ref = nullptr,
           *ref2 = nullptr, *ref_prim = nullptr, *split = nullptr, *lvl = nullptr,
           *nch = nullptr, *coff = nullptr, *leaf_stats = nullptr;
  float* ref_box = nullptr;
  Pending *pa = nullptr, *pb = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  float4* node = nullptr;
  float4* tri = nullptr;
  uint32_t nref = 0, nnode = 0;
  std::vector<uint32_t> level_base, level_count;
  BuildParams p{};
  {
    double ext = 0;
    for (int a = 0; a < 3; a++) ext = std::fmax(ext, (double)scene_hi[a] - scene_lo[a]);
    ext = ext * 1.0001 + 1e-6;
    for (int a = 0; a < 3; a++)
      p.root_lo[a] = (float)(0.5 * ((double)scene_lo[a] + scene_hi[a]) - 0.5 * ext);
    p.ext = (float)ext;
    p.pad = (float)(ext * 4e-6);
    p.rec = d_rec;
    p.ntri = ntri;
    p.clip_level = opts->clip_level < 0 ? 0 : (opts->clip_level > kLevels ? kLevels : opts->clip_level);
  }
  uint32_t leaf_cap = opts->leaf_cap < 1 ? 1u : (uint32_t)opts->leaf_cap;

  // 1-2: reference counts and offsets
  BTRY(hipMalloc((void**)&cnt, (size_t)(ntri + 1) * 4));
  BTRY(hipMalloc((void**)&off, (size_t)(ntri + 1) * 4));
  BTRY(hipMemsetAsync(cnt + ntri, 0, 4, s));
  hipLaunchKernelGGL(k_count, dim3(blocks(ntri)), dim3(256), 0, s, p, cnt);
  BTRY(hipGetLastError());
  BTRY(rocprim::exclusive_scan(nullptr, tmp_bytes, cnt, off, 0u, (size_t)(ntri + 1), rocprim::plus<uint32_t>(), s));
  BTRY(hipMalloc(&tmp, tmp_bytes));
  BTRY(rocprim::exclusive_scan(tmp, tmp_bytes, cnt, off, 0u, (size_t)(ntri + 1), rocprim::plus<uint32_t>(), s));
  BTRY(hipMemcpyAsync(&nref, off + ntri, 4, hipMemcpyDeviceToHost, s));
  BTRY(hipStreamSynchronize(s));
  BTRY(hipFree(tmp));
  tmp = nullptr;

  // 3-4: keyed references, sorted
  BTRY(hipMalloc((void**)&key, (size_t)nref * 8));
  BTRY(hipMalloc((void**)&key2, (size_t)nref * 8));
  BTRY(hipMalloc((void**)&ref, (size_t)nref * 4));
  BTRY(hipMalloc((void**)&ref2, (size_t)nref * 4));
  BTRY(hipMalloc((void**)&ref_prim, (size_t)nref * 4));
  BTRY(hipMalloc((void**)&ref_box, (size_t)nref * 24));
  hipLaunchKernelGGL(k_emit, dim3(blocks(ntri)), dim3(256), 0, s, p, off, key, ref, ref_prim, ref_box);
  BTRY(hipGetLastError());
  tmp_bytes = 0;
  BTRY(rocprim::radix_sort_pairs(nullptr, tmp_bytes, key, key2, ref, ref2, (size_t)nref, 0u, 3u * kLevels, s));
  BTRY(hipMalloc(&tmp, tmp_bytes));
  BTRY(rocprim::radix_sort_pairs(tmp, tmp_bytes, key, key2, ref, ref2, (size_t)nref, 0u, 3u * kLevels, s));
  BTRY(hipFree(tmp));
  tmp = nullptr;
  BTRY(hipFree(cnt));
  cnt = nullptr;

  // 5: breadth-first split; every interior node has >= 2 children, so
  // nodes < 2 x references
  {
    size_t cap = 2 * (size_t)nref + 1;
    BTRY(hipMalloc((void**)&node, cap * 32));
    BTRY(hipMalloc((void**)&pa, (size_t)nref * sizeof(Pending) + sizeof(Pending)));
    BTRY(hipMalloc((void**)&pb, (size_t)nref * sizeof(Pending) + sizeof(Pending)));
    BTRY(hipMalloc((void**)&split, ((size_t)nref + 1) * 9 * 4));
    BTRY(hipMalloc((void**)&lvl, ((size_t)nref + 1) * 4));
    BTRY(hipMalloc((void**)&nch, ((size_t)nref + 2) * 4));
    BTRY(hipMalloc((void**)&coff, ((size_t)nref + 2) * 4));
    BTRY(hipMalloc((void**)&leaf_stats, 8));
    BTRY(hipMemsetAsync(leaf_stats, 0, 8, s));
    Pending root{0, nref, 0};
    BTRY(hipMemcpyAsync(pa, &root, sizeof root, hipMemcpyHostToDevice, s));
    uint32_t np = 1;
    tmp_bytes = 0;
    BTRY(rocprim::exclusive_scan(nullptr, tmp_bytes, nch, coff, 0u, (size_t)(nref + 2), rocprim::plus<uint32_t>(), s));
    BTRY(hipMalloc(&tmp, tmp_bytes));
    while (np > 0) {
      hipLaunchKernelGGL(k_split, dim3(blocks(np)), dim3(256), 0, s, pa, np, key2, leaf_cap, split,
                         lvl, nch);
      BTRY(hipGetLastError());
      BTRY(hipMemsetAsync(nch + np, 0, 4, s));
      size_t tb = tmp_bytes;
      BTRY(rocprim::exclusive_scan(tmp, tb, nch, coff, 0u, (size_t)(np + 1), rocprim::plus<uint32_t>(), s));
      uint32_t nnext = 0;
      BTRY(hipMemcpyAsync(&nnext, coff + np, 4, hipMemcpyDeviceToHost, s));
      hipLaunchKernelGGL(k_link, dim3(blocks(np)), dim3(256), 0, s, pa, np, split, lvl, nch, coff,
                         nnode, nnode + np, node, pb, leaf_stats);
      BTRY(hipGetLastError());
      BTRY(hipStreamSynchronize(s));
      level_base.push_back(nnode);
      level_count.push_back(np);
      nnode += np;
      if (nnode + nnext > cap) {
        err = hipErrorInvalidValue;  // cannot happen (>= 2 children per interior)
        goto done;
      }
      std::swap(pa, pb);
      np = nnext;
    }
  }

  // 6: boxes, deepest level first
  for (size_t l = level_base.size(); l-- > 0;) {
    hipLaunchKernelGGL(k_boxes, dim3(blocks(level_count[l])), dim3(256), 0, s, node,
                       level_base[l], level_count[l], ref2, ref_box);
    BTRY(hipGetLastError());
  }

  // 7: records in leaf order
  BTRY(hipMalloc((void**)&tri, (size_t)(nref ? nref : 1) * 48));
  hipLaunchKernelGGL(k_gather, dim3(blocks(nref)), dim3(256), 0, s, d_rec, ref2, ref_prim, nref, tri);
  BTRY(hipGetLastError());
  BTRY(hipStreamSynchronize(s));

  // compact node array into a plain allocation of the final size
  {
    float4* fin = nullptr;
    BTRY(hipMalloc((void**)&fin, (size_t)nnode * 32));
    BTRY(hipMemcpyAsync(fin, node, (size_t)nnode * 32, hipMemcpyDeviceToDevice, s));
    BTRY(hipStreamSynchronize(s));
    out->node = fin;
  }
  out->tri = tri;
  tri = nullptr;
  out->nref = nref;
  out->nnode = nnode;
  out->depth = (uint32_t)level_base.size();
  {
    uint32_t ls[2] = {0, 0};
    BTRY(hipMemcpy(ls, leaf_stats, 8, hipMemcpyDeviceToHost));
    out->leaves = ls[0];
    out->max_leaf = ls[1];
  }

done:
  if (tmp) (void)hipFree(tmp);
  for (void* q : {(void*)cnt, (void*)off, (void*)key, (void*)key2, (void*)ref, (void*)ref2,
                  (void*)ref_prim, (void*)split, (void*)lvl, (void*)nch, (void*)coff,
                  (void*)ref_box, (void*)pa, (void*)pb, (void*)node, (void*)leaf_stats})
    if (q) (void)hipFree(q);
  (void)hipStreamSynchronize(s);
  if (tri) (void)hipFree(tri);
  if (err != hipSuccess && out->node) {
    (void)hipFree(out->node);
    *out = rt_device_tree{};
  }
  return err;
}
