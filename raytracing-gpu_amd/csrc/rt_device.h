// rt_device.h -- gfx950 device twins of the reference cpu/rt arithmetic.
//
// Every function reproduces the float (and double) operation sequence of the
// reference so the GPU image is bit-identical to cpu/rt.  The kernels are built
// with -ffp-contract=off (no v_fma contraction of a*b+c), IEEE division and
// square root (hipcc's default correctly-rounded f32 div/sqrt), denormals kept.
//
//   vector algebra   cpu/vector3.c:3-47, cpu/vector3-extern.c:5-23
//   colour algebra   cpu/colors.c:3-49
//   ray bounce       cpu/ray.c:16-25
#pragma once

#include <hip/hip_runtime.h>

namespace rt {

struct f3 {
  float x, y, z;
};

__device__ __forceinline__ f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
  return f3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
// vector3_scale multiplies scalar-first (r * a.x); float multiply commutes, so
// only the operand values matter.
__device__ __forceinline__ f3 scale(f3 a, float s) { return f3{s * a.x, s * a.y, s * a.z}; }
// (x*x' + y*y') + z*z', left to right, no fma
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// vector3_length: float sum, double sqrt, rounded to float (== correctly
// rounded sqrtf of the float sum; done in f64 to not depend on the f32 lowering)
__device__ __forceinline__ float length(f3 a) {
  float s = a.x * a.x + a.y * a.y + a.z * a.z;
  return (float)__builtin_sqrt((double)s);
}
__device__ __forceinline__ f3 normalize(f3 a) {
  float l = length(a);
  return f3{a.x / l, a.y / l, a.z / l};
}
__device__ __forceinline__ bool is_zero(f3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }

// ---- colours (float channels in [0,255]) ----
struct col {
  float r, g, b;
};

// init_color: x*255 then clamp to [0,255] with two compares (NaN passes through
// both, as in the reference: no fminf/fmaxf here).
__device__ __forceinline__ float chan(float x) {
  float y = x * 255.0f;
  if (y > 255.0f) y = 255.0f;
  if (y < 0.0f) y = 0.0f;
  return y;
}
__device__ __forceinline__ col init_color(float r, float g, float b) {
  return col{chan(r), chan(g), chan(b)};
}
__device__ __forceinline__ col color_add(col a, col b) {
  a.r += b.r;
  if (a.r > 255.0f) a.r = 255.0f;
  a.g += b.g;
  if (a.g > 255.0f) a.g = 255.0f;
  a.b += b.b;
  if (a.b > 255.0f) a.b = 255.0f;
  return a;
}
__device__ __forceinline__ col color_mul(col a, float coef) {
  return init_color(a.r / 255.0f * coef, a.g / 255.0f * coef, a.b / 255.0f * coef);
}
__device__ __forceinline__ col color_mul2(col a, col b) {
  return init_color((a.r / 255.0f) * (b.r / 255.0f), (a.g / 255.0f) * (b.g / 255.0f),
                    (a.b / 255.0f) * (b.b / 255.0f));
}

// cpu/ray.c:16-25: d' = d - N * (2 * (N . d)), N not normalised
__device__ __forceinline__ f3 bounce_dir(f3 d, f3 n) { return sub(d, scale(n, 2.0f * dot(n, d))); }

}  // namespace rt
