/* rt_internal.h -- shared declarations of the host C side (not installed). */
#ifndef RT_INTERNAL_H
#define RT_INTERNAL_H

#include <stddef.h>
#include <stdint.h>

#include "rt_hip.h"
#include "rt_hip_test.h"
#include "rt_scene.h"

#ifdef __cplusplus
extern "C" {
#endif

int rt_set_error(int code, const char *fmt, ...);
/* rt_frame_from_camera without the even-size rule (the gpu/rt
 * compatibility mode's 3x frame) */
int rt_frame_from_camera_any(const rt_camera *cam, rt_frame *out);

/* ---- reference-exact host math (cpu/vector3*.c), no contraction ---- */
rt_vec3 rt_v_sub(rt_vec3 a, rt_vec3 b);
rt_vec3 rt_v_add(rt_vec3 a, rt_vec3 b);
rt_vec3 rt_v_cross(rt_vec3 a, rt_vec3 b);
rt_vec3 rt_v_scale(rt_vec3 a, float s);
float rt_v_length(rt_vec3 a);
rt_vec3 rt_v_normalize(rt_vec3 a);

/* ---- flattened device image of a scene (built on the host) ----
 *
 * Triangle record (48 B, 3 x float4), in traversal order:
 *   q0 = v0.x v0.y v0.z e1.x
 *   q1 = e1.y e1.z e2.x e2.y
 *   q2 = e2.z  bits(prim)  bits(object)  flags
 * flags bit 0 (RT_REC_ZERO_RISK_BIT): the object has a triangle whose
 * interpolated normal can be exactly zero (rt_tri_normal_can_vanish).
 * prim = global triangle index in (object, LIFO triangle) order, which is the
 * tie-break key of cpu/hit.c:59,82.  e1/e2 are the
 * exact subtractions cpu/hit.c:16-17 performs.
 * Normals (36 B per prim, indexed by prim): the three vertex normals
 * normalised exactly as cpu/hit.c:11-13 does per test.
 *
 * Octree node (32 B, 2 x float4): encoding in rt_cull.h (shared with the
 * device traversal).
 */
typedef struct rt_flat_scene {
  size_t ntri;              /* scene triangles (prims)                       */
  size_t nrec;              /* triangle records (>= ntri with duplicates)    */
  float *tri;               /* nrec * 12 floats                              */
  float *nrm;               /* ntri * 9 floats                               */
  size_t nobj;
  float *mat;               /* nobj * 12: ka.xyz kd.xyz ks.xyz ns nr pad      */
  size_t nlight;
  float *light;             /* nlight * 8: type r g b v.xyz pad               */
  size_t nnode;
  float *node;              /* nnode * 8                                     */
  uint32_t root_count;      /* 1 (root is node 0) or 0 for FLAT              */
  float scene_lo[3], scene_hi[3];
  size_t leaves, max_depth, max_leaf;
} rt_flat_scene;

#define RT_TRI_FLOATS 12
#define RT_NODE_FLOATS 8
#define RT_MAT_FLOATS 12
#define RT_LIGHT_FLOATS 8


#define RT_REC_ZERO_RISK_BIT 1u /* = RT_REC_ZERO_RISK of csrc/rt_kernels.h */

int rt_flatten(const rt_scene *scene, int accel, rt_flat_scene *out);
int rt_tri_normal_can_vanish(const float *nrm9);
void rt_flat_free(rt_flat_scene *f);
int rt_flat_validate(const rt_flat_scene *f);

#ifdef __cplusplus
}
#endif
#endif
