/* asan_scene.c -- host-only scene lifecycle under AddressSanitizer + UBSan
 * (tests/test_host.py::test_scene_lifecycle_asan builds it from the product's
 * host C sources; no GPU, no HIP).
 *
 * Loads every reference scene given on the command line, writes and reloads
 * it as .svati and .obj, appends an .obj, flattens and builds both octrees,
 * runs the host traversal model, edits it in place the supported way (the
 * camera size; an object's triangle_count set to 0 -- how tools/noground.py
 * drops C5's ground quad without touching the objects array) and frees
 * everything.  Any heap error (double free, overflow, leak with
 * detect_leaks=1) aborts with ASan's report. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt_hip.h"
#include "rt_internal.h"

#define CHECK(x)                                                              \
  do {                                                                        \
    int rc_ = (x);                                                            \
    if (rc_) {                                                                \
      fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_,   \
              rt_last_error());                                               \
      return 1;                                                               \
    }                                                                         \
  } while (0)

static int exercise(rt_scene *s, const char *tmp)
{
  char p1[512], p2[512];
  snprintf(p1, sizeof p1, "%s/a.svati", tmp);
  snprintf(p2, sizeof p2, "%s/a.obj", tmp);
  s->camera.width = 32;
  s->camera.height = 18;
  CHECK(rt_scene_write_svati(s, p1));
  CHECK(rt_scene_write_obj(s, p2));
  rt_scene *a = NULL, *b = NULL;
  CHECK(rt_scene_load_svati(p1, &a));
  CHECK(rt_scene_load_obj(p2, &b));
  if (rt_scene_triangle_count(a) != rt_scene_triangle_count(s) ||
      rt_scene_triangle_count(b) != rt_scene_triangle_count(s))
  {
    fprintf(stderr, "round trip changed the triangle count\n");
    return 1;
  }
  CHECK(rt_scene_append_obj(a, p2));
  for (int accel = RT_ACCEL_FLAT; accel <= RT_ACCEL_OCTREE; accel++)
  {
    rt_flat_scene f;
    CHECK(rt_flatten(a, accel, &f));
    CHECK(rt_flat_validate(&f));
    rt_flat_free(&f);
  }
  CHECK(rt_accel_validate(a, RT_ACCEL_OCTREE));
  rt_accel_probe_result pr;
  CHECK(rt_accel_probe(a, RT_ACCEL_OCTREE, 7, 1, &pr));
  if (pr.mismatches)
  {
    fprintf(stderr, "probe mismatches %llu\n", pr.mismatches);
    return 1;
  }
  rt_scene_free(a);
  rt_scene_free(b);
  /* drop an object's triangles in place (an object block of 0 triangles has
   * no .svati form: the reference grammar reads its material keys as
   * top-level tokens, cpu/parse_obj.c:51) and build from what is left */
  if (s->object_count > 1)
  {
    s->objects[0].triangle_count = 0;
    rt_flat_scene f;
    CHECK(rt_flatten(s, RT_ACCEL_OCTREE, &f));
    CHECK(rt_flat_validate(&f));
    rt_flat_free(&f);
  }
  return 0;
}

int main(int argc, char **argv)
{
  if (argc < 3)
  {
    fprintf(stderr, "usage: %s tmpdir scene.svati...\n", argv[0]);
    return 2;
  }
  for (int i = 2; i < argc; i++)
  {
    rt_scene *s = NULL;
    CHECK(rt_scene_load_svati(argv[i], &s));
    if (exercise(s, argv[1]))
      return 1;
    rt_scene_free(s);
  }
  rt_scene *syn = NULL;
  CHECK(rt_scene_synthetic(3, 2, 400, 0x5EEDull, 64, 36, &syn));
  if (exercise(syn, argv[1]))
    return 1;
  rt_scene_free(syn);
  /* error paths free what they allocated */
  rt_scene *bad = NULL;
  if (rt_scene_load_svati("/nonexistent.svati", &bad) == 0 || bad)
    return 1;
  printf("asan scene lifecycle ok\n");
  return 0;
}
