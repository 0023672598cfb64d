/*
 * rt_main.c -- the `rt` command line, drop-in for the reference cpu/rt:
 *   rt file.svati output.ppm                  (cpu/rt.c:5-10, same usage error)
 * Optional flags may follow the two positional arguments:
 *   --gpus N          tile the frame over N GPUs of this node (RCCL gather)
 *   --accel flat|octree|octree_gpu
 *   --stats           print query counters and render time to stderr
 * Errors exit with status 1 via errx(), as the reference does.
 */
#include <err.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt_hip.h"

int main(int argc, char *argv[])
{
  if (argc < 3)
    errx(1, "usage: %s file.svati output.ppm", argv[0]);
  int gpus = 1, accel = -1, want_stats = 0;
  for (int i = 3; i < argc; i++)
  {
    if (!strcmp(argv[i], "--gpus") && i + 1 < argc)
      gpus = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--accel") && i + 1 < argc)
    {
      const char *a = argv[++i];
      accel = !strcmp(a, "flat")         ? RT_ACCEL_FLAT
              : !strcmp(a, "octree")     ? RT_ACCEL_OCTREE
              : !strcmp(a, "octree_gpu") ? RT_ACCEL_OCTREE_GPU
                                         : -2;
      if (accel == -2)
        errx(1, "unknown accel %s", a);
    }
    else if (!strcmp(argv[i], "--stats"))
      want_stats = 1;
    else
      errx(1, "usage: %s file.svati output.ppm [--gpus N] [--accel flat|octree|octree_gpu] [--stats]",
           argv[0]);
  }
  rt_stats st;
  double ms = 0;
  int rc = rt_raytrace_multi(argv[1], argv[2], gpus, accel, &st, &ms);
  /* input/output and parse errors print the reference's own text and
   * newline (cpu/parser.c:70-71,110-111, cpu/parse_obj.c:80-81,
   * cpu/printer.c:6-7: errx(1, "%s\n", ...)); device errors name the code */
  if (rc == RT_EIO || rc == RT_EPARSE)
    errx(1, "%s\n", rt_last_error());
  if (rc)
    errx(1, "%s: %s", rt_strerror(rc), rt_last_error());
  if (want_stats)
    fprintf(stderr, "closest_hit_queries=%llu shadow_queries=%llu render_ms=%.3f mrays_per_s=%.2f\n",
            st.closest, st.shadow, ms, ms > 0 ? (st.closest + st.shadow) / (ms * 1e3) : 0.0);
  return 0;
}
