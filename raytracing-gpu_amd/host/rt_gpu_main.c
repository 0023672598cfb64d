/*
 * rt_gpu_main.c -- the `rt_gpu` command line, drop-in for the reference's
 * gpu/rt (gpu/rt.cpp:56-97): `rt_gpu file.svati output.png`, exactly two
 * arguments (the same usage error), gpu/rt's output semantics (3x3
 * supersampling, uint8 colours, <= 11 bounces, RGBA PNG; csrc/rt_render.hip
 * compat_kernel).  An optional third argument `--accel flat|octree|octree_gpu`
 * picks the acceleration (default: by scene size, as `rt`).
 */
#include <err.h>
#include <string.h>

#include "rt_hip.h"

int main(int argc, char *argv[])
{
  int accel = -1;
  if (argc == 5 && !strcmp(argv[3], "--accel"))
  {
    accel = !strcmp(argv[4], "flat")         ? RT_ACCEL_FLAT
            : !strcmp(argv[4], "octree")     ? RT_ACCEL_OCTREE
            : !strcmp(argv[4], "octree_gpu") ? RT_ACCEL_OCTREE_GPU
                                             : -2;
    if (accel == -2)
      errx(1, "unknown accel %s", argv[4]);
  }
  else if (argc != 3)
    errx(1, "usage: %s file.svati output.png", argv[0]);
  int rc = rt_raytrace_gpu(argv[1], argv[2], accel);
  if (rc == RT_EIO || rc == RT_EPARSE)
    errx(1, "%s\n", rt_last_error());
  if (rc)
    errx(1, "%s: %s", rt_strerror(rc), rt_last_error());
  return 0;
}
