/* rt_error.c -- error codes and the per-thread detail message (rt_scene.h). */
#include <stdarg.h>
#include <stdio.h>

#include "rt_internal.h"

static _Thread_local char last_error[512] = "";

const char *rt_strerror(int code)
{
  switch (code)
  {
  case RT_OK: return "success";
  case RT_EINVAL: return "invalid argument";
  case RT_EIO: return "I/O error";
  case RT_EPARSE: return "parse error";
  case RT_ENOMEM: return "out of host memory";
  case RT_EHIP: return "HIP runtime error";
  case RT_ENODEV: return "no usable gfx950 device";
  case RT_EDEPTH: return "reflection depth or traversal stack overflow";
  case RT_ERCCL: return "RCCL error";
  case RT_EZERONORMAL: return "zero interpolated normal (cpu/hit.c:79,99 not reproduced)";
  case RT_EHITBUF: return "hit-record buffer overflow (grown; render again)";
  case RT_EINEXACT: return "inexact tuning knob active (cpu/rt parity not guaranteed)";
  default: return "unknown error";
  }
}

const char *rt_last_error(void) { return last_error; }

int rt_set_error(int code, const char *fmt, ...)
{
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(last_error, sizeof last_error, fmt, ap);
  va_end(ap);
  return code;
}
