#!/bin/bash
# Build a variant of librtgpu.so with extra compile flags into
# raytracing-gpu_amd/lib/var_<name>/ (A/B measurements; load it with
# RTGPU_LIB=raytracing-gpu_amd/lib/var_<name>/librtgpu.so).
#   tools/build_variant.sh <name> "<-Dflags>"
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
make -s -C "$R/raytracing-gpu_amd" OUT="$R/raytracing-gpu_amd/lib/var_$1" XFLAGS="$2" -j8 \
  "$R/raytracing-gpu_amd/lib/var_$1/librtgpu.so"
