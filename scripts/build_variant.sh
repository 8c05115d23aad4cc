#!/bin/bash
# Builds a variant of libfovrt.so with extra compile flags into exp/ (A/B experiments with
# scripts/ab_libs.sh; exp/ is git-ignored and travels to the GPU box):
#   scripts/build_variant.sh NAME -DFLAG ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=${1:?name}; shift
P=$ROOT/foveated-rendering-using-ray-tracing_amd
mkdir -p "$ROOT/exp"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -w "$@" -shared \
  -o "$ROOT/exp/lib_$NAME.so" $P/csrc/k_trace.hip $P/csrc/k_image.hip $P/csrc/k_bvh.hip $P/csrc/scene.cpp \
  $P/csrc/context.cpp $P/csrc/group.cpp -lz -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
