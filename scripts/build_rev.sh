#!/bin/bash
# Builds libfovrt.so of a git revision into abv/lib_<name>.so (A/B against the working tree):
#   scripts/build_rev.sh NAME REV [extra hipcc flags]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=${1:?name}; REV=${2:?rev}; shift 2
WT=$(mktemp -d /tmp/fovrt_rev.XXXXXX)
git -C "$ROOT" worktree add -f --detach "$WT" "$REV" > /dev/null 2>&1
P=$WT/foveated-rendering-using-ray-tracing_amd
mkdir -p "$ROOT/abv"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -w "$@" -shared \
  -o "$ROOT/abv/lib_$NAME.so" $P/csrc/k_trace.hip $P/csrc/k_image.hip $P/csrc/k_bvh.hip $P/csrc/scene.cpp \
  $P/csrc/context.cpp $P/csrc/group.cpp -lz -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
git -C "$ROOT" worktree remove --force "$WT"
