#!/bin/bash
# Round 6: the refraction-class chunk (FOVRT_SHADE_CHUNK_REFR) with the traversal loop's early exit, C3.
set -o pipefail
mkdir -p gpurun_out
bash scripts/ab_bench.sh r06c3 3 def:- c16:FOVRT_SHADE_CHUNK_REFR=16 c32:FOVRT_SHADE_CHUNK_REFR=32 || exit 2
echo done
