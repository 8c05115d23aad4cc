#!/bin/bash
# Round 5: rebuild hitch variants. Host tree released at init (FOVRT_BVH_RELEASE), warm-up build at init
# (FOVRT_BVH_WARMUP), eager code-object loading, each with phase timing (FOVRT_BVH_PHASES).
set -o pipefail
mkdir -p gpurun_out
run() { local name=$1; shift; env FOVRT_BVH_PHASES=1 "$@" timeout -k 10 120 python scripts/rebuild_probe.py $SC > gpurun_out/rbe_$name.log 2>&1 || exit 3; }
SC="1 2"; run base
SC="1 2"; run rel FOVRT_BVH_RELEASE=1
SC="1 2"; run rel_warm FOVRT_BVH_RELEASE=1 FOVRT_BVH_WARMUP=1
SC="1 2"; run eager_rel_warm FOVRT_BVH_RELEASE=1 FOVRT_BVH_WARMUP=1 HIP_ENABLE_DEFERRED_LOADING=0
SC="2 1"; run rev
for f in base rel rel_warm eager_rel_warm rev; do
  echo "== $f"; grep -v "^bvh phase\|^bvh entry" gpurun_out/rbe_$f.log
  grep "^bvh entry" gpurun_out/rbe_$f.log | awk '{print $NF, $(NF-1)}' | sort -rn | head -3 | tr '\n' ' '; echo
done
