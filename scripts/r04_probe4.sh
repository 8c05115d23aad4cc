#!/bin/bash
# BVH warm-up (tests, rebuild probe); Sibson strip cursor change (tests) and its 4 / 5 waves-per-SIMD builds (gaze probe).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "bvh or BVH or rebuild or positions or sibson or Sibson" > gpurun_out/p4_tests.log 2>&1 || { tail -30 gpurun_out/p4_tests.log; exit 5; }
tail -1 gpurun_out/p4_tests.log
timeout -k 10 120 python scripts/rebuild_probe.py > gpurun_out/r04e_rebuild_probe.txt 2>&1 || exit 1
cat gpurun_out/r04e_rebuild_probe.txt
for o in 4 5; do echo "occ $o"; FOVRT_SIB_STRIP_OCC=$o timeout -k 10 300 python scripts/gaze_probe.py c 90 180 || exit 8; done
FOVRT_SIB_STRIP_OCC=5 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "sibson or Sibson" > gpurun_out/p4_occ5.log 2>&1 || { tail -30 gpurun_out/p4_occ5.log; exit 6; }
tail -1 gpurun_out/p4_occ5.log
