#!/bin/bash
# A/B of library variants on the bench workload: scripts/ab_libs.sh <lib.so>... (default build first)
set -o pipefail
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/ab_default.log 2>&1 || exit 1
for L in "$@"; do
  n=$(basename "$L" .so)
  FOVRT_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/ab_$n.log 2>&1 || exit 2
done
