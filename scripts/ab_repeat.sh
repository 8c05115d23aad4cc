#!/bin/bash
# Interleaved, repeated A/B of library variants: scripts/ab_repeat.sh <reps> <lib.so>...
# Each round runs the default build, then every variant (bench workload, 10 timed frames), so slow
# drift of the box affects all of them alike. Summary: python scripts/ab_repeat_summary.py
set -o pipefail
R=${1:?reps}
shift
mkdir -p gpurun_out
for i in $(seq 1 "$R"); do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/rep_default_$i.log 2>&1 || exit 1
  for L in "$@"; do
    n=$(basename "$L" .so)
    FOVRT_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/rep_${n}_$i.log 2>&1 || exit 2
  done
done
