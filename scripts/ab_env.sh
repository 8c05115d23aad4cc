#!/bin/bash
# Interleaved, repeated A/B of variants given as environment settings (bench workload, 10 timed frames):
#   scripts/ab_env.sh <reps> "name:VAR=val VAR2=val" ...   (FOVRT_LIB=exp/lib_x.so selects a library build)
# Each round runs every variant once, so slow drift of the box affects all of them alike.
# Summary: python scripts/ab_repeat_summary.py (reads gpurun_out/rep_<name>_<i>.log)
set -o pipefail
R=${1:?reps}
shift
mkdir -p gpurun_out
for i in $(seq 1 "$R"); do
  for spec in "$@"; do
    n=${spec%%:*}
    vars=${spec#*:}
    env $vars timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 --warmup 20 > gpurun_out/rep_${n}_$i.log 2>&1 || exit 2
  done
done
