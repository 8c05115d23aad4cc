#!/bin/bash
# Interleaved, repeated A/B of the stages alone (scripts/stage_probe.py, median of 15 per run) over
# variants given as environment settings: scripts/ab_stage.sh <reps> "name:VAR=val ..." ...
# Summary: python scripts/ab_stage_summary.py (reads gpurun_out/stage_<name>_<i>.log)
set -o pipefail
R=${1:?reps}
shift
mkdir -p gpurun_out
for i in $(seq 1 "$R"); do
  for spec in "$@"; do
    n=${spec%%:*}
    vars=${spec#*:}
    env $vars timeout -k 10 200 python scripts/stage_probe.py 15 > gpurun_out/stage_${n}_$i.log 2>&1 || exit 2
  done
done
