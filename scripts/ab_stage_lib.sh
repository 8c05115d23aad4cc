#!/bin/bash
# Interleaved stage_probe A/B of the working tree's library against exp/lib_<name>.so:
#   scripts/ab_stage_lib.sh <name> [reps] [K]
set -o pipefail
N=${1:?name}; R=${2:-3}; K=${3:-20}
for i in $(seq 1 "$R"); do
  FOVRT_LIB=exp/lib_$N.so timeout -k 10 200 python -u scripts/stage_probe.py "$K" | sed "s/^/$N /" || exit 2
  timeout -k 10 200 python -u scripts/stage_probe.py "$K" | sed "s/^/tree /" || exit 2
done
