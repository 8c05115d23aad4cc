#!/bin/bash
# Sibson alone at 4K (scripts/sibson_probe.py) for library variants, interleaved: scripts/ab_sibson.sh <reps> <lib.so>...
set -o pipefail
R=${1:?reps}; shift
for i in $(seq 1 "$R"); do
  for L in "$@"; do
    echo -n "$(basename $L .so) "; FOVRT_LIB=$L timeout -k 10 60 python scripts/sibson_probe.py 20 || exit 1
  done
done
