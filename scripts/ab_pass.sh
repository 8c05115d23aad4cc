#!/bin/bash
# One pass alone at 4K for library variants, interleaved: scripts/ab_pass.sh <pass> <reps> <lib.so>...
set -o pipefail
P=${1:?pass}; R=${2:?reps}; shift 2
for i in $(seq 1 "$R"); do
  for L in "$@"; do
    echo -n "$(basename $L .so) "; FOVRT_LIB=$L timeout -k 10 60 python scripts/pass_probe.py "$P" 20 || exit 1
  done
done
