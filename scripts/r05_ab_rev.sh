#!/bin/bash
# Interleaved same-box A/B of a whole older tree (exp/<name>: its own bench.py, fovrt mirror and libfovrt.so)
# against the working tree, under the driver's exact bench command:
#   scripts/r05_ab_rev.sh <pairs> <name>...
# Logs: gpurun_out/abrev_<tree>_<i>.log (one JSON line each); summary: python scripts/r05_ab_rev_summary.py
set -o pipefail
P=${1:?pairs}
shift
mkdir -p gpurun_out
ROOT=$(pwd)
for i in $(seq 1 "$P"); do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/abrev_head_$i.log 2>&1 || exit 1
  for n in "$@"; do
    (cd "exp/$n" && timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline) \
      > "gpurun_out/abrev_${n}_$i.log" 2>&1 || exit 2
  done
  echo "pair $i done"
done
