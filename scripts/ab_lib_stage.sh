#!/bin/bash
# Interleaved A/B of library builds on the stages alone: for each rep, each "name:lib" (lib "-" = the in-tree
# build) runs scripts/stage_probe.py 15; then one FETCH_SIZE and one WRITE_SIZE pass per build, summed for the
# kernels named in $AB_KERNELS (default: Sibson and JFA kernels).
#   scripts/ab_lib_stage.sh <tag> <reps> name:lib ...   -> gpurun_out/<tag>_summary.txt
set -o pipefail
TAG=${1:?tag}; R=${2:?reps}; shift 2
ROOT=$(pwd)
KS=${AB_KERNELS:-k_sibson_runs k_sibson_wide k_jfa_step k_jfa_final}
mkdir -p gpurun_out
S=gpurun_out/${TAG}_summary.txt
: > "$S"
for i in $(seq 1 "$R"); do
  for spec in "$@"; do
    n=${spec%%:*}; lib=${spec#*:}
    if [ "$lib" = "-" ]; then unset FOVRT_LIB; else export FOVRT_LIB=$ROOT/$lib; fi
    timeout -k 10 200 python scripts/stage_probe.py 15 > gpurun_out/${TAG}_${n}_$i.log 2>&1 || { cat gpurun_out/${TAG}_${n}_$i.log; exit 2; }
    echo "$n $i $(cat gpurun_out/${TAG}_${n}_$i.log)" | tee -a "$S"
  done
done
cd /tmp && export TMPDIR=/tmp
for spec in "$@"; do
  n=${spec%%:*}; lib=${spec#*:}
  if [ "$lib" = "-" ]; then unset FOVRT_LIB; else export FOVRT_LIB=$ROOT/$lib; fi
  for C in FETCH_SIZE WRITE_SIZE; do
    OUT=$ROOT/gpurun_out/${TAG}_${n}_$C
    mkdir -p "$OUT"
    timeout -s KILL 120 rocprofv3 --pmc $C -f csv -d "$OUT" -o run -- python3 "$ROOT/scripts/stage_probe.py" 2 > "$OUT/out.txt" 2> "$OUT/err.log" || exit 4
    f=$(find "$OUT" -name "*counter_collection.csv" | head -1)
    echo "$n $(python3 "$ROOT/scripts/pmc_kernel_sum.py" "$f" $KS | tr '\n' ' ')" | tee -a "$ROOT/$S"
  done
done
