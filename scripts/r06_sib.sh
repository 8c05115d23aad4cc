#!/bin/bash
# Sibson iteration: its GPU tests, the stages-alone kernel durations, and HBM traffic per kernel (FETCH_SIZE and
# WRITE_SIZE passes over the stage probe). Reads: 2 x FETCH_SIZE KiB (gfx950), writes: WRITE_SIZE KiB.
#   scripts/r06_sib.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:?tag}
K=${2:-sibson or jfa or frame_driver or pipelined}
ROOT=$(pwd)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python scripts/stage_probe.py 10 > gpurun_out/${TAG}_stage_probe.txt 2>&1 || exit 2
cat gpurun_out/${TAG}_stage_probe.txt
bash scripts/stage_kernels.sh ${TAG}_sk > gpurun_out/${TAG}_stage_kernels.txt 2>&1 || exit 3
grep -i "sibson\|jfa" gpurun_out/${TAG}_stage_kernels.txt
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  OUT=$ROOT/gpurun_out/${TAG}_pmc_$C
  mkdir -p "$OUT"
  timeout -s KILL 120 rocprofv3 --pmc $C -f csv -d "$OUT" -o run -- python3 "$ROOT/scripts/stage_probe.py" 2 > "$OUT/out.txt" 2> "$OUT/err.log" || exit 4
  f=$(find "$OUT" -name "*counter_collection.csv" | head -1)
  python3 "$ROOT/scripts/pmc_kernel_sum.py" "$f" k_sibson_runs k_sibson_rowp k_sibson_strip k_jfa_step k_jfa_final k_jfa_init
done
