#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes plus a kernel trace of scripts/stage_probe.py (K=3), for the library
# in FOVRT_LIB (default: the tree's): scripts/pmc_fw.sh <name>; CSVs in gpurun_out/pmcfw_<name>_{f,w,t}
set -eo pipefail
NAME=${1:?name}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp
export TMPDIR=/tmp
for P in f:FETCH_SIZE w:WRITE_SIZE; do
  OUT=$ROOT/gpurun_out/pmcfw_${NAME}_${P%%:*}
  mkdir -p "$OUT"
  timeout -s KILL 120 rocprofv3 --pmc ${P#*:} -f csv -d "$OUT" -o run -- python3 "$ROOT/scripts/stage_probe.py" 3 > "$OUT/out.txt" 2> "$OUT/err.log"
done
OUT=$ROOT/gpurun_out/pmcfw_${NAME}_t
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o run -- python3 "$ROOT/scripts/stage_probe.py" 10 > "$OUT/out.txt" 2> "$OUT/err.log"
