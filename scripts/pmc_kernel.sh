#!/bin/bash
# Counter passes over one probe script: scripts/pmc_kernel.sh <name> <script.py> [args...]
# Each pass in its own rocprofv3 run (<= 8 SQ counters per pass); CSVs in gpurun_out/pmck_<name>_<pass>.
set -eo pipefail
NAME=${1:?name}; SCRIPT=${2:?script}; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES"
P2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
i=1
for P in "$P1" "$P2" "$P3" "$P4"; do
  OUT=$ROOT/gpurun_out/pmck_${NAME}_$i
  mkdir -p "$OUT"
  timeout -s KILL 120 rocprofv3 --pmc $P -f csv -d "$OUT" -o run -- python3 "$ROOT/$SCRIPT" "$@" > "$OUT/out.txt" 2> "$OUT/err.log"
  i=$((i+1))
done
