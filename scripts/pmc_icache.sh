#!/bin/bash
# Instruction-cache counters of the stage probe's kernels (one pass, the SQC icache counters the box lists):
#   scripts/pmc_icache.sh  -> gpurun_out/rocprof_counters.txt, gpurun_out/pmck_icache/
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp
export TMPDIR=/tmp
[ -s "$ROOT/gpurun_out/rocprof_counters.txt" ] || timeout -s KILL 60 rocprofv3 -L > "$ROOT/gpurun_out/rocprof_counters.txt" 2>&1 || true
C="SQC_ICACHE_MISSES SQC_ICACHE_REQ SQ_IFETCH SQ_WAIT_INST_ANY"
echo "icache counters: $C"
[ -n "$C" ] || exit 0
OUT=$ROOT/gpurun_out/pmck_icache
mkdir -p "$OUT"
timeout -s KILL 90 rocprofv3 --pmc $C SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -f csv -d "$OUT" -o run -- python3 "$ROOT/scripts/stage_probe.py" 3 > "$OUT/out.txt" 2> "$OUT/err.log"
echo "rc=$?"
