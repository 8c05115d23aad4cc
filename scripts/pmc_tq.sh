#!/bin/bash
# Counter passes over the traversal probe (scripts/trace_probe.py, diagnostic library):
#   scripts/pmc_tq.sh <lib.so> <tag>   -> gpurun_out/pmc_tq_<tag>_{A,B,C}/
set -eo pipefail
LIB=${1:?lib}
TAG=${2:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export FOVRT_LIB=$ROOT/$LIB
cd /tmp
export TMPDIR=/tmp
pass() {
  local name=$1; shift
  mkdir -p "$ROOT/gpurun_out/pmc_tq_${TAG}_$name"
  timeout -k 10 240 rocprofv3 --pmc "$@" -f csv -d "$ROOT/gpurun_out/pmc_tq_${TAG}_$name" -o run -- \
    python3 "$ROOT/scripts/trace_probe.py" > "$ROOT/gpurun_out/pmc_tq_${TAG}_$name/probe.json" \
    2> "$ROOT/gpurun_out/pmc_tq_${TAG}_$name/err.log"
}
pass A SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS
pass B TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCP_LATENCY_sum
pass C TCC_HIT_sum TCC_MISS_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum
pass D SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE
