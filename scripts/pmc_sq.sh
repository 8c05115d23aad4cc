#!/bin/bash
# Wave-cycle breakdown of the kernels of the bench workload (two short counter passes):
#   scripts/pmc_sq.sh [bench args...]  -> gpurun_out/pmc_sq1, gpurun_out/pmc_sq2
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$ROOT/gpurun_out/rocprof_counters.txt" 2>&1 || true
bash "$ROOT/scripts/pmc_probe.sh" sq1 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU" "$@"
bash "$ROOT/scripts/pmc_probe.sh" sq2 "SQ_INSTS_LDS SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "$@"
