#!/bin/bash
# Sibson on the wide-hole mask (scripts/sib_mask_probe.py, FOVRT_SIB_STRIP=$1): kernel trace, then SQ and TA
# counter passes (only the counters this box lists) -> gpurun_out/pmc_sib$1/
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
S=${1:-1}
cd /tmp
export TMPDIR=/tmp
export FOVRT_SIB_STRIP=$S
OUT=$ROOT/gpurun_out/pmc_sib$S
mkdir -p "$OUT"
[ -s "$ROOT/gpurun_out/rocprof_counters.txt" ] || timeout -s KILL 60 rocprofv3 -L > "$ROOT/gpurun_out/rocprof_counters.txt" 2>&1 || true
have() { for c in "$@"; do grep -qw "$c" "$ROOT/gpurun_out/rocprof_counters.txt" && printf '%s ' "$c"; done; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o trace -- python3 "$ROOT/scripts/sib_mask_probe.py" 2 > "$OUT/trace_out.txt" 2>&1 || exit 1
A=$(have SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY)
B=$(have SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM_RD TA_BUSY_avr TA_TA_BUSY_avr TD_BUSY_avr TD_TD_BUSY_avr)
echo "pass A: $A"; echo "pass B: $B"
timeout -s KILL 90 rocprofv3 --pmc $A -f csv -d "$OUT" -o pmcA -- python3 "$ROOT/scripts/sib_mask_probe.py" 1 > "$OUT/a_out.txt" 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $B -f csv -d "$OUT" -o pmcB -- python3 "$ROOT/scripts/sib_mask_probe.py" 1 > "$OUT/b_out.txt" 2>&1 || exit 1
echo done
