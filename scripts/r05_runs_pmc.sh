#!/bin/bash
# k_sibson_runs / k_sibson_strip at the centred and the 90-degree gaze: TA busy, L1 accesses and wave time.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for g in c 90; do
  timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VALU -f csv -d $GRAFT_REPO_ROOT/gpurun_out/rpmc_$g -o s -- python3 $GRAFT_REPO_ROOT/scripts/gaze_probe.py $g > $GRAFT_REPO_ROOT/gpurun_out/rpmc_$g.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $GRAFT_REPO_ROOT/gpurun_out/rkt_$g -o k -- python3 $GRAFT_REPO_ROOT/scripts/gaze_probe.py $g > $GRAFT_REPO_ROOT/gpurun_out/rkt_$g.log 2>&1 || exit 2
done
echo ok
