#!/bin/bash
# k_sibson_strip at the 90-degree gaze (reached from the centred one, as gaze_probe.py 90 does): the strips'
# trip counts (strip_stats.py) and one SQ counter pass over the same probe.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python scripts/strip_stats.py 90 > gpurun_out/strip_stats_90.txt 2>&1 || { tail -5 gpurun_out/strip_stats_90.txt; exit 1; }
cat gpurun_out/strip_stats_90.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS -f csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_strip90 -o s -- python3 $GRAFT_REPO_ROOT/scripts/gaze_probe.py 90 > $GRAFT_REPO_ROOT/gpurun_out/pmc_strip90.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmc_strip90.log; exit 2; }
echo pmc ok
