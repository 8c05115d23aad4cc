#!/bin/bash
# k_sibson_strip counters at the 90-degree gaze: the default build and the no-row-load ablation (exp/lib_abl2.so),
# SQ instruction / wave-time counters; then L2 hit / miss and L1->L2 requests of the default build.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
SQ="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS"
timeout -s KILL 120 rocprofv3 --pmc $SQ -f csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc2_base -o s -- python3 $GRAFT_REPO_ROOT/scripts/gaze_probe.py 90 > $GRAFT_REPO_ROOT/gpurun_out/pmc2_base.log 2>&1 || exit 1
FOVRT_LIB=$GRAFT_REPO_ROOT/exp/lib_abl2.so timeout -s KILL 120 rocprofv3 --pmc $SQ -f csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc2_abl2 -o s -- python3 $GRAFT_REPO_ROOT/scripts/gaze_probe.py 90 > $GRAFT_REPO_ROOT/gpurun_out/pmc2_abl2.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -f csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc2_l2 -o s -- python3 $GRAFT_REPO_ROOT/scripts/gaze_probe.py 90 > $GRAFT_REPO_ROOT/gpurun_out/pmc2_l2.log 2>&1 || exit 3
echo pmc ok
