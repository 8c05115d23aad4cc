#!/bin/bash
# Kernel trace of 60 latency-mode frames of the eye-tracked circle from 100 degrees (the last ones: its slowest, warm).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $GRAFT_REPO_ROOT/gpurun_out/lattrace -o k -- python3 $GRAFT_REPO_ROOT/scripts/latency_probe.py latency 60 100 > $GRAFT_REPO_ROOT/gpurun_out/lattrace.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/lattrace.log; exit 1; }
echo ok
