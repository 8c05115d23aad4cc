#!/bin/bash
# Kernel trace of 16 latency-mode frames of the eye-tracked circle from 140 degrees (its slowest frames).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $GRAFT_REPO_ROOT/gpurun_out/lattrace -o k -- python3 $GRAFT_REPO_ROOT/scripts/latency_probe.py latency 16 140 > $GRAFT_REPO_ROOT/gpurun_out/lattrace.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/lattrace.log; exit 1; }
echo ok
