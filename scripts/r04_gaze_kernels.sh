#!/bin/bash
# Per-kernel Sibson times at the eye-tracked probe gazes (kernel trace of scripts/gaze_probe.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/gaze_probe.txt 2>&1 || { tail -5 gpurun_out/gaze_probe.txt; exit 1; }
cat gpurun_out/gaze_probe.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_gaze -o gz -- python3 $GRAFT_REPO_ROOT/scripts/gaze_probe.py 90 180 > $GRAFT_REPO_ROOT/gpurun_out/gaze_prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/gaze_prof.log; exit 2; }
echo prof ok
