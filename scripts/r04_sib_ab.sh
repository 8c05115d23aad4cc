#!/bin/bash
# Sibson A/B at the probe gazes: the strip kernel on / off, then a kernel trace with it on.
set -o pipefail
mkdir -p gpurun_out
for v in 0 1; do
  FOVRT_SIB_STRIP=$v timeout -k 10 240 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/gaze_probe_strip$v.txt 2>&1 || { tail -5 gpurun_out/gaze_probe_strip$v.txt; exit 1; }
  echo "strip=$v"; cat gpurun_out/gaze_probe_strip$v.txt
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_gaze -o gz -- python3 $GRAFT_REPO_ROOT/scripts/gaze_probe.py 90 180 > $GRAFT_REPO_ROOT/gpurun_out/gaze_prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/gaze_prof.log; exit 2; }
echo prof ok
