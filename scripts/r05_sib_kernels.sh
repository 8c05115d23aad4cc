#!/bin/bash
# Per-kernel Sibson times at one eye-tracked gaze per run (kernel traces of scripts/gaze_probe.py 90 / 180).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for g in 90 180; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_sib$g -o sib -- python3 $GRAFT_REPO_ROOT/scripts/gaze_probe.py $g > $GRAFT_REPO_ROOT/gpurun_out/sib_prof_$g.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/sib_prof_$g.log; exit 2; }
done
echo prof ok
