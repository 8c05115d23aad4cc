#!/bin/bash
# The Sibson GPU tests, then per-kernel Sibson times at the probe gazes reached in sequence (c 45 90 180).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sibson or golden" \
  > gpurun_out/sk2_tests.log 2>&1 || { tail -30 gpurun_out/sk2_tests.log; exit 1; }
tail -1 gpurun_out/sk2_tests.log
cd /tmp && export TMPDIR=/tmp
for g in 90 180; do
  timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d $GRAFT_REPO_ROOT/gpurun_out/sk2_$g -o k -- python3 $GRAFT_REPO_ROOT/scripts/gaze_probe.py c 45 $g > $GRAFT_REPO_ROOT/gpurun_out/sk2_$g.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/sk2_$g.log; exit 2; }
done
echo prof ok
