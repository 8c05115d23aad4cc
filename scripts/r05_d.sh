#!/bin/bash
# Round 5: where the second rebuild's 20 ms goes. Phase timing with the entry's HIP calls split, then
# the same probe under rocprofv3 (HIP runtime + kernel trace; the program directly after --).
set -o pipefail
mkdir -p gpurun_out/rbprof
FOVRT_BVH_PHASES=1 timeout -k 10 120 python scripts/rebuild_probe.py 1 2 > gpurun_out/rb_api.log 2>&1 || exit 3
grep -v "^bvh phase" gpurun_out/rb_api.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d gpurun_out/rbprof -o rb -- python3 scripts/rebuild_probe.py 1 2 > gpurun_out/rbprof/run.log 2>&1 || { tail -20 gpurun_out/rbprof/run.log; exit 4; }
grep "rebuild ms\|after a frame" gpurun_out/rbprof/run.log
python3 scripts/rb_api_summary.py gpurun_out/rbprof > gpurun_out/rbprof/summary.txt 2>&1; head -60 gpurun_out/rbprof/summary.txt
