#!/bin/bash
# Round-4 check: GPU suite, one bench line, rebuild probe (plain and under a runtime trace).
set -o pipefail
mkdir -p gpurun_out
K=${1:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r04_bench.log 2>&1 || { tail -5 gpurun_out/r04_bench.log; exit 2; }
echo bench ok
timeout -k 10 120 python scripts/rebuild_probe.py > gpurun_out/rebuild_probe.log 2>&1 || { tail -5 gpurun_out/rebuild_probe.log; exit 3; }
cat gpurun_out/rebuild_probe.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --runtime-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_rebuild -o rb -- python3 $GRAFT_REPO_ROOT/scripts/rebuild_probe.py > $GRAFT_REPO_ROOT/gpurun_out/rebuild_prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/rebuild_prof.log; exit 4; }
echo prof ok
