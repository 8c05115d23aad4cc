#!/bin/bash
# GPU parity suite (optionally -k filtered) then the stages-alone probe: scripts/gpu_quick.sh [pytest -k expr]
set -o pipefail
mkdir -p gpurun_out
K=${1:-}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 200 python scripts/stage_probe.py 10 > gpurun_out/probe.txt 2>&1 || exit 2
cat gpurun_out/probe.txt
