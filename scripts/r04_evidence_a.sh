#!/bin/bash
# Round-4 evidence, part A: the GPU suite, the bench line, its kernel trace and HBM counter passes.
set -o pipefail
TAG=${1:-r04a}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > "gpurun_out/${TAG}_bench.log" 2>&1 || { tail -5 "gpurun_out/${TAG}_bench.log"; exit 2; }
echo "bench done"
bash scripts/profile.sh "$TAG" || exit 3
echo "profile done"
