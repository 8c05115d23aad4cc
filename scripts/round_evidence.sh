#!/bin/bash
# Round evidence on one GPU box: the GPU suite, the bench line with its rocprofv3 kernel trace and HBM
# counter passes (scripts/profile.sh), one bench line per BASELINE config (+ the eye-tracked C3), the
# group scaling model (bunny, vokselia) and the stages alone.
#   scripts/round_evidence.sh <tag>
set -o pipefail
TAG=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash scripts/profile.sh "$TAG" || exit 2
echo "profile done"
timeout -k 10 400 python bench.py > "gpurun_out/${TAG}_bench.log" 2>&1 || exit 3
echo "bench done"
bash scripts/configs_bench.sh || exit 4
timeout -k 10 200 python scripts/stage_probe.py 10 > "gpurun_out/${TAG}_stage_probe.txt" 2>&1 || exit 5
timeout -k 10 500 python scripts/shard_model.py bunny > "gpurun_out/${TAG}_shard_model.jsonl" 2>&1 || exit 6
timeout -k 10 500 python scripts/shard_model.py vokselia >> "gpurun_out/${TAG}_shard_model.jsonl" 2>&1 || exit 7
echo "all done"
