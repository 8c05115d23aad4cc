#!/bin/bash
# Round-5 evidence: the bench workload's kernel stats and HBM traffic (scripts/profile.sh), every BASELINE
# config (+ the eye-tracked circle and saccade lines, both pipeline modes in each line), the stages alone,
# the gaze probe and the rebuild probe.
set -o pipefail
TAG=${1:-r05a}
mkdir -p gpurun_out
bash scripts/profile.sh "$TAG" --steps 20 --warmup 5 || { echo "profile failed"; exit 1; }
bash scripts/configs_bench.sh || exit 2
python scripts/configs_summary.py "gpurun_out/${TAG}_configs.jsonl" > /dev/null || exit 3
timeout -k 10 200 python scripts/stage_probe.py 10 > "gpurun_out/${TAG}_stage_probe.txt" 2>&1 || exit 4
timeout -k 10 200 python scripts/gaze_probe.py > "gpurun_out/${TAG}_gaze_probe.txt" 2>&1 || exit 5
timeout -k 10 120 python scripts/rebuild_probe.py > "gpurun_out/${TAG}_rebuild_probe.txt" 2>&1 || exit 6
echo "all done"
