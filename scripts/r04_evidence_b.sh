#!/bin/bash
# Round-4 evidence, part B: every BASELINE config (+ the eye-tracked circle and saccade lines), the stages alone,
# the gaze probe and the rebuild probe (the group model: scripts/r04_evidence_c.sh).
set -o pipefail
TAG=${1:-r04a}
mkdir -p gpurun_out
bash scripts/configs_bench.sh || exit 1
python scripts/configs_summary.py "gpurun_out/${TAG}_configs.jsonl" > /dev/null || exit 2
timeout -k 10 200 python scripts/stage_probe.py 10 > "gpurun_out/${TAG}_stage_probe.txt" 2>&1 || exit 3
timeout -k 10 200 python scripts/gaze_probe.py > "gpurun_out/${TAG}_gaze_probe.txt" 2>&1 || exit 4
timeout -k 10 120 python scripts/rebuild_probe.py > "gpurun_out/${TAG}_rebuild_probe.txt" 2>&1 || exit 5
echo "all done"
