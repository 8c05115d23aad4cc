#!/bin/bash
# Round-6 evidence on one GPU box: the GPU suite; the bench workload's kernel trace and HBM traffic
# (scripts/profile.sh -> profiles/<tag>_kernel_stats.csv, _pmc_traffic.json) and SIMD issue counters
# (scripts/pmc_sq.sh + pmc_issue.py -> profiles/<tag>_pmc_issue.json); then the driver's bench command (it reads the
# traffic and issue profiles just written); every BASELINE config in both pipeline modes (+ the eye-tracked circle
# and saccades); the stages alone and their kernels; the gaze and rebuild probes; the group model for vokselia.
# Files written to profiles/ on the box are copied to gpurun_out/<tag>_profiles/ (only gpurun_out comes back).
#   scripts/r06_evidence.sh <tag>
set -o pipefail
TAG=${1:?tag}
ROOT=$(pwd)
mkdir -p gpurun_out/${TAG}_profiles
keep() { cp -f profiles/${TAG}_* gpurun_out/${TAG}_profiles/ 2>/dev/null; true; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
bash scripts/profile.sh "$TAG" --steps 20 --warmup 5 > gpurun_out/${TAG}_profile.txt 2>&1 || { tail gpurun_out/${TAG}_profile.txt; exit 2; }
head -12 gpurun_out/${TAG}_profile.txt; keep
bash scripts/pmc_sq.sh || exit 3
python3 scripts/pmc_issue.py gpurun_out "$TAG" > gpurun_out/${TAG}_issue.txt 2>&1 || exit 3
echo "$TAG" > profiles/CURRENT  # the bench below quotes this run's traffic and issue profiles
keep
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 4
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));r=d['roofline'];print('bench', d['value'], d['fps'], d['fps_serial_mean'], d['pipeline_latency_mode']['fps'], r['megakernel_ms'], r['megakernel_ms_serialised'], r.get('traffic'), d['cpu_baseline'].get('value'))"
echo "configs" && bash scripts/configs_bench.sh > gpurun_out/${TAG}_configs_run.txt 2>&1 || { tail gpurun_out/${TAG}_configs_run.txt; exit 5; }
python3 scripts/configs_summary.py "gpurun_out/${TAG}_configs.jsonl" > /dev/null || exit 5
timeout -k 10 200 python scripts/stage_probe.py 10 > gpurun_out/${TAG}_stage_probe.txt 2>&1 || exit 6
cat gpurun_out/${TAG}_stage_probe.txt
bash scripts/stage_kernels.sh ${TAG}_stagek > gpurun_out/${TAG}_stage_kernels.txt 2>&1 || exit 7
timeout -k 10 200 python scripts/gaze_probe.py > gpurun_out/${TAG}_gaze_probe.txt 2>&1 || exit 8
cat gpurun_out/${TAG}_gaze_probe.txt
timeout -k 10 120 python scripts/rebuild_probe.py > gpurun_out/${TAG}_rebuild_probe.txt 2>&1 || exit 9
timeout -k 10 500 python scripts/shard_model.py vokselia > gpurun_out/${TAG}_shard_model_vokselia.jsonl 2>&1 || exit 10
echo "all done"
