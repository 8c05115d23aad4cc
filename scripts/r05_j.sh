#!/bin/bash
# Round 5: latency mode with a polled host wait: C3 (static gaze) and the eye-tracked circle.
set -o pipefail
mkdir -p gpurun_out
summ() {
python - "$1" <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[1], j['value'], j['fps'], j['fps_serial'], 'pipelined latency', j.get('frame_clock_pipelined', {}).get('latency_ms'))
lm = j.get('pipeline_latency_mode'); print('  latency mode fps', lm['fps'], 'latency', lm['frame_clock']['latency_ms'], 'interval p50', lm['frame_clock']['interval_ms']['p50'])
PY
}
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05j_c3.log 2>&1 || exit 1
summ gpurun_out/r05j_c3.log
timeout -k 10 300 python bench.py --no-cpu-baseline --gaze-path circle --steps 360 --warmup 5 > gpurun_out/r05j_circle.log 2>&1 || exit 2
summ gpurun_out/r05j_circle.log
