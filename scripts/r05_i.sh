#!/bin/bash
# Round 5: megakernel wave priority A/B (FOVRT_SHADE_PRIO) and the eye-tracked circle in both pipeline modes.
set -o pipefail
mkdir -p gpurun_out
bash scripts/ab_env.sh 4 "p0:FOVRT_SHADE_PRIO=0" "p2:FOVRT_SHADE_PRIO=2" "p3:FOVRT_SHADE_PRIO=3" || exit 1
python scripts/ab_repeat_summary.py 2>&1 | tail -8
timeout -k 10 300 python bench.py --no-cpu-baseline --gaze-path circle --steps 360 --warmup 5 > gpurun_out/r05i_circle.log 2>&1 || exit 2
python - <<'PY'
import json
j = json.loads([l for l in open('gpurun_out/r05i_circle.log') if l.startswith('{')][-1])
print('circle', j['value'], j['fps'], j['fps_serial'], 'pipelined clock', j.get('frame_clock_pipelined', {}).get('latency_ms'))
print('latency mode', j.get('pipeline_latency_mode'))
PY
