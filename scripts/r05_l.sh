#!/bin/bash
# Round 5: stream priority schemes (FOVRT_STREAM_PRIORITY 0 / 4) on C3 and the eye-tracked circle, both modes.
set -o pipefail
mkdir -p gpurun_out
summ() {
python - "$1" <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
lm = j['pipeline_latency_mode']; pl = j.get('frame_clock_pipelined', {}).get('latency_ms', {})
print("%-28s thr fps %6.1f lat p50/p99 %5.1f/%5.1f | serial fps %6.1f | latency-mode fps %6.1f lat p50/p99 %5.2f/%5.2f" % (
  sys.argv[1].split('/')[-1], j['fps'], pl.get('p50', 0), pl.get('p99', 0), j['fps_serial'], lm['fps'],
  lm['frame_clock']['latency_ms']['p50'], lm['frame_clock']['latency_ms']['p99']))
PY
}
for i in 1 2; do
for p in 0 4; do
  FOVRT_STREAM_PRIORITY=$p timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05l_c3_p${p}_$i.log 2>&1 || exit 1
  summ gpurun_out/r05l_c3_p${p}_$i.log
done
done
for p in 0 4; do
  FOVRT_STREAM_PRIORITY=$p timeout -k 10 300 python bench.py --no-cpu-baseline --gaze-path circle --steps 360 --warmup 5 > gpurun_out/r05l_circle_p$p.log 2>&1 || exit 2
  summ gpurun_out/r05l_circle_p$p.log
done
