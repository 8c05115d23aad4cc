#!/bin/bash
# Latency mode: how much of the front stages to overlap with the previous frame's Sibson (FOVRT_LAT_OVERLAP, percent
# of their span): the eye-tracked circle and the C3 bench line (its latency-mode block) for 100 / 50 / 0.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for o in 100 50 0; do
    FOVRT_LAT_OVERLAP=$o timeout -k 10 150 python scripts/latency_circle_probe.py latency 360 | sed "s/^/ovl $o /" >> gpurun_out/latovl.txt 2>&1 || exit 2
  done
done
cat gpurun_out/latovl.txt
for o in 100 50 0; do
  FOVRT_LAT_OVERLAP=$o timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/latovl_bench_$o.log 2>&1 || exit 3
  python - gpurun_out/latovl_bench_$o.log $o <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
lm = j['pipeline_latency_mode']
print('ovl', sys.argv[2], j['value'], j['fps'], 'serial', j['fps_serial'], 'latency mode', lm['fps'], lm['frame_clock']['latency_ms'])
PY
done
