#!/bin/bash
# Latency mode, eye-tracked circle: the front stages' span estimated as the smallest of the last eight (default
# build) against the last frame's (exp/lib_lat0.so), twice, interleaved; then one bench line per build (C3, the
# latency-mode block); the latency GPU tests first.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "latency or frame_driver" \
  > gpurun_out/latfront_tests.log 2>&1 || { tail -30 gpurun_out/latfront_tests.log; exit 1; }
tail -1 gpurun_out/latfront_tests.log
for i in 1 2; do
  timeout -k 10 150 python scripts/latency_circle_probe.py latency 360 >> gpurun_out/latfront.txt 2>&1 || exit 2
  FOVRT_LIB=$PWD/exp/lib_lat0.so timeout -k 10 150 python scripts/latency_circle_probe.py latency 360 | sed 's/^/OLD /' >> gpurun_out/latfront.txt 2>&1 || exit 3
done
cat gpurun_out/latfront.txt
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/latfront_bench_new.log 2>&1 || exit 4
FOVRT_LIB=$PWD/exp/lib_lat0.so timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/latfront_bench_old.log 2>&1 || exit 5
for f in new old; do python - gpurun_out/latfront_bench_$f.log $f <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
lm = j['pipeline_latency_mode']
print(sys.argv[2], j['value'], j['fps'], 'latency mode', lm['fps'], lm['frame_clock']['latency_ms'])
PY
done
