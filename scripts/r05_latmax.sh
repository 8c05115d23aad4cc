#!/bin/bash
# Latency mode on the eye-tracked circle: the just-in-time Sibson estimate from the last frame (default) against
# the largest of the last 2 / 4 frames (FOVRT_LAT_SIB_MAX), twice, interleaved; the latency GPU tests first.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "latency or frame_driver" \
  > gpurun_out/latmax_tests.log 2>&1 || { tail -30 gpurun_out/latmax_tests.log; exit 1; }
tail -1 gpurun_out/latmax_tests.log
for i in 1 2; do
  for m in 1 2 4; do
    FOVRT_LAT_SIB_MAX=$m timeout -k 10 150 python scripts/latency_circle_probe.py latency 360 >> gpurun_out/latmax.txt 2>&1 || exit 2
  done
done
timeout -k 10 150 python scripts/latency_circle_probe.py throughput 360 >> gpurun_out/latmax.txt 2>&1 || exit 3
cat gpurun_out/latmax.txt
