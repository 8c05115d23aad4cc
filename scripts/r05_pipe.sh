#!/bin/bash
# Sibson strip kernel: the row's last run summed one row later (default build, 3 waves/SIMD) against the
# unpipelined form (exp/lib_p0.so) and the pipelined form at 4 waves/SIMD with spills (exp/lib_p4.so):
# the Sibson GPU tests, then Sibson alone per gaze for the three builds, twice, interleaved.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sibson or golden" \
  > gpurun_out/pipe_tests.log 2>&1 || { tail -30 gpurun_out/pipe_tests.log; exit 1; }
tail -1 gpurun_out/pipe_tests.log
for i in 1 2; do
  timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/pipe_on_$i.txt 2>&1 || exit 2
  FOVRT_LIB=$PWD/exp/lib_p0.so timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/pipe_p0_$i.txt 2>&1 || exit 3
  FOVRT_LIB=$PWD/exp/lib_p4.so timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/pipe_p4_$i.txt 2>&1 || exit 4
done
grep -H gaze gpurun_out/pipe_*.txt | cut -c1-100
