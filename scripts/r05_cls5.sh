#!/bin/bash
# Sibson strip lists: 4 cost classes (default) against 5 (exp/lib_c5.so, a class at 64 half-rows) and 5 with strips
# over 2 x 24 rows (exp/lib_h24c5.so): the Sibson GPU tests, then Sibson alone per gaze, twice, interleaved.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sibson or golden" \
  > gpurun_out/cl5_tests.log 2>&1 || { tail -30 gpurun_out/cl5_tests.log; exit 1; }
tail -1 gpurun_out/cl5_tests.log
for i in 1 2; do
  timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/cl5_def_$i.txt 2>&1 || exit 2
  FOVRT_LIB=$PWD/exp/lib_c5.so timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/cl5_c5_$i.txt 2>&1 || exit 3
  FOVRT_LIB=$PWD/exp/lib_h24c5.so timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/cl5_h24_$i.txt 2>&1 || exit 4
done
grep -H gaze gpurun_out/cl5_*.txt | cut -c1-100
