#!/bin/bash
# Sibson strip kernel: whole-row prefixes in xy / z planes (paired loads, default build) against 16-byte texels
# (exp/lib_g16.so): the Sibson GPU tests, Sibson alone per gaze for both builds twice.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sibson or golden" \
  > gpurun_out/gpl_tests.log 2>&1 || { tail -30 gpurun_out/gpl_tests.log; exit 1; }
tail -2 gpurun_out/gpl_tests.log
for i in 1 2; do
  timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/gpl_on_$i.txt 2>&1 || exit 2
  FOVRT_LIB=$PWD/exp/lib_g16.so timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/gpl_off_$i.txt 2>&1 || exit 3
done
grep -H gaze gpurun_out/gpl_*.txt
