#!/bin/bash
# Sibson strip kernel: strips listed by cost class, costliest claimed first (default build) against one class
# (exp/lib_cls1.so): the Sibson GPU tests, Sibson alone per gaze for both builds twice, the strip statistics.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sibson or golden" \
  > gpurun_out/ord_tests.log 2>&1 || { tail -30 gpurun_out/ord_tests.log; exit 1; }
tail -2 gpurun_out/ord_tests.log
for i in 1 2; do
  timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/ord_on_$i.txt 2>&1 || exit 2
  FOVRT_LIB=$PWD/exp/lib_cls1.so timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/ord_off_$i.txt 2>&1 || exit 3
done
grep -H gaze gpurun_out/ord_*.txt
timeout -k 10 200 python scripts/strip_stats.py 45 90 180 > gpurun_out/ord_strip_stats.txt 2>&1 && cat gpurun_out/ord_strip_stats.txt
