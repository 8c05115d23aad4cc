#!/bin/bash
# Strip-kernel threshold 2 x 32 rows (default build): the Sibson GPU tests, then Sibson alone per gaze against
# 2 x 24 (exp/lib_sh24.so) and 2 x 16 (exp/lib_sh16.so), twice, interleaved.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sibson or golden" \
  > gpurun_out/sh2_tests.log 2>&1 || { tail -30 gpurun_out/sh2_tests.log; exit 1; }
tail -1 gpurun_out/sh2_tests.log
for i in 1 2; do
  timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/sh2_32_$i.txt 2>&1 || exit 2
  FOVRT_LIB=$PWD/exp/lib_sh24.so timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/sh2_24_$i.txt 2>&1 || exit 3
  FOVRT_LIB=$PWD/exp/lib_sh16.so timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/sh2_16_$i.txt 2>&1 || exit 4
done
grep -H gaze gpurun_out/sh2_*.txt | cut -c1-100
