#!/bin/bash
# Timing ablations of k_sibson_strip's row step (diagnostic builds, wrong results): SIBS_ABL 1 = no run-end
# settling, 2 = no row loads, 4 = no segment loop, 3 = 1 + 2. Sibson alone per gaze (gaze_probe.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python scripts/gaze_probe.py 90 180 > gpurun_out/abl_base.txt 2>&1 || exit 1
for v in 1 2 4 3; do
  FOVRT_LIB=$PWD/exp/lib_abl$v.so timeout -k 10 150 python scripts/gaze_probe.py 90 180 > gpurun_out/abl_$v.txt 2>&1 || exit 2
done
grep -H gaze gpurun_out/abl_*.txt
