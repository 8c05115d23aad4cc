#!/bin/bash
# Timing ablations of k_sibson_strip's row step on the class-table build (diagnostic builds, wrong results):
# SIBS_ABL 8 = only the loop skeleton, 1 = no run sum (ends found), 2 = no row loads, 4 = no run-end search.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/abl2_base.txt 2>&1 || exit 1
for v in 8 1 2 4; do
  FOVRT_LIB=$PWD/exp/lib_abl$v.so timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/abl2_$v.txt 2>&1 || exit 2
done
grep -H gaze gpurun_out/abl2_*.txt
