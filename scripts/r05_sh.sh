#!/bin/bash
# Strip-kernel threshold: discs over 2 x 64 rows (default) against 2 x 32 (exp/lib_sh32.so) and 2 x 48
# (exp/lib_sh48.so): Sibson alone per gaze, twice, interleaved.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/sh_def_$i.txt 2>&1 || exit 1
  FOVRT_LIB=$PWD/exp/lib_sh32.so timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/sh_32_$i.txt 2>&1 || exit 2
  FOVRT_LIB=$PWD/exp/lib_sh48.so timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/sh_48_$i.txt 2>&1 || exit 3
done
grep -H gaze gpurun_out/sh_*.txt | cut -c1-100
