#!/bin/bash
# Round 5: Sibson changes (row-range whole-row prefixes, multi-segment closed form in k_sibson_runs, strip
# waves per strip): parity on the working tree, then the gaze probe (Sibson alone) per library.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "sibson" > gpurun_out/gpu_p.log 2>&1 || { tail -30 gpurun_out/gpu_p.log; exit 1; }
tail -2 gpurun_out/gpu_p.log
for v in head tree sw8 sw16; do
  if [ $v = tree ]; then L=""; else L="FOVRT_LIB=exp/lib_$v.so"; fi
  env $L timeout -k 10 200 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/r05p_gaze_$v.txt 2>&1 || { tail -5 gpurun_out/r05p_gaze_$v.txt; exit 2; }
  echo "== $v"; sed 's/; rows.*//' gpurun_out/r05p_gaze_$v.txt
done
