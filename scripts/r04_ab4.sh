#!/bin/bash
# Sibson long-border-run split: the Sibson GPU tests, then the wide-hole mask probe and the 90/180-degree gaze
# probe with k_sibson_wide (FOVRT_SIB_STRIP=0) and k_sibson_strip (FOVRT_SIB_STRIP=1).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "sibson or Sibson" > gpurun_out/sib_tests.log 2>&1 || { tail -30 gpurun_out/sib_tests.log; exit 1; }
tail -2 gpurun_out/sib_tests.log
for s in 0 1; do
  echo "strip $s"
  FOVRT_SIB_STRIP=$s timeout -k 10 200 python scripts/sib_mask_probe.py 5 || exit 1
  FOVRT_SIB_STRIP=$s timeout -k 10 300 python scripts/gaze_probe.py c 90 180 || exit 1
done
