#!/bin/bash
# Sibson parity first (the new strip kernel), then the whole GPU suite, a bench line, the rebuild probe and the
# gaze probe with its kernel trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "sibson or Sibson" > gpurun_out/sib_tests.log 2>&1 || { tail -30 gpurun_out/sib_tests.log; exit 1; }
tail -2 gpurun_out/sib_tests.log
bash scripts/r04_check.sh && bash scripts/r04_gaze_kernels.sh
