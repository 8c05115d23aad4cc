#!/bin/bash
# Round 5: the memoised inverse log-polar map (parity tests that recompute the mask) and the latency mode's
# just-in-time schedule (C3, eye-tracked circle).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "sampling or logpolar or gaze or latency or pipelined or sibson" > gpurun_out/gpu_n.log 2>&1 || { tail -30 gpurun_out/gpu_n.log; exit 1; }
tail -2 gpurun_out/gpu_n.log
bash scripts/r05_j.sh
