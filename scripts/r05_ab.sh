#!/bin/bash
# GPU suite on the working tree, then interleaved A/B against exp/<names> (r05_ab_rev.sh) and its summary.
set -o pipefail
P=${1:?pairs}; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash scripts/r05_ab_rev.sh "$P" "$@" || exit 2
python scripts/r05_ab_rev_summary.py gpurun_out
