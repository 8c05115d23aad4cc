#!/bin/bash
# JFA and Sibson parity (the new kernels), the Sibson strip A/B at the probe gazes, then the stage probe.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "sibson or Sibson or jfa or JFA or frame_driver or fullsize" > gpurun_out/sib_tests.log 2>&1 || { tail -30 gpurun_out/sib_tests.log; exit 1; }
tail -2 gpurun_out/sib_tests.log
bash scripts/r04_sib_ab.sh || exit 2
timeout -k 10 200 python scripts/stage_probe.py 10 > gpurun_out/r04_stage_probe.txt 2>&1 || exit 3
cat gpurun_out/r04_stage_probe.txt
