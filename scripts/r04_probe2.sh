#!/bin/bash
# JFA tail fusion: the JFA GPU tests, then the stages' kernels alone with and without it.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "jfa or JFA or jump or Jump or sibson or Sibson" > gpurun_out/jfa_tests.log 2>&1 || { tail -30 gpurun_out/jfa_tests.log; exit 5; }
tail -1 gpurun_out/jfa_tests.log
FOVRT_JFA_TAIL=0 bash scripts/stage_kernels.sh stagek_tail0 > gpurun_out/stagek_tail0.txt || exit 3
FOVRT_JFA_TAIL=1 bash scripts/stage_kernels.sh stagek_tail1 > gpurun_out/stagek_tail1.txt || exit 4
for t in tail0 tail1; do echo "== $t"; grep -h "jfa\|geometry=" gpurun_out/stagek_$t.txt gpurun_out/stagek_$t/out.txt; done
