#!/bin/bash
# Sibson A/B (k_sibson_strip with whole-row prefixes vs k_sibson_wide), the strip kernel's counters, and the
# stages' kernels alone with the JFA steps in XCD order and in round-robin order.
set -o pipefail
mkdir -p gpurun_out
bash scripts/r04_ab4.sh > gpurun_out/ab4.log 2>&1 || { tail -30 gpurun_out/ab4.log; exit 1; }
tail -12 gpurun_out/ab4.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "jfa or JFA or jump or Jump" > gpurun_out/jfa_tests.log 2>&1 || { tail -30 gpurun_out/jfa_tests.log; exit 5; }
tail -1 gpurun_out/jfa_tests.log
bash scripts/pmc_sibstrip.sh 1 || exit 2
FOVRT_JFA_XCD=0 bash scripts/stage_kernels.sh stagek_xcd0 > gpurun_out/stagek_xcd0.txt || exit 3
FOVRT_JFA_XCD=1 bash scripts/stage_kernels.sh stagek_xcd1 > gpurun_out/stagek_xcd1.txt || exit 4
for t in xcd0 xcd1; do echo "== $t"; grep -h "jfa\|sibson\|geometry=" gpurun_out/stagek_$t.txt gpurun_out/stagek_$t/out.txt; done
