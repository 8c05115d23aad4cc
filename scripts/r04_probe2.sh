#!/bin/bash
# JFA tail fusion and Sibson's mid-size wide discs by strips: GPU tests (both), the stages' kernels alone
# (tail off / default / mid on), the gaze probe with mid off / on.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "jfa or JFA or jump or Jump or sibson or Sibson" > gpurun_out/jfa_tests.log 2>&1 || { tail -30 gpurun_out/jfa_tests.log; exit 5; }
tail -1 gpurun_out/jfa_tests.log
FOVRT_SIB_STRIP_MID=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "sibson or Sibson" > gpurun_out/mid_tests.log 2>&1 || { tail -30 gpurun_out/mid_tests.log; exit 6; }
tail -1 gpurun_out/mid_tests.log
FOVRT_JFA_TAIL=0 bash scripts/stage_kernels.sh stagek_tail0 > gpurun_out/stagek_tail0.txt || exit 3
bash scripts/stage_kernels.sh stagek_tail1 > gpurun_out/stagek_tail1.txt || exit 4
FOVRT_SIB_STRIP_MID=1 bash scripts/stage_kernels.sh stagek_mid1 > gpurun_out/stagek_mid1.txt || exit 7
for t in tail0 tail1 mid1; do echo "== $t"; grep -h "jfa\|sibson\|geometry=" gpurun_out/stagek_$t.txt gpurun_out/stagek_$t/out.txt; done
for m in 0 1; do echo "mid $m"; FOVRT_SIB_STRIP_MID=$m timeout -k 10 300 python scripts/gaze_probe.py c 45 90 180 || exit 8; done
