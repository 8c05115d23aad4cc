#!/bin/bash
set -o pipefail
for L in 1 0; do
  echo "lazy=$L $(FOVRT_JFA_LAZY_OUTPUTS=$L timeout -k 10 120 python scripts/frame_digest.py 3840 2160 4 2)" || exit 1
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06p_tests.log 2>&1 || { tail -30 gpurun_out/r06p_tests.log; exit 2; }
tail -1 gpurun_out/r06p_tests.log
rm -f gpurun_out/stage_lazy_* gpurun_out/stage_eager_*
bash scripts/ab_stage.sh 3 lazy:FOVRT_JFA_LAZY_OUTPUTS=1 eager:FOVRT_JFA_LAZY_OUTPUTS=0 || exit 3
for f in gpurun_out/stage_lazy_*.log gpurun_out/stage_eager_*.log; do echo "$f $(cat $f)"; done
bash scripts/ab_bench.sh r06p 3 lazy:FOVRT_JFA_LAZY_OUTPUTS=1 eager:FOVRT_JFA_LAZY_OUTPUTS=0 || exit 4
bash scripts/ab_lib_stage.sh r06q 3 w7:- w6:abv/lib_siw6.so || exit 5
