#!/bin/bash
set -o pipefail
for L in - abv/lib_jfa0.so; do
  if [ "$L" = "-" ]; then unset FOVRT_LIB; else export FOVRT_LIB=$PWD/$L; fi
  echo "$L $(timeout -k 10 120 python scripts/frame_digest.py 3840 2160 4 2)" || exit 1
done
unset FOVRT_LIB
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "jfa or sibson or frame" > gpurun_out/${TAG:-r06m}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG:-r06m}_tests.log; exit 2; }
tail -1 gpurun_out/${TAG:-r06m}_tests.log
AB_KERNELS="k_jfa_step k_jfa_init k_jfa_final" bash scripts/ab_lib_stage.sh ${TAG:-r06m} 3 skip:- noskip:abv/lib_jfa0.so || exit 3
bash scripts/stage_kernels.sh ${TAG:-r06m}_sk > gpurun_out/${TAG:-r06m}_sk.txt 2>&1; grep jfa gpurun_out/${TAG:-r06m}_sk.txt
