#!/bin/bash
set -o pipefail
FOVRT_JFA_LAZY_OUTPUTS=1 bash scripts/stage_kernels.sh r06o_lazy > gpurun_out/r06o_lazy.txt 2>&1 || exit 1
FOVRT_JFA_LAZY_OUTPUTS=0 bash scripts/stage_kernels.sh r06o_eager > gpurun_out/r06o_eager.txt 2>&1 || exit 2
echo LAZY; grep -i "sibson\|jfa\|fill" gpurun_out/r06o_lazy.txt
echo EAGER; grep -i "sibson\|jfa\|fill" gpurun_out/r06o_eager.txt
