#!/bin/bash
# Sibson strip kernel A/B on the wide-hole mask and the probe gazes, with kernel traces.
set -o pipefail
mkdir -p gpurun_out
for v in 0 1; do
  FOVRT_SIB_STRIP=$v timeout -k 10 200 python scripts/sib_mask_probe.py 3 || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_sibmask -o sm -- python3 $GRAFT_REPO_ROOT/scripts/sib_mask_probe.py 2 > $GRAFT_REPO_ROOT/gpurun_out/sibmask_prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/sibmask_prof.log; exit 2; }
echo prof ok
cd $GRAFT_REPO_ROOT && bash scripts/r04_sib_ab.sh
