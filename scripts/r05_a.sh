#!/bin/bash
# Round-5 first call: interleaved A/B of the round-3 final tree (exp/r03) against HEAD under the driver's
# bench command, then the rebuild probe under a HIP runtime + kernel trace (where do the slow rebuilds go).
set -o pipefail
mkdir -p gpurun_out
bash scripts/r05_ab_rev.sh 4 r03 || exit 1
python scripts/r05_ab_rev_summary.py > gpurun_out/abrev_summary.txt && cat gpurun_out/abrev_summary.txt
timeout -k 10 120 python scripts/rebuild_probe.py > gpurun_out/rebuild_probe.log 2>&1 || { tail -5 gpurun_out/rebuild_probe.log; exit 3; }
cat gpurun_out/rebuild_probe.log
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --stats -f csv \
  -d $R/gpurun_out/prof_rebuild -o rb -- python3 $R/scripts/rebuild_probe.py > $R/gpurun_out/rebuild_prof.log 2>&1 \
  || { tail -5 $R/gpurun_out/rebuild_prof.log; exit 4; }
echo prof ok
