#!/bin/bash
# End-of-round evidence on the GPU box: the default bench line, its rocprof kernel trace and HBM
# counters (scripts/profile.sh), and one bench line per BASELINE config (scripts/configs_bench.sh).
#   scripts/round_profile.sh <tag>   ->  gpurun_out/<tag>_bench.log, gpurun_out/prof_<tag>/, gpurun_out/cfg_C*.log
set -eo pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
mkdir -p gpurun_out
bash scripts/profile.sh "$TAG"
echo "profile done"
timeout -k 10 400 python bench.py > "gpurun_out/${TAG}_bench.log" 2>&1
echo "bench done"
bash scripts/configs_bench.sh
