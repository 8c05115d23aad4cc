#!/bin/bash
# Kernel trace of a short pipelined bench run (for timeline analysis with scripts/timeline.py):
#   scripts/trace_timeline.sh TAG [bench args]   (FOVRT_LIB selects a variant library)
set -eo pipefail
TAG=${1:?tag}; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/tl_$TAG
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$OUT" -o run -- \
  python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline "$@" > "$OUT/bench.json" 2> "$OUT/err.log"
