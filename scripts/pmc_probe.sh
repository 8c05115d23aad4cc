#!/bin/bash
# One rocprofv3 counter pass over a short bench run: scripts/pmc_probe.sh <name> "<counters>" [bench args...]
set -eo pipefail
NAME=${1:?name}
CTRS=${2:?counters}
shift 2
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/pmc_$NAME
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc $CTRS -f csv -d "$OUT" -o run -- \
  python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline "$@" > "$OUT/bench.json" 2> "$OUT/err.log"
