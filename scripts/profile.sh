#!/bin/bash
# Per-round profile of the bench workload on the GPU box (run through gpurun):
#   1. rocprofv3 --kernel-trace --stats      -> per-kernel average durations (the default bench command;
#                                               the CPU baseline launches no kernel and is skipped)
#   2. rocprofv3 --pmc FETCH_SIZE            -> HBM read bytes per dispatch   (own pass)
#   3. rocprofv3 --pmc WRITE_SIZE            -> HBM write bytes per dispatch  (own pass)
#   4. scripts/pmc_traffic.py                -> profiles/<tag>_pmc_traffic.json (read by bench.py)
# Usage: scripts/profile.sh <tag> [bench args...]
set -eo pipefail
TAG=${1:?tag}
shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT" "$ROOT/profiles"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline "$@" > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/fetch" -o run -- \
  python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline "$@" > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/write" -o run -- \
  python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline "$@" > "$OUT/bench_write.json" 2> "$OUT/write.err"
python3 "$ROOT/scripts/pmc_traffic.py" "$OUT" "$TAG" "$@"
