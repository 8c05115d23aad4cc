#!/bin/bash
# Stages alone (scripts/stage_probe.py) plus their per-kernel rocprofv3 stats: scripts/stage_prof.sh TAG
set -eo pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/stage_$TAG
mkdir -p "$OUT"
timeout -k 10 200 python3 "$ROOT/scripts/stage_probe.py" 10 > "$OUT/probe.txt" 2>&1
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- \
  python3 "$ROOT/scripts/stage_probe.py" 30 > "$OUT/probe_prof.txt" 2>&1
