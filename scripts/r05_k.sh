#!/bin/bash
set -o pipefail
ROOT=$(pwd)
mkdir -p gpurun_out/tl_lat
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d "$ROOT/gpurun_out/tl_lat" -o run -- python3 "$ROOT/scripts/latency_probe.py" latency 14 > "$ROOT/gpurun_out/tl_lat/out.txt" 2>&1 || exit 1
cd "$ROOT"
python3 scripts/timeline2.py gpurun_out/tl_lat 8 2 > gpurun_out/tl_lat/timeline.txt
head -3 gpurun_out/tl_lat/timeline.txt
