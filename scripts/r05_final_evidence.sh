#!/bin/bash
# Round-5 closing run: the whole GPU suite, then the evidence (kernel stats, HBM traffic, every config in both
# pipeline modes, stage / gaze / rebuild probes) under the given tag.
set -o pipefail
TAG=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
bash scripts/r05_evidence.sh "$TAG" || exit 2
