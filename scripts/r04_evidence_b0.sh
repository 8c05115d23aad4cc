#!/bin/bash
# The JFA / Sibson GPU tests of the current build, then evidence part B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "jfa or JFA or jump or Jump or sibson or Sibson" > gpurun_out/jfa_tests.log 2>&1 || { tail -30 gpurun_out/jfa_tests.log; exit 5; }
tail -1 gpurun_out/jfa_tests.log
bash scripts/r04_evidence_b.sh "$@"
