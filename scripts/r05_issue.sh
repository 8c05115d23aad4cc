#!/bin/bash
# SQ / L2 counter passes of the bench workload (scripts/pmc_sq.sh) for profiles/<tag>_pmc_issue.json.
set -o pipefail
mkdir -p gpurun_out
bash scripts/pmc_sq.sh || exit 1
ls gpurun_out/pmc_sq1 gpurun_out/pmc_sq2 | head
