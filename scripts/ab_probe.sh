#!/bin/bash
# Stages-alone probe (scripts/stage_probe.py) for the default build and each variant library:
#   scripts/ab_probe.sh exp/lib_A.so ...   -> one line per library
set -o pipefail
echo "default $(timeout -k 10 120 python scripts/stage_probe.py 10 2>&1 | tail -1)"
for L in "$@"; do
  echo "$(basename $L .so) $(FOVRT_LIB=$L timeout -k 10 120 python scripts/stage_probe.py 10 2>&1 | tail -1)"
done
