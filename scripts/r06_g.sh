#!/bin/bash
set -o pipefail
for L in - abv/lib_chain0.so abv/lib_chain1.so; do
  if [ "$L" = "-" ]; then unset FOVRT_LIB; else export FOVRT_LIB=$PWD/$L; fi
  echo "$L $(timeout -k 10 120 python scripts/frame_digest.py 3840 2160 4 3)" || exit 1
  echo "$L $(timeout -k 10 120 python scripts/frame_digest.py 1920 1080 4 3)" || exit 1
done
unset FOVRT_LIB
bash scripts/ab_bench.sh r06g 3 chain2:- chain0:FOVRT_LIB=$PWD/abv/lib_chain0.so chain1:FOVRT_LIB=$PWD/abv/lib_chain1.so || exit 2
