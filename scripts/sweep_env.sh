#!/bin/bash
# bench.py under a list of environment settings: scripts/sweep_env.sh "VAR=a" "VAR=b" ...
set -o pipefail
i=0
for e in "$@"; do
  env $e timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/sweep_$i.log 2>&1 || exit 1
  echo "$e" > gpurun_out/sweep_$i.env
  i=$((i+1))
done
