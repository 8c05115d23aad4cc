#!/bin/bash
# The default bench line N times in a row on one box (run-to-run spread): scripts/bench_repeat.sh N [args]
set -o pipefail
N=${1:?n}; shift
for i in $(seq 1 "$N"); do
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/brep_$i.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/brep_$i.log') if l.startswith('{')][-1]); print(d['fps'], d['ms_per_step'], d['roofline']['megakernel_ms'])"
done
