#!/bin/bash
# Round 5: does the warm-up length move the timed region? (driver's 20/5 against 20/60), interleaved.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for w in 5 60; do
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup $w --no-cpu-baseline --serial-frames 10 > gpurun_out/r05o_w${w}_$i.log 2>&1 || exit 1
    python - gpurun_out/r05o_w${w}_$i.log <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[1].split('/')[-1], j['value'], j['fps'], j['roofline']['megakernel_ms'])
PY
  done
done
