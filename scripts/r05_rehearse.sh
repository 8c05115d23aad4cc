#!/bin/bash
# The multi-rank bench path rehearsed on one device (--local-ranks: contexts of one process, peer copies instead of
# RCCL): 2 and 4 ranks on one 4K view, and 2 views with the composite. Not scaling measurements.
set -o pipefail
mkdir -p gpurun_out
for args in "--local-ranks 2" "--local-ranks 4" "--local-ranks 2 --views 2 --composite"; do
  timeout -k 10 240 python bench.py $args --steps 10 --warmup 3 --no-cpu-baseline --serial-frames 10 > gpurun_out/rehearse.log 2>&1 || { tail -20 gpurun_out/rehearse.log; exit 1; }
  python - gpurun_out/rehearse.log "$args" <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], '->', j['value'], j['fps'], j['config'].get('parallelism'))
PY
done
