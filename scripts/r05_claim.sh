#!/bin/bash
# Strip claims with a wave-wide look at the lists: the Sibson GPU tests, Sibson alone per gaze twice, one bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sibson or golden" \
  > gpurun_out/claim_tests.log 2>&1 || { tail -30 gpurun_out/claim_tests.log; exit 1; }
tail -1 gpurun_out/claim_tests.log
for i in 1 2; do
  timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/claim_$i.txt 2>&1 || exit 2
done
grep -H gaze gpurun_out/claim_*.txt
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/claim_bench.log 2>&1 || exit 3
python - gpurun_out/claim_bench.log <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(j['value'], j['fps'], j['fps_serial'], j['roofline']['megakernel_ms'], j['stages']['sibson'])
PY
