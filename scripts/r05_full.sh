#!/bin/bash
# Full GPU suite, the bench line (twice) and Sibson alone per gaze (default build, then exp/lib_wm0.so: no run merging).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full_tests.log 2>&1 || { tail -30 gpurun_out/full_tests.log; exit 1; }
tail -2 gpurun_out/full_tests.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/full_bench_$i.log 2>&1 || { tail -5 gpurun_out/full_bench_$i.log; exit 2; }
  python - gpurun_out/full_bench_$i.log <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(j['value'], j['fps'], j['fps_serial'], j['roofline']['megakernel_ms'], j['stages']['sibson'])
PY
done
timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/full_gaze_on.txt 2>&1 || exit 3
FOVRT_LIB=$PWD/exp/lib_wm0.so timeout -k 10 150 python scripts/gaze_probe.py c 45 90 180 > gpurun_out/full_gaze_off.txt 2>&1 || exit 4
grep -H gaze gpurun_out/full_gaze_*.txt
