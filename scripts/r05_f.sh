#!/bin/bash
# Round 5: quantised BVH nodes (QNode). The GPU suite, two bench lines, then the rebuild hitch variants.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05f_bench_$i.log 2>&1 || { tail -5 gpurun_out/r05f_bench_$i.log; exit 2; }
  python - gpurun_out/r05f_bench_$i.log <<'EOF'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
r = j['roofline']
print(j['value'], j['fps'], j['fps_serial'], r['megakernel_ms'], r.get('megakernel_ms_serialised'), j['bvh']['rebuild_ms'])
print('latency mode', j.get('pipeline_latency_mode'))
EOF
done
bash scripts/r05_e.sh
