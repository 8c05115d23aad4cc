#!/bin/bash
# Round 5: the rebuild fix (host tree released at creation) and the latency mode's reconstruction ordering:
# targeted GPU tests, two bench lines, the rebuild probe.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "latency or pipelined or frame_driver" > gpurun_out/gpu_g.log 2>&1 || { tail -40 gpurun_out/gpu_g.log; exit 1; }
tail -2 gpurun_out/gpu_g.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05g_bench_$i.log 2>&1 || { tail -5 gpurun_out/r05g_bench_$i.log; exit 2; }
  python - gpurun_out/r05g_bench_$i.log <<'EOF'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
r = j['roofline']
print(j['value'], j['fps'], j['fps_serial'], r['megakernel_ms'], r.get('megakernel_ms_serialised'), j['bvh'])
print('latency mode', j.get('pipeline_latency_mode'))
print('throughput mode clock', j.get('frame_clock_pipelined'))
EOF
done
timeout -k 10 120 python scripts/rebuild_probe.py 1 2 > gpurun_out/rb_g.log 2>&1 || exit 3
cat gpurun_out/rb_g.log
