#!/bin/bash
# Round-5 check of the PTX-faithful build: GPU suite, two bench lines (driver command), and the rebuild
# probe under environment variants (lazy code-object loading off, phase timing).
set -o pipefail
mkdir -p gpurun_out
K=${1:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05b_bench_$i.log 2>&1 || { tail -5 gpurun_out/r05b_bench_$i.log; exit 2; }
done
python scripts/r05_ab_rev_summary.py gpurun_out 2>/dev/null | head -1
for f in gpurun_out/r05b_bench_*.log; do python -c "
import json,sys
j=json.loads([l for l in open('$f') if l.startswith('{')][-1])
r=j['roofline']
print('$f', j['value'], j['fps'], j['fps_serial'], r['megakernel_ms'], r['megakernel_ms_serialised'], j['bvh']['rebuild_ms'])
"; done
timeout -k 10 120 python scripts/rebuild_probe.py > gpurun_out/rb_default.log 2>&1 || exit 3
HIP_ENABLE_DEFERRED_LOADING=0 timeout -k 10 120 python scripts/rebuild_probe.py > gpurun_out/rb_eager.log 2>&1 || exit 4
FOVRT_BVH_PHASES=1 timeout -k 10 120 python scripts/rebuild_probe.py > gpurun_out/rb_phases.log 2>&1 || exit 5
for f in rb_default rb_eager rb_phases; do echo "== $f"; grep -v "^bvh phase" gpurun_out/$f.log; done
