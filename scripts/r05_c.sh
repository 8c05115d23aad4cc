#!/bin/bash
# Round 5: the new GPU tests (latency pipeline mode, strip kernel on whole images), one bench line with
# both pipeline modes, and the rebuild hitch probe with GPU phase times under loading/warm-up variants.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "latency_pipeline or sibson_strip or pipelined or frame_driver" > gpurun_out/gpu_new.log 2>&1 || { tail -40 gpurun_out/gpu_new.log; exit 1; }
tail -3 gpurun_out/gpu_new.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05c_bench.log 2>&1 || { tail -5 gpurun_out/r05c_bench.log; exit 2; }
python - <<'EOF'
import json
j = json.loads([l for l in open('gpurun_out/r05c_bench.log') if l.startswith('{')][-1])
print(j['value'], j['fps'], j['fps_serial'], j['roofline']['megakernel_ms'], j['bvh']['rebuild_ms'])
print('latency', j.get('pipeline_latency_mode'))
print('lat', j.get('latency'))
EOF
run() { local name=$1; shift; env "$@" timeout -k 10 120 python scripts/rebuild_probe.py $SC > gpurun_out/rb_$name.log 2>&1 || exit 3; }
SC="1 2"; run phases FOVRT_BVH_PHASES=1
SC="1 2"; run eager_phases FOVRT_BVH_PHASES=1 HIP_ENABLE_DEFERRED_LOADING=0
SC="2 1"; run eager_rev HIP_ENABLE_DEFERRED_LOADING=0
SC="1 2"; run warm1 FOVRT_BVH_WARMUP=1
SC="1 2"; run warm2 FOVRT_BVH_WARMUP=2
SC="1 2"; run eager_warm1 FOVRT_BVH_WARMUP=1 HIP_ENABLE_DEFERRED_LOADING=0
for f in phases eager_phases eager_rev warm1 warm2 eager_warm1; do echo "== $f"; grep -v "^bvh phase" gpurun_out/rb_$f.log; done
echo "== phases (first 3 builds of each scene)"; grep "^bvh phase" gpurun_out/rb_phases.log | head -21
