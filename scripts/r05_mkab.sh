#!/bin/bash
# Megakernel change A/B: the full GPU suite on the default build, then interleaved bench pairs against
# exp/lib_mk0.so (the build before the change), under the driver's bench command.
set -o pipefail
mkdir -p gpurun_out
P=${1:-3}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mkab_tests.log 2>&1 || { tail -30 gpurun_out/mkab_tests.log; exit 1; }
tail -1 gpurun_out/mkab_tests.log
for i in $(seq 1 $P); do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/mkab_new_$i.log 2>&1 || exit 2
  FOVRT_LIB=$PWD/exp/lib_mk0.so timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/mkab_old_$i.log 2>&1 || exit 3
  echo "pair $i done"
done
python - <<'PY'
import json, glob
for tag in ("new", "old"):
    for f in sorted(glob.glob(f"gpurun_out/mkab_{tag}_*.log")):
        j = json.loads([l for l in open(f) if l.startswith("{")][-1])
        r = j["roofline"]
        print(tag, j["value"], j["fps"], j["fps_serial"], r["megakernel_ms"], r.get("megakernel_ms_serialised"))
PY
