#!/bin/bash
# Megakernel traversal steps per wave-wide ballot: 3 (default) against 2 (exp/lib_tu2.so) and 4 (exp/lib_tu4.so),
# two interleaved bench triples under the driver's command.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/tu_3_$i.log 2>&1 || exit 1
  FOVRT_LIB=$PWD/exp/lib_tu2.so timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/tu_2_$i.log 2>&1 || exit 2
  FOVRT_LIB=$PWD/exp/lib_tu4.so timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/tu_4_$i.log 2>&1 || exit 3
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/tu_*.log")):
    j = json.loads([l for l in open(f) if l.startswith("{")][-1])
    r = j["roofline"]
    print(f, j["value"], j["fps"], r["megakernel_ms"], r.get("megakernel_ms_serialised"))
PY
