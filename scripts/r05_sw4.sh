#!/bin/bash
# Megakernel at 4 waves/SIMD (exp/lib_sw4.so: 128 VGPRs, 76 spilled) against 3 (default, 168 VGPRs): two interleaved
# bench pairs under the driver's command (the default build's line also shows roofline.issue).
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/sw4_def_$i.log 2>&1 || exit 1
  FOVRT_LIB=$PWD/exp/lib_sw4.so timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/sw4_4_$i.log 2>&1 || exit 2
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/sw4_*.log")):
    j = json.loads([l for l in open(f) if l.startswith("{")][-1])
    r = j["roofline"]
    print(f, j["value"], j["fps"], r["megakernel_ms"], r.get("megakernel_ms_serialised"), "issue" in r)
PY
