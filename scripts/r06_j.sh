#!/bin/bash
# latency-form megakernel: bit-identity against the throughput form, GPU tests, 1080p C2 A/B, shard model
set -o pipefail
for L in 0 2; do
  echo "lat=$L $(FOVRT_SHADE_LAT=$L timeout -k 10 120 python scripts/frame_digest.py 1920 1080 4 3)" || exit 1
  echo "lat=$L $(FOVRT_SHADE_LAT=$L timeout -k 10 120 python scripts/frame_digest.py 3840 2160 4 2)" || exit 1
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "shade or megakernel or handoff or group or c2 or frame" > gpurun_out/r06j_tests.log 2>&1 || { tail -30 gpurun_out/r06j_tests.log; exit 2; }
tail -1 gpurun_out/r06j_tests.log
BENCH_ARGS="--scene bunny --width 1920 --height 1080 --spp 4 --dmd 1 --mask logpolar10" bash scripts/ab_bench.sh r06j 3 lat:- nolat:FOVRT_SHADE_LAT=0 || exit 3
timeout -k 10 500 python scripts/shard_model.py bunny > gpurun_out/r06j_shard_model_bunny.jsonl 2>&1 || exit 4
