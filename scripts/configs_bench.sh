#!/bin/bash
# One bench line per BASELINE.json config that fits one GPU (configs[3]/[4] as their one-GPU share:
# one 4K vokselia view; the 4/8-GPU tilings themselves run under the driver's multi-GPU bench):
#   scripts/configs_bench.sh  ->  gpurun_out/cfg_C*.log (summary: scripts/configs_summary.py)
set -o pipefail
mkdir -p gpurun_out
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-frames 1 "$@" > gpurun_out/cfg_$name.log 2>&1 || { tail -5 gpurun_out/cfg_$name.log; exit 1; }
  echo "$name done"
}
run C1 --scene box --width 512 --height 512 --spp 1 --dmd 1 --mask uniform
run C2 --scene bunny --width 1920 --height 1080 --spp 4 --dmd 1 --mask logpolar10
run C3 --no-cpu-baseline
# C3 with an eye-tracked gaze (the log-polar mask recomputed each frame): the full cursor circle (360 timed
# frames, one degree each), and saccades (90 degrees every 30 frames); frame_clock_pipelined has p50/p99/max
run C3gaze --no-cpu-baseline --gaze-path circle --steps 360 --warmup 5 --serial-frames 360
run C3sacc --no-cpu-baseline --gaze-path saccade --steps 360 --warmup 5 --serial-frames 360
run C4 --no-cpu-baseline --scene vokselia --spp 8 --dmd 1 --mask saliency
run C5 --no-cpu-baseline --scene vokselia --spp 8 --dmd 3 --mask saliency
