#!/bin/bash
# Megakernel time against the amount of work (critical path vs throughput): bunny at 4K with 1/2/4/8
# spp, 1080p at 4 spp, and the refraction cap. Lines in gpurun_out/sp_*.log.
set -o pipefail
mkdir -p gpurun_out
run() {
  local name=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 "$@" > gpurun_out/sp_$name.log 2>&1 || { tail -5 gpurun_out/sp_$name.log; exit 1; }
}
for s in 1 2 4 8; do run 4k_spp$s --spp $s; done
run 1080_spp4 --width 1920 --height 1080
run 1080_spp4_dmd1 --width 1920 --height 1080 --dmd 1
run 1080_spp4_dmd1_rmd8 --width 1920 --height 1080 --dmd 1 --refraction-max-depth 8
run 4k_rmd8 --refraction-max-depth 8
run 540_spp4 --width 960 --height 540
