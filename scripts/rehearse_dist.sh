#!/bin/bash
# One-GPU rehearsal of bench.py's multi-GPU modes: the ranks of a group as contexts of one process
# (fr_group with device-to-device copies; RCCL cannot put two ranks on one device). 1 view over 4 ranks
# (the default strong-scaling layout), the same with both chains on rank 0, a moving camera, and 2 views
# x 2 ranks with the stereo composite, and 8 ranks (JFA -> Sibson in turns on view ranks 0 and 2). Correctness of the path, not a scaling measurement.
set -eo pipefail
mkdir -p gpurun_out
A="--steps 4 --warmup 2 --width 1920 --height 1080 --no-cpu-baseline"
timeout -k 10 200 python bench.py $A --local-ranks 4 > gpurun_out/rehearse_tiles.log 2>&1
timeout -k 10 200 python bench.py $A --local-ranks 4 --no-split > gpurun_out/rehearse_nosplit.log 2>&1
timeout -k 10 200 python bench.py $A --local-ranks 2 --pan 0.02 > gpurun_out/rehearse_pan.log 2>&1
timeout -k 10 200 python bench.py $A --local-ranks 4 --views 2 --composite > gpurun_out/rehearse_views.log 2>&1
timeout -k 10 200 python bench.py $A --local-ranks 8 > gpurun_out/rehearse_eight.log 2>&1
tail -n1 gpurun_out/rehearse_*.log | cut -c1-400
