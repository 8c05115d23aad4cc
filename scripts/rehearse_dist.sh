#!/bin/bash
# Multi-process rehearsal of bench.py's distributed paths on a one-GPU box (gloo, both ranks on
# GPU 0): 2 views x 1 rank (weak scaling), 1 view tile-sharded over 2 ranks (sparse gather of the traced
# pixels), the same with a moving camera (tile slabs + HISTORY_CACHE all-gather), and 3 ranks with the
# tile-slab gather.
set -eo pipefail
export FOVRT_DIST_BACKEND=gloo
A="--steps 3 --warmup 1 --width 1920 --height 1080 --no-cpu-baseline"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py $A --views 2 --composite > gpurun_out/rehearse_views.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29512 bench.py $A --views 1 --tile 128 > gpurun_out/rehearse_tiles.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29513 bench.py $A --views 1 --tile 128 --pan 0.02 > gpurun_out/rehearse_pan.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 \
  --master-port 29514 bench.py $A --views 1 --tile 128 --dense-gather > gpurun_out/rehearse_dense.log 2>&1
