#!/bin/bash
# per-class C3 shading stats (the miss-class bound), gaze probe, shard model (bunny)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q -s --timeout 250 --timeout-method thread -k "c3_shading or c2_shading" > gpurun_out/r06i_fullsize.log 2>&1 || { tail -30 gpurun_out/r06i_fullsize.log; exit 1; }
grep -a "per class" gpurun_out/r06i_fullsize.log
timeout -k 10 200 python scripts/gaze_probe.py > gpurun_out/r06i_gaze_probe.txt 2>&1 || exit 2
cat gpurun_out/r06i_gaze_probe.txt
timeout -k 10 500 python scripts/shard_model.py bunny > gpurun_out/r06i_shard_model_bunny.jsonl 2>&1 || exit 3
cat gpurun_out/r06i_shard_model_bunny.jsonl | cut -c1-300
