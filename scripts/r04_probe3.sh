#!/bin/bash
# BVH builder changes (tests, rebuild probe), then the G = 4 / 8 group model with two reconstruction costs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "bvh or BVH or rebuild or positions" > gpurun_out/bvh_tests.log 2>&1 || { tail -30 gpurun_out/bvh_tests.log; exit 5; }
tail -1 gpurun_out/bvh_tests.log
timeout -k 10 120 python scripts/rebuild_probe.py > gpurun_out/r04d_rebuild_probe.txt 2>&1 || exit 1
cat gpurun_out/r04d_rebuild_probe.txt
for rc in 0.5,0.17 0.5,0.12; do
  FOVRT_MODEL_LAYOUTS=4:1,8:2 FOVRT_RECON_COST=$rc timeout -k 10 400 python scripts/shard_model.py bunny > gpurun_out/r04d_model_$rc.jsonl 2>&1 || exit 2
  echo "recon_cost $rc"; python3 -c "
import json,sys
for l in open('gpurun_out/r04d_model_$rc.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d.get('G'), d.get('jfa_ranks'), d.get('tiles'), d.get('model_frame_ms_form2', d.get('pipelined_frame_ms')), d.get('speedup_form2'))
"
done
