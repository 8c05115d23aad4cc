#!/bin/bash
# shard model (bunny) for the in-tree library and exp/ variants, after the group tests
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "schedule or handoff or group" > gpurun_out/gpu_tests.log 2>&1; tail -1 gpurun_out/gpu_tests.log
for L in foveated-rendering-using-ray-tracing_amd/libfovrt.so exp/lib_nospread.so exp/lib_chunk.so; do
  n=$(basename $L .so); FOVRT_LIB=$L timeout -k 10 400 python scripts/shard_model.py bunny > gpurun_out/sm_$n.jsonl 2>/dev/null || exit 3
done
echo done
