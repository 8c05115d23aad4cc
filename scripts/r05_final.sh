#!/bin/bash
# Round-5 final check: the whole GPU suite (-v, so the new cases are named) and two bench lines under the driver's command.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || { tail -40 gpurun_out/final_tests.log; exit 1; }
grep -E "binade|passed|failed" gpurun_out/final_tests.log | tail -4
for i in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final_bench_$i.log 2>&1 || { tail -5 gpurun_out/final_bench_$i.log; exit 2; }
  tail -1 gpurun_out/final_bench_$i.log | cut -c1-300
done
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 3; }
tail -1 gpurun_out/final_smoke.log
