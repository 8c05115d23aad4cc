set -o pipefail
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || exit 1
for w in 8 16 24 32 48 64; do
  FOVRT_WAIT_THRESHOLD=$w timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_w$w.log 2>&1 || exit 2
done
FOVRT_WAIT_THRESHOLD=32 timeout -k 10 200 python scripts/diag_stamps.py > gpurun_out/diag.log 2>&1
