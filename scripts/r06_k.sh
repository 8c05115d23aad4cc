#!/bin/bash
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "latency or pipelined or frame or sibson or snapshot" > gpurun_out/r06k_tests.log 2>&1 || { tail -30 gpurun_out/r06k_tests.log; exit 1; }
tail -1 gpurun_out/r06k_tests.log
bash scripts/ab_bench.sh r06k 3 new:- old:FOVRT_LIB=$PWD/abv/lib_old.so || exit 2
