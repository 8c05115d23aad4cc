#!/bin/bash
# Round 6 start: GPU suite, the driver's bench command, stages alone.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06a_tests.log 2>&1 || { tail -30 gpurun_out/r06a_tests.log; exit 1; }
tail -2 gpurun_out/r06a_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r06a_bench.json 2> gpurun_out/r06a_bench.err || { tail -5 gpurun_out/r06a_bench.err; exit 2; }
python -c "import json;d=json.load(open('gpurun_out/r06a_bench.json'));print(d['value'],d['fps'],d['fps_serial'],d['roofline']['megakernel_ms'],d['roofline']['megakernel_ms_serialised'],d['pipeline_latency_mode']['fps'],d['fps_serial_mean'])"
timeout -k 10 200 python scripts/stage_probe.py 10 > gpurun_out/r06a_stage_probe.txt 2>&1 || exit 3
cat gpurun_out/r06a_stage_probe.txt
