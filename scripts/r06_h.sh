#!/bin/bash
# GPU suite, then the eye-tracked circle bench under a kernel trace (per-kernel time of the eye-tracked frame)
set -o pipefail
ROOT=$(pwd)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06h_tests.log 2>&1 || { tail -30 gpurun_out/r06h_tests.log; exit 1; }
tail -1 gpurun_out/r06h_tests.log
cd /tmp && export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/r06h_circle
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT -o run -- python3 $ROOT/bench.py --no-cpu-baseline --gaze-path circle --steps 60 --warmup 20 --serial-frames 20 > $OUT/bench.json 2> $OUT/err.log || { tail $OUT/err.log; exit 2; }
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/tot*100:5.1f}% {float(r["AverageNs"])/1e3:9.1f} us avg x{int(r["Calls"]):5d}  {r["Name"][:90]}')
PY
