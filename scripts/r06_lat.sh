#!/bin/bash
# Kernel trace of C3 frames in latency mode (static gaze): per-frame timeline
set -o pipefail
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/r06_lat
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $OUT -o run -- python3 $ROOT/scripts/latency_probe.py latency 30 > $OUT/out.txt 2>&1 || exit 1
f=$(find $OUT -name "*kernel_trace.csv" | head -1)
python3 $ROOT/scripts/lat_timeline.py $f | tail -12
python3 - "$f" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ev = [(r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fr::", "")[:28], int(r["Start_Timestamp"]) / 1e3, int(r["End_Timestamp"]) / 1e3) for r in rows]
g = [i for i, e in enumerate(ev) if e[0].startswith("k_gbuffer")]
i0, i1 = g[-4], g[-2]
t0 = ev[i0][1]
for e in ev[i0:i1]:
    print(f"{e[1]-t0:9.1f} {e[2]-t0:9.1f} {e[2]-e[1]:8.1f}  {e[0]}")
PY
