#!/bin/bash
# Per-kernel durations of the stages run alone (scripts/stage_probe.py): rocprofv3 kernel trace ->
# gpurun_out/${1:-stagek}/ (stats csv) and a summary line per kernel.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-stagek}
cd /tmp
export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 150 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o run -- python3 "$ROOT/scripts/stage_probe.py" 5 > "$OUT/out.txt" 2>&1 || exit 1
f=$(find "$OUT" -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:40]:
    print(f'{float(r["AverageNs"])/1e3:9.1f} us avg {float(r["MinNs"])/1e3:9.1f} min x{int(r["Calls"]):5d}  {r["Name"][:110]}')
PY
