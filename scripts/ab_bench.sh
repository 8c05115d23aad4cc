#!/bin/bash
# Interleaved A/B of the bench under environment settings (FOVRT_LIB=abv/lib_x.so selects a library build):
#   scripts/ab_bench.sh <tag> <reps> "name:VAR=val VAR2=val" ...  [BENCH_ARGS="--gaze-path" ...]
# Every rep runs each variant once (box drift hits them alike); one summary line per run in
# gpurun_out/<tag>_summary.txt: Mrays/s, pipelined fps, megakernel ms (timed region / serialised), latency-mode fps,
# serial fps (mean).
set -o pipefail
TAG=${1:?tag}; R=${2:?reps}; shift 2
mkdir -p gpurun_out
S=gpurun_out/${TAG}_summary.txt
: > "$S"
for i in $(seq 1 "$R"); do
  for spec in "$@"; do
    n=${spec%%:*}; vars=${spec#*:}
    [ "$vars" = "-" ] && vars=""
    L=gpurun_out/${TAG}_${n}_$i.json
    env $vars timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 --warmup 20 --serial-frames 20 $BENCH_ARGS > "$L" 2> "${L%.json}.err" || { tail -5 "${L%.json}.err"; exit 2; }
    python3 - "$L" "$n" "$i" <<'PY' | tee -a "$S"
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; lm = d.get("pipeline_latency_mode") or {}
st = " ".join(f"{k}={v['ms']:.3f}" for k, v in d["stages"].items())
print(f"{sys.argv[2]:10s} {sys.argv[3]} {d['value']:8.1f} Mrays/s {d['fps']:7.2f} fps mk {r['megakernel_ms']:.3f}/{r['megakernel_ms_serialised']:.3f} "
      f"lat {lm.get('fps', 0):7.2f} serial {d['fps_serial_mean']:7.2f} | {st}")
PY
  done
done
