#!/bin/bash
# Interleaved A/B of environment settings on BASELINE configs (AB_CONFIGS, default "C2 C4 C1"; 40 timed frames):
#   scripts/ab_configs.sh <reps> "name:VAR=val" ...  -> gpurun_out/abc_<cfg>_<name>_<i>.log
set -o pipefail
R=${1:?reps}; shift
mkdir -p gpurun_out
declare -A ARGS=([C1]="--scene box --width 512 --height 512 --spp 1 --dmd 1 --mask uniform"
                 [C2]="--scene bunny --width 1920 --height 1080 --spp 4 --dmd 1 --mask logpolar10"
                 [C3]=""
                 [C4]="--scene vokselia --spp 8 --dmd 1 --mask saliency")
for i in $(seq 1 "$R"); do
  for c in ${AB_CONFIGS:-C2 C4 C1}; do
    for spec in "$@"; do
      n=${spec%%:*}; vars=${spec#*:}
      env $vars timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 --warmup 20 ${ARGS[$c]} \
        > gpurun_out/abc_${c}_${n}_$i.log 2>&1 || exit 2
    done
  done
done
python3 - <<'PY'
import glob, json, re, collections, statistics
r = collections.defaultdict(list)
for f in glob.glob("gpurun_out/abc_*.log"):
    c, n, i = re.match(r"gpurun_out/abc_(C\d)_(.*)_(\d+)\.log", f).groups()
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    r[(c, n)].append(d["fps"])
for k in sorted(r):
    print(k, "fps mean %.1f" % statistics.mean(r[k]), [round(x, 1) for x in r[k]])
PY
