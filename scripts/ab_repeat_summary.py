#!/usr/bin/env python3
"""Mean / min / max fps and megakernel ms per variant of an ab_repeat.sh run (gpurun_out/rep_*.log)."""
import collections, glob, json, re, statistics

runs = collections.defaultdict(list)
for f in glob.glob("gpurun_out/rep_*.log"):
    name = re.match(r"gpurun_out/rep_(.*)_\d+\.log", f).group(1)
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:
        continue
    runs[name].append((d["fps"], d["roofline"].get("megakernel_ms", 0.0), d["stages"]["shading"]["ms"]))
for name, v in sorted(runs.items()):
    fps = [x[0] for x in v]
    mk = [x[1] for x in v]
    sh = [x[2] for x in v]
    print(f"{name:14s} n={len(v)} fps mean {statistics.mean(fps):7.2f} [{min(fps):.2f}, {max(fps):.2f}]  "
          f"mk {statistics.mean(mk):.3f} ms  shading(serialised) {statistics.mean(sh):.3f} ms")
