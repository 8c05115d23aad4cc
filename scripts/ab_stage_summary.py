#!/usr/bin/env python3
"""Mean [min, max] per stage and variant of an ab_stage.sh run (gpurun_out/stage_<name>_<i>.log)."""
import collections, glob, re, statistics

runs = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/stage_*.log"):
    name = re.match(r"gpurun_out/stage_(.*)_\d+\.log", f).group(1)
    line = [l for l in open(f).read().splitlines() if "ms (median" in l]
    if not line:
        continue
    for k, v in re.findall(r"(\w+)=([\d.]+)", line[-1]):
        runs[name][k].append(float(v))
stages = ["geometry", "sampling", "optimize", "shading", "jfa", "sibson", "pullpush", "atrous"]
print(f"{'variant':12s} " + " ".join(f"{s:>16s}" for s in stages))
for name, d in sorted(runs.items()):
    print(f"{name:12s} " + " ".join(f"{statistics.mean(d[s]):7.3f}[{min(d[s]):.3f}]" if d[s] else " " * 16 for s in stages))
