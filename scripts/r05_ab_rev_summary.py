"""Summary of scripts/r05_ab_rev.sh: per tree, value / fps / megakernel ms of every run and their means."""
import glob
import json
import os
import re
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
runs = {}
for p in sorted(glob.glob(os.path.join(d, "abrev_*_*.log"))):
    m = re.match(r"abrev_(.+)_(\d+)\.log", os.path.basename(p))
    line = [l for l in open(p) if l.startswith("{")]
    if not m or not line:
        continue
    j = json.loads(line[-1])
    r = j["roofline"]
    runs.setdefault(m.group(1), []).append((int(m.group(2)), j["value"], j["fps"], r["megakernel_ms"],
                                           r.get("megakernel_ms_serialised"), j.get("fps_serial")))
for tree, rs in runs.items():
    rs.sort()
    n = len(rs)
    mean = [sum(x[k] or 0 for x in rs) / n for k in range(1, 6)]
    print(f"{tree:10s} n={n} Mrays/s {mean[0]:8.1f} fps {mean[1]:6.1f} mk_live {mean[2]:.3f} mk_serial {mean[3]:.3f} "
          f"fps_serial {mean[4]:6.1f}")
    for x in rs:
        print(f"    run {x[0]}: {x[1]:8.1f} {x[2]:6.1f} {x[3]:.3f} {x[4]} {x[5]}")
