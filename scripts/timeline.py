#!/usr/bin/env python3
"""Kernel timeline of two pipelined frames from a rocprofv3 kernel trace: timeline.py <dir> [frame]."""
import csv, glob, sys
f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True))[0]
rows = list(csv.DictReader(open(f)))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("fr::", "")[:26])
            for r in rows)
sp = [k for k in ks if k[2].startswith("k_shade_paths")]
i = int(sys.argv[2]) if len(sys.argv) > 2 else 6
t0, t1 = sp[i][0], sp[i + 1][0]
print(f"frame {i}: {(t1 - t0) / 1e3:.1f} us between megakernel starts; megakernel {(sp[i][1] - sp[i][0]) / 1e3:.1f} us")
for s, e, n in ks:
    if t0 <= s < t1:
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {n}")
