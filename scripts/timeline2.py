#!/usr/bin/env python3
"""Kernel timeline with queue ids over a window: tl2.py <dir> <frame> <nframes>"""
import csv, glob, sys
f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True))[0]
rows = list(csv.DictReader(open(f)))
qk = [k for k in rows[0].keys() if "Queue" in k or "Stream" in k]
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("fr::", "").replace("void ","")[:22], "/".join(r[k] for k in qk)) for r in rows)
sp = [k for k in ks if k[2].startswith("k_shade_paths")]
i = int(sys.argv[2]); n = int(sys.argv[3])
t0, t1 = sp[i][0], sp[i + n][0]
print("cols", qk, f"{n} frames {(t1-t0)/1e3/n:.1f} us/frame")
for s, e, nm, q in ks:
    if t0 - 300000 <= s < t1:
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {q:8s} {nm}")
