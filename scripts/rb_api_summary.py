"""Long HIP API calls in a rocprofv3 --hip-runtime-trace --kernel-trace CSV run (scripts/r05_d.sh), each
with the calls and kernels just before it.  Usage: rb_api_summary.py <rocprofv3 output dir> [min_ms]"""
import csv
import glob
import os
import sys

root = sys.argv[1]
min_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0


def rows(pattern):
    out = []
    for p in glob.glob(os.path.join(root, "**", pattern), recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


api = rows("*hip_api_trace.csv")
ker = rows("*kernel_trace.csv")
print("api rows", len(api), "kernel rows", len(ker))
ev = []
for r in api:
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "api", r["Function"], r.get("Thread_Id", "")))
for r in ker:
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "kernel", r["Kernel_Name"][:60], ""))
ev.sort()
t0 = ev[0][0] if ev else 0
for i, (s, e, kind, name, tid) in enumerate(ev):
    if kind == "api" and (e - s) / 1e6 >= min_ms:
        print("== %s %.3f ms at %.3f ms (thread %s)" % (name, (e - s) / 1e6, (s - t0) / 1e6, tid))
        for s2, e2, k2, n2, t2 in ev[max(0, i - 8):i]:
            print("   before: %-6s %-50s %.3f ms at %.3f" % (k2, n2, (e2 - s2) / 1e6, (s2 - t0) / 1e6))
        for s2, e2, k2, n2, t2 in ev[i + 1:i + 4]:
            print("   after:  %-6s %-50s %.3f ms at %.3f" % (k2, n2, (e2 - s2) / 1e6, (s2 - t0) / 1e6))
