#!/usr/bin/env python3
"""Prints a rocprofv3 kernel_stats.csv (name, calls, average us, total ms) sorted by total time."""
import csv, glob, sys
f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True))[0]
rows = list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{r['Name'].split('(')[0].replace('fr::', '')[:40]:40s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f} us {float(r['TotalDurationNs'])/1e6:9.2f} ms")
