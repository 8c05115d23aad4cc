#!/usr/bin/env python3
"""Per-launch Sibson kernel durations (ms) from a rocprofv3 results database, in dispatch order:
python scripts/sibson_kstats.py gpurun_out/<dir>/<name>_results.db"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end from kernels where name like '%sibson%' order by start").fetchall()
for n, s, e in rows:
    print(n.split("(")[0].split("::")[-1], round((e - s) / 1e6, 3))
