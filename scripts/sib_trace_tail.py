"""Per-kernel Sibson times of the last Sibson passes in a rocprofv3 kernel trace (the probe's alone runs at its
last gaze). Usage: python scripts/sib_trace_tail.py <kernel_trace.csv> [passes]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
sib = [r for r in rows if "sibson" in r["Kernel_Name"] or "jfa_final" in r["Kernel_Name"]]
runs = [i for i, r in enumerate(sib) if "k_sibson_runs" in r["Kernel_Name"]]
acc = collections.defaultdict(list)
for a, b in zip(runs[-n:], runs[-n + 1:] + [len(sib)]):
    per = collections.defaultdict(float)
    for r in sib[a:b]:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        per[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    for k, v in per.items():
        acc[k].append(v)
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:40s} median {sorted(v)[len(v) // 2]:8.1f} us over {len(v)}")
