"""Per-launch averages of rocprofv3 --pmc counters for the kernels whose name contains a pattern.
Usage: python scripts/pmc_kernel_sum.py <counter_collection.csv> <pattern>..."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for pat in sys.argv[2:]:
    acc = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in rows:
        if pat in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r["Dispatch_Id"])
    print(pat, {c: f"{v / max(len(disp[c]), 1):.4g}" for c, v in sorted(acc.items())}, "launches", max((len(v) for v in disp.values()), default=0))
