#!/usr/bin/env python3
"""Per-kernel counter means from rocprofv3 --pmc CSV directories: pmc_summary.py <kernel substring> <dir>..."""
import csv
import glob
import sys
from collections import defaultdict


def main():
    kern = sys.argv[1]
    for d in sys.argv[2:]:
        vals = defaultdict(list)
        for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    if kern in row["Kernel_Name"]:
                        vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
        print(d, {k: round(sum(v) / len(v), 1) for k, v in sorted(vals.items())})


if __name__ == "__main__":
    main()
