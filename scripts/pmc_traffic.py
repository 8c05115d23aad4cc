#!/usr/bin/env python3
"""Condenses a scripts/profile.sh run into the files committed under profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of the bench command
  profiles/<tag>_pmc_traffic.json   per-kernel HBM bytes per dispatch from the FETCH_SIZE / WRITE_SIZE passes

FETCH_SIZE and WRITE_SIZE are in KiB. On gfx950 FETCH_SIZE counts half the bytes of wide (16 B/lane)
streaming reads (MI355X_MICROARCH.md, HBM section): the corrected read figure doubles it; the raw
value is kept beside it. bench.py takes `traffic` for its roofline kernel from this file when the
workload matches.
"""
import csv
import glob
import json
import os
import shutil
import sys


def find(d, pattern):
    hits = sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))
    if not hits:
        raise SystemExit(f"no {pattern} under {d}")
    return hits[0]


def short(name):
    return name.split("(")[0].replace("fr::", "")


def counters(path, counter):
    per_dispatch = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            key = (row["Dispatch_Id"], short(row["Kernel_Name"]))
            per_dispatch[key] = per_dispatch.get(key, 0.0) + float(row["Counter_Value"])
    out = {}
    for (_, k), v in per_dispatch.items():
        s = out.setdefault(k, [0.0, 0])
        s[0] += v
        s[1] += 1
    return {k: (s[0] / s[1], s[1]) for k, s in out.items()}


def main():
    out_dir, tag = sys.argv[1], sys.argv[2]
    bench_args = sys.argv[3:]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    stats = find(os.path.join(out_dir, "trace"), "*kernel_stats.csv")
    shutil.copyfile(stats, os.path.join(root, "profiles", f"{tag}_kernel_stats.csv"))
    durations = {}
    with open(stats) as f:
        for row in csv.DictReader(f):
            durations[short(row["Name"])] = float(row["AverageNs"])
    fetch = counters(find(os.path.join(out_dir, "fetch"), "*counter_collection.csv"), "FETCH_SIZE")
    write = counters(find(os.path.join(out_dir, "write"), "*counter_collection.csv"), "WRITE_SIZE")
    bench = {}
    try:
        with open(os.path.join(out_dir, "bench_trace.json")) as f:
            bench = json.loads(f.read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError):
        pass
    # the roofline stage's kernels over the timed region only: bench.py runs `warmup` pipelined frames,
    # `steps` timed pipelined frames, then serialised stage frames; one k_shade_paths per frame
    timed = {}
    try:
        trace = find(os.path.join(out_dir, "trace"), "*kernel_trace.csv")
        steps, warmup = bench.get("steps", 20), bench.get("warmup", 5)
        per = {}
        with open(trace) as f:
            for row in csv.DictReader(f):
                per.setdefault(short(row["Kernel_Name"]), []).append(
                    (int(row["Start_Timestamp"]), int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
        for k in ("k_shade_paths", "k_shade_resolve", "k_carry_history"):
            d = [ns for _, ns in sorted(per.get(k, []))][warmup:warmup + steps]
            if d:
                timed[k] = {"dispatches": len(d), "avg_ns": sum(d) / len(d)}
    except SystemExit:
        pass
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        fr_kib, n = fetch.get(k, (0.0, 0))
        wr_kib, _ = write.get(k, (0.0, 0))
        rd = 2 * fr_kib * 1024
        wr = wr_kib * 1024
        ent = {"dispatches": n, "fetch_size_kib_raw": round(fr_kib, 1), "write_size_kib": round(wr_kib, 1),
               "hbm_read_bytes": rd, "hbm_write_bytes": wr, "hbm_bytes": rd + wr}
        if k in durations:
            ent["avg_ns"] = durations[k]
            ent["hbm_GBs"] = round((rd + wr) / durations[k], 1)
        kernels[k] = ent
    doc = {"tag": tag, "bench_args": bench_args, "config": bench.get("config"),
           "correction": "hbm_read_bytes = 2 x FETCH_SIZE (gfx950 half-count of wide streaming reads); "
                         "hbm_write_bytes = WRITE_SIZE; both per dispatch, averaged over the profiled dispatches",
           "kernels": kernels,
           "timed_region": timed,
           "timed_region_note": "kernel-trace durations of the roofline stage's kernels over the bench's timed "
                                "(pipelined) frames only; bench.py's live HIP-event average covers the same frames"}
    with open(os.path.join(root, "profiles", f"{tag}_pmc_traffic.json"), "w") as f:
        json.dump(doc, f, indent=1)
    for k, e in sorted(kernels.items(), key=lambda kv: -kv[1].get("avg_ns", 0)):
        print(f"{k:28s} {e.get('avg_ns', 0) / 1e3:10.1f} us  {e['hbm_bytes'] / 1e6:10.2f} MB  {e.get('hbm_GBs', 0):8.1f} GB/s")


if __name__ == "__main__":
    main()
