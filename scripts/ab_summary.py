#!/usr/bin/env python3
"""Prints value / fps / stage ms of the bench logs an A/B or sweep run left under gpurun_out/."""
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab_*.log")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(f, "unreadable", e)
        continue
    st = " ".join(f"{k}={v['ms']:.3f}" for k, v in d["stages"].items())
    print(f"{f:40s} {d['value']:8.1f} Mrays/s {d['fps']:7.2f} fps mk={d['roofline'].get('megakernel_ms', 0):.3f} {st}")
