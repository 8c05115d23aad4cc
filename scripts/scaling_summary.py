#!/usr/bin/env python3
"""Megakernel ms, segments per frame and fps of scripts/scaling_probe.sh runs."""
import glob, json
for f in sorted(glob.glob("gpurun_out/sp_*.log")):
    ls = [l for l in open(f) if l.startswith("{")]
    if not ls:
        continue
    d = json.loads(ls[-1])
    r = d["rays"]
    segs = sum(v for k, v in r.items() if k not in ("gbuffer_primary", "truncated", "overflow")) / d["steps"]
    print(f"{f[14:-4]:24s} mk {d['roofline']['megakernel_ms_serialised']:.3f} ms serialised, {segs / 1e6:6.2f} M seg/frame,"
          f" {segs / d['roofline']['megakernel_ms_serialised'] / 1e6:5.2f} Gseg/s  fps {d['fps']:.1f}")
