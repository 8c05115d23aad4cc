#!/usr/bin/env python3
"""Condenses the two SQ counter passes of scripts/pmc_sq.sh (gpurun_out/pmc_sq1, pmc_sq2) into
profiles/<tag>_pmc_issue.json: per kernel and dispatch, what bounds it at the SIMD.

The SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* counters count quad-cycles per wave (MI355X_MICROARCH.md,
per-instruction constants). A wave64 VALU instruction occupies its SIMD for one quad-cycle, and a SIMD issues one
VALU instruction per quad-cycle, so for a kernel whose waves stay resident for the whole launch (the persistent
megakernel: SQ_WAVES = resident waves) the SIMD's VALU busy fraction is
  valu_busy_per_simd = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES x (SQ_WAVES / SIMDs).
bench.py attaches the dominant kernel's entry to its roofline object as `issue` when the workload matches.
Usage: python scripts/pmc_issue.py <gpurun_out dir> <tag> [simds]"""
import csv
import glob
import json
import os
import sys


def short(name):
    return name.split("(")[0].replace("void ", "").replace("fr::", "").split("<")[0]


def per_kernel(path):
    acc, disp = {}, {}
    with open(path) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            acc.setdefault(k, {}).setdefault(r["Counter_Name"], 0.0)
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp.setdefault(k, set()).add(r["Dispatch_Id"])
    return {k: {c: v / len(disp[k]) for c, v in d.items()} for k, d in acc.items()}


def main():
    out, tag = sys.argv[1], sys.argv[2]
    simds = int(sys.argv[3]) if len(sys.argv) > 3 else 1024  # 256 CUs x 4 SIMDs
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    a = per_kernel(glob.glob(os.path.join(out, "pmc_sq1", "**", "*counter_collection.csv"), recursive=True)[0])
    b = per_kernel(glob.glob(os.path.join(out, "pmc_sq2", "**", "*counter_collection.csv"), recursive=True)[0])
    bench = {}
    try:
        with open(os.path.join(out, "pmc_sq1", "bench.json")) as f:
            bench = json.loads([l for l in f if l.startswith("{")][-1])
    except (OSError, ValueError, IndexError):
        pass
    kernels = {}
    for k in sorted(set(a) & set(b)):
        x, y = a[k], b[k]
        wc, waves = x.get("SQ_WAVE_CYCLES", 0.0), y.get("SQ_WAVES", 0.0)
        if not wc or not waves:
            continue
        ent = {"sq_waves": waves, "waves_per_simd": round(waves / simds, 2),
               "valu_issue_per_wave": round(x["SQ_ACTIVE_INST_VALU"] / wc, 4),
               "wait_any_per_wave": round(x["SQ_WAIT_ANY"] / wc, 4),
               "wait_inst_any_per_wave": round(x["SQ_WAIT_INST_ANY"] / wc, 4),
               "valu_insts": x["SQ_INSTS_VALU"], "vmem_rd_insts": x["SQ_INSTS_VMEM_RD"], "salu_insts": x["SQ_INSTS_SALU"]}
        # (only where every wave of the launch can be resident at once: at most 8 per SIMD)
        ent["valu_busy_per_simd"] = round(ent["valu_issue_per_wave"] * waves / simds, 3) if waves <= 8 * simds else None
        hit, miss = y.get("TCC_HIT_sum", 0.0), y.get("TCC_MISS_sum", 0.0)
        if hit + miss:
            ent["l2_hit"] = round(hit / (hit + miss), 3)
        if x["SQ_INSTS_VMEM_RD"]:
            ent["l1_accesses_per_vmem_rd"] = round(y.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0.0) / x["SQ_INSTS_VMEM_RD"], 2)
        kernels[k] = ent
    doc = {"tag": tag, "config": bench.get("config"), "simds": simds,
           "note": "valu_busy_per_simd holds for kernels whose waves stay resident for the whole launch "
                   "(the persistent megakernel); SQ_* wave counters in quad-cycles", "kernels": kernels}
    with open(os.path.join(root, "profiles", f"{tag}_pmc_issue.json"), "w") as f:
        json.dump(doc, f, indent=1)
    for k in ("k_shade_paths",):
        if k in kernels:
            print(k, kernels[k])


if __name__ == "__main__":
    main()
