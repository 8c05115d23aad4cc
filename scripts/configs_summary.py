#!/usr/bin/env python3
"""Condenses gpurun_out/cfg_C*.log (scripts/configs_bench.sh) into one JSON line per config."""
import glob, json, re, sys

out = []
for f in sorted(glob.glob("gpurun_out/cfg_C*.log")):
    name = re.search(r"cfg_(C\d\w*)\.log", f).group(1)
    lines = [l for l in open(f) if l.startswith("{")]
    if not lines:
        continue
    d = json.loads(lines[-1])
    c = d["config"]
    row = {"config": name, "scene": c["scene"], "width": c["width"], "height": c["height"], "spp": c["spp"],
           "diffuse_max_depth": c["diffuse_max_depth"], "mask_mode": c["mask_mode"],
           "foveal_density": c["foveal_density"], "Mrays_s": d["value"], "fps": d["fps"],
           "ms_per_step": d["ms_per_step"], "stages_ms": {k: v["ms"] for k, v in d["stages"].items()},
           "megakernel_ms": d["roofline"].get("megakernel_ms"), "gaze": c.get("gaze"),
           "frame_ms_serial": d.get("frame_ms_serial"), "fps_serial": d.get("fps_serial"),
           "frame_clock_pipelined": d.get("frame_clock_pipelined"), "steps": d.get("steps"),
           "fps_serial_mean": d.get("fps_serial_mean"), "pipeline_latency_mode": d.get("pipeline_latency_mode")}
    if "cpu_baseline" in d:
        row["cpu_baseline"] = {k: d["cpu_baseline"][k] for k in ("value", "unit", "cores", "kind", "fps")}
    out.append(row)
dst = sys.argv[1] if len(sys.argv) > 1 else None
text = "\n".join(json.dumps(r) for r in out) + "\n"
if dst:
    open(dst, "w").write(text)
print(text, end="")
