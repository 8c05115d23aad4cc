"""Markdown rows of DESIGN.md §5 (pipeline modes) and BASELINE.md §6 from a configs jsonl (scripts/configs_bench.sh
lines, condensed by scripts/configs_summary.py). Usage: python scripts/config_tables.py <configs.jsonl>"""
import json
import subprocess
import sys

names = {"C1": "C1", "C2": "C2", "C3": "C3", "C3gaze": "C3, eye-tracked circle", "C3sacc": "C3, saccades",
         "C4": "C4 (1 view)", "C5": "C5 (1 eye)"}
bnames = dict(names, C4="C4 (one GPU's share)", C5="C5 (one eye)")
out = subprocess.run([sys.executable, "scripts/configs_summary.py", sys.argv[1]], capture_output=True, text=True,
                     check=True).stdout
rows = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
print("DESIGN §5")
for j in rows:
    lm = j["pipeline_latency_mode"]
    fc, lf, fs = j["frame_clock_pipelined"]["latency_ms"], lm["frame_clock"]["latency_ms"], j["frame_ms_serial"]
    print(f"| {names[j['config']]} | {j['fps']:,.0f} | {fc['p50']:.1f} / {fc['p99']:.1f} | {1000 / fs['p50']:,.0f} / "
          f"{j['fps_serial_mean']:,.0f} | {lm['fps']:,.0f} | {lf['p50']:.2f} / {lf['p99']:.2f} |")
print("BASELINE §6")
for j in rows:
    lm = j["pipeline_latency_mode"]
    fc, lf, fs = j["frame_clock_pipelined"]["latency_ms"], lm["frame_clock"]["latency_ms"], j["frame_ms_serial"]
    cpu = j.get("cpu_baseline", {}).get("fps")
    cpu_s = f"{cpu:.3g}" if cpu else ("(§4)" if j["config"] == "C3" else "—")
    print(f"| {bnames[j['config']]} | {j['Mrays_s']:,.0f} | {j['fps']:,.1f} / {lm['fps']:,.1f} / {j['fps_serial_mean']:,.1f} | "
          f"{fc['p50']:.3g} / {fc['p99']:.3g} | {lf['p50']:.3g} / {lf['p99']:.3g} | {fs['p50']:.3g} / {fs['p99']:.3g} | {cpu_s} |")
