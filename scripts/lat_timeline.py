"""Per-frame timeline of a kernel trace of fr_frame calls (rocprofv3 --kernel-trace csv): for each frame, in ms
from its G-buffer start: the G-buffer end, the megakernel start / end, JumpFlooding start, Sibson start / end and
the last A-Trous pass end. Usage: python scripts/lat_timeline.py <kernel_trace.csv>"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ev = [(r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fr::", ""), int(r["Start_Timestamp"]) / 1e6,
       int(r["End_Timestamp"]) / 1e6) for r in rows]
starts = [i for i, e in enumerate(ev) if e[0].startswith("k_gbuffer")]
print("frame  gbuf_end  mk_start  mk_end  jfa_start  sib_start  sib_end  atrous_end  | mk_ms sib_ms")
prev = None
for n, i in enumerate(starts):
    t0 = ev[i][1]
    j = starts[n + 1] if n + 1 < len(starts) else len(ev)
    # this frame's kernels: the megakernel after this G-buffer, then its reconstruction (the next kernels of each kind)
    def first(name, after):
        for e in ev[i:]:
            if e[0].startswith(name) and e[1] >= after:
                return e
        return None
    g = ev[i]
    mk = first("k_shade_paths", t0)
    if not mk:
        break
    jf = first("k_jfa_init", mk[2])
    sr = first("k_sibson_runs", jf[2] if jf else mk[2])
    # this frame's Sibson: its k_sibson_runs and the Sibson kernels after it, up to the next k_sibson_runs
    sib_end = float("nan")
    if sr:
        k = ev.index(sr)
        sib = [sr] + [e for e in ev[k + 1:] if e[0].startswith("k_sibson")]
        nxt = next((m for m, e in enumerate(sib[1:], 1) if e[0] == "k_sibson_runs"), len(sib))
        sib_end = max(e[2] for e in sib[:nxt])
    at = [e for e in ev if e[0].startswith("k_atrous") and e[1] >= mk[2]][:1]
    at_end = at[-1][2] if at else float("nan")
    rel = lambda x: x - t0
    print(f"{n:5d} {rel(g[2]):9.2f} {rel(mk[1]):9.2f} {rel(mk[2]):7.2f} {rel(jf[1]) if jf else float('nan'):10.2f} "
          f"{rel(sr[1]) if sr else float('nan'):10.2f} {rel(sib_end):8.2f} {rel(at_end):11.2f}  | {mk[2] - mk[1]:5.2f} "
          f"{sib_end - sr[1] if sr else float('nan'):6.2f}")
