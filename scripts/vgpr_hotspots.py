"""Where a kernel's high-numbered VGPRs are used: a register-pressure map from the device assembly.
   hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S -gline-tables-only ... -o k.s k.hip
   python scripts/vgpr_hotspots.py k.s <kernel-name-substring> [threshold]
Counts, per source line (.loc), the instructions touching VGPRs numbered >= threshold (default 150): the
allocator only reaches those registers where the live set is that large."""
import collections
import re
import sys

path, kname = sys.argv[1], sys.argv[2]
thr = int(sys.argv[3]) if len(sys.argv) > 3 else 150
lines = open(path).read().split('\n')
start = next(i for i, l in enumerate(lines) if re.match(r'^_Z\S*' + re.escape(kname) + r'\S*:', l))
end = next(i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end'))
files = {}
for l in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]+)")?', l)
    if m:
        files[m.group(1)] = (m.group(3) or m.group(2)).split('/')[-1]
cur = None
hist = collections.Counter()
maxreg = collections.defaultdict(int)
for l in lines[start:end]:
    m = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)', l)
    if m:
        cur = (files.get(m.group(1), m.group(1)), int(m.group(2)))
        continue
    regs = [int(x) for x in re.findall(r'\bv(\d+)\b', l)] + [int(b) for a, b in re.findall(r'\bv\[(\d+):(\d+)\]', l)]
    if regs and max(regs) >= thr:
        hist[cur] += 1
        maxreg[cur] = max(maxreg[cur], max(regs))
for k, v in hist.most_common(50):
    print(v, maxreg[k], k)
