#!/bin/bash
# VGPR / SGPR / scratch / LDS of the gfx950 kernels of one source (a device-only compile; no GPU needed):
#   scripts/kernel_regs.sh [csrc/k_trace.hip] [kernel-name regex] [extra hipcc flags]
SRC=${1:-foveated-rendering-using-ray-tracing_amd/csrc/k_trace.hip}
RE=${2:-.}
[ $# -ge 2 ] && shift 2 || set --
T=$(mktemp -d)
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 --cuda-device-only --no-gpu-bundle-output -w "$@" -o "$T/co" "$SRC" || exit 1
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$T/co" > "$T/notes.txt"
python3 - "$RE" "$T/notes.txt" <<'PY'
import re, sys
txt = open(sys.argv[2]).read()
rx = re.compile(sys.argv[1])
for blk in txt.split("- .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if not rx.search(name):
        continue
    def g(k):
        m = re.search(r"\." + k + r":\s+(\d+)", blk)
        return m.group(1) if m else "?"
    print("%-64s vgpr %4s sgpr %4s scratch %5s lds %6s vspill %s" % (name[:64], g("vgpr_count"), g("sgpr_count"),
          g("private_segment_fixed_size"), g("group_segment_fixed_size"), g("vgpr_spill_count")))
PY
rm -rf "$T"
