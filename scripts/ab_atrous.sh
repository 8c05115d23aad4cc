# A-Trous alone at 4K, interleaved A/B of env settings, with a bit-exact check of every variant's output
# against the first: scripts/ab_atrous.sh "name:VAR=val ..." ...  (3 rounds of 50 passes)
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "atrous" 2>&1 | tail -1
for r in 1 2 3; do for spec in "$@"; do
  n=${spec%%:*}; vars=${spec#*:}
  env $vars FR_PASS_DUMP=/tmp/at_$n.npy timeout -k 10 120 python -u scripts/pass_probe.py atrous 50 | sed "s/^/$n /"
done; done
python - "$@" <<'PY'
import sys, numpy as np
names = [s.split(":")[0] for s in sys.argv[1:]]
a = np.load(f"/tmp/at_{names[0]}.npy").view(np.uint32)
for n in names[1:]:
    b = np.load(f"/tmp/at_{n}.npy").view(np.uint32)
    print(n, "bit-identical to", names[0] if np.array_equal(a, b) else f"DIFFERS in {np.count_nonzero(a != b)} words")
PY
