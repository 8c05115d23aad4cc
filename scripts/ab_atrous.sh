set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "atrous" 2>&1 | tail -3
for r in 1 2 3; do for e in 0 1; do
  FOVRT_ATROUS_ROWS2=$e FR_PASS_DUMP=/tmp/at_$e.npy timeout -k 10 120 python -u scripts/pass_probe.py atrous 50 | sed "s/^/rows2=$e /"
done; done
python - <<'PY'
import numpy as np
a=np.load("/tmp/at_0.npy")
for e in (1,):
    b=np.load(f"/tmp/at_{e}.npy")
    print(e, 'bit-identical' if np.array_equal(a.view(np.uint32), b.view(np.uint32)) else f'DIFF {np.count_nonzero(a.view(np.uint32)!=b.view(np.uint32))}')
PY
