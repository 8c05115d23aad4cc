#!/bin/bash
# k_sibson_strip ablation on the wide-hole mask (FOVRT_SIB_STRIP_VARIANT bits: 1 no row sums, 2 no run-end
# settling, 4 no block-total loads, 8 prefix loads at lane-contiguous columns, 16 every row sum from one row)
set -o pipefail
for v in 0 4 8 12 16 24; do
  echo "variant $v"; FOVRT_SIB_STRIP=1 FOVRT_SIB_STRIP_VARIANT=$v timeout -k 10 200 python scripts/sib_mask_probe.py 3 || exit 1
done
