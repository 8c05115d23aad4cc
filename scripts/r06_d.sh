#!/bin/bash
set -o pipefail
bash scripts/ab_lib_stage.sh r06d 3 new:- sold:abv/lib_sold.so sx0l0:abv/lib_sx0l0.so sx0l1:abv/lib_sx0l1.so snolds:abv/lib_snolds.so || exit 1
bash scripts/ab_bench.sh r06e 3 base:- cu32:FOVRT_RECON_CUS=32 cu64:FOVRT_RECON_CUS=64 cu32d:"FOVRT_RECON_CUS=32 FOVRT_CU_DISJOINT=1" cu128:FOVRT_RECON_CUS=128 || exit 2
