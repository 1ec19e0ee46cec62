#!/bin/bash
# x6d lab, timing only: variant 3 skips the B operand's LDS-DMA after the prologue (half the DMA issues per
# k-tile; C is wrong) -- does the DMA issue cost bound the main loop?
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  K3M_X6D_VARIANT=0 timeout -k 10 200 python -u scripts/x6d_bench.py 10 "fwd ffn" x6d > gpurun_out/x6dnb_v0_$r.txt 2>&1
  K3M_X6D_VARIANT=3 timeout -k 10 200 python -u scripts/x6d_bench.py 10 "fwd ffn" x6d > gpurun_out/x6dnb_v3_$r.txt 2>&1
done
K3M_X6D_VARIANT=3 bash scripts/pmc_x6d.sh x6dnb "fwd ffn1 plain" x6d > gpurun_out/pmc_x6dnb.log 2>&1
