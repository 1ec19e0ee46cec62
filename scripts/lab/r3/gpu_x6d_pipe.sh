#!/bin/bash
# x6d lab: fragment reads of kt+1 under the MFMAs of kt (K3M_X6D_VARIANT=2) vs variant 0 and the x6 kernel,
# plus the PMC passes of variant 2 on the FFN1 forward
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  K3M_X6D_VARIANT=0 timeout -k 10 200 python -u scripts/x6d_bench.py 10 fwd > gpurun_out/x6dp_v0_$r.txt 2>&1
  K3M_X6D_VARIANT=2 timeout -k 10 200 python -u scripts/x6d_bench.py 10 fwd > gpurun_out/x6dp_v2_$r.txt 2>&1
done
K3M_X6D_VARIANT=2 bash scripts/pmc_x6d.sh x6dp "fwd ffn1 plain" x6d > gpurun_out/pmc_x6dp.log 2>&1
