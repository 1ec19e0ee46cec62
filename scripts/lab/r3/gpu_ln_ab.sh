#!/bin/bash
# bf16 LayerNorm A/B: one-wave-per-row kernels (K3M_LN_BF16_VEC=0) vs half-wave 16-B kernels, and rows per
# backward slab (K3M_LN_ROWS_PER_SLAB); timing of scripts/ln_bench.py per setting.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/ln_ab.txt
for vec in 0 1; do
  for rps in 4 8 16 32; do
    echo "--- K3M_LN_BF16_VEC=$vec K3M_LN_ROWS_PER_SLAB=$rps" >> gpurun_out/ln_ab.txt
    K3M_LN_BF16_VEC=$vec K3M_LN_ROWS_PER_SLAB=$rps timeout -k 10 120 python -u scripts/ln_bench.py >> gpurun_out/ln_ab.txt 2>&1
  done
done
