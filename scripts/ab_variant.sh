#!/bin/bash
# A/B of lab x6 tile variants (K3M_X6_VARIANT, gemm_x6p.hip) on the forward shapes and the fp32 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in 0 1 2 0 1 2; do
  echo "== variant $v"
  K3M_X6_VARIANT=$v timeout -k 10 300 python scripts/gemm_bench.py fwd 10 fp32 || exit $?
done
for v in 0 1 2; do
  echo "== bench variant $v"
  K3M_X6_VARIANT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 4 --no-cpu-baseline || exit $?
done
