#!/bin/bash
# A/B of lab x6 tile variants (K3M_X6_VARIANT, gemm_x6p.hip) on the forward shapes and the fp32 bench.
# usage: scripts/ab_variant.sh "0 3 4" [bench]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VS=${1:-"0 1 2"}
for r in 1 2; do
  for v in $VS; do
    echo "== variant $v"
    K3M_X6_VARIANT=$v timeout -k 10 300 python scripts/gemm_bench.py fwd 10 fp32 || exit $?
  done
done
if [ "${2:-}" = "bench" ]; then
  for v in $VS; do
    echo "== bench variant $v"
    K3M_X6_VARIANT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 4 --no-cpu-baseline | cut -c1-300 || exit $?
  done
fi
