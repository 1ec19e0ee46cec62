#!/bin/bash
# Interleaved A/B of the persistent x6 walk: gemm_bench on the text-layer shapes and the fp32 bench,
# K3M_X6_PERSIST=0 vs 1, two rounds each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for p in 0 1; do
    echo "== round $r persist=$p"
    K3M_X6_PERSIST=$p timeout -k 10 300 python scripts/gemm_bench.py all 10 fp32 || exit $?
  done
done
for r in 1 2; do
  for p in 0 1; do
    echo "== bench round $r persist=$p"
    K3M_X6_PERSIST=$p timeout -k 10 300 python bench.py --steps 10 --warmup 4 --no-cpu-baseline || exit $?
  done
done
