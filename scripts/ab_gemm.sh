#!/bin/bash
# Same-box A/B of two library builds on the GEMM microbenchmark: interleaved runs of scripts/gemm_bench.py.
# usage: scripts/ab_gemm.sh A.so B.so ROUNDS [filter] [reps] [dtype]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
a=$1; b=$2; rounds=$3; shift 3
for r in $(seq 1 "$rounds"); do
  for lib in "$a" "$b"; do
    echo "## $(basename "$lib") round $r"
    K3M_LIB="$lib" timeout -k 10 300 python scripts/gemm_bench.py "$@" || exit $?
  done
done
