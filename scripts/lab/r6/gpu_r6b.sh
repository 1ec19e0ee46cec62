#!/bin/bash
# epilogue-wave bf16 GEMM: bit-identity test, then the nt shapes with K3M_B16_WS 0 vs 3 (interleaved)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_gemm_b16_ws.py > gpurun_out/r6b_test.log 2>&1 || { tail -40 gpurun_out/r6b_test.log; exit 1; }
tail -4 gpurun_out/r6b_test.log
for r in 1 2; do
  for ws in 0 3; do
    echo "== K3M_B16_WS=$ws round $r"
    K3M_B16_WS=$ws timeout -k 10 120 python scripts/gemm_bench.py fwd 20 bf16 2>/dev/null || exit 1
    K3M_B16_WS=$ws timeout -k 10 120 python scripts/gemm_bench.py "co " 20 bf16 2>/dev/null | grep -E "co img|co pv|co txt ffn2" || exit 1
    K3M_B16_WS=$ws timeout -k 10 120 python scripts/gemm_bench.py "img fwd" 20 bf16 2>/dev/null || exit 1
  done
done
