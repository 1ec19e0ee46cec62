#!/bin/bash
# flash-long backward with two dS^T images (K3M_FLASH_LONG_DQ2): flash tests under both settings, then timings
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for d in 1 0; do
  K3M_FLASH_LONG_DQ2=$d timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_gemm_bf16.py -k "flash" > gpurun_out/r6l_test_$d.log 2>&1
  rc=$?
  echo "DQ2=$d: $(grep -E "passed|failed" gpurun_out/r6l_test_$d.log | tail -1)"
  [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r6l_test_$d.log | head -10; exit $rc; }
done
for r in 1 2; do
  for d in 1 0; do
    echo "== K3M_FLASH_LONG_DQ2=$d round $r"
    K3M_FLASH_LONG_DQ2=$d timeout -k 10 120 python scripts/attn_bench.py bf16 cfg5 2>/dev/null | grep flash || exit 1
  done
done
