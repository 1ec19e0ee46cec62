#!/bin/bash
# flash-long LDS-DMA backward: bit-identity vs the register form, the flash tests, then config-5 attention timings
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_gemm_bf16.py -k "flash" > gpurun_out/r6d_test.log 2>&1 || { tail -40 gpurun_out/r6d_test.log; exit 1; }
tail -3 gpurun_out/r6d_test.log
for r in 1 2; do
  for b in 1 2; do
    echo "== K3M_FLASH_LONG_FWD,BWD=$b round $r"
    K3M_FLASH_LONG_BWD=$b K3M_FLASH_LONG_FWD=$b timeout -k 10 120 python scripts/attn_bench.py bf16 cfg5 2>/dev/null | grep flash || exit 1
  done
done
