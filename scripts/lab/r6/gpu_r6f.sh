#!/bin/bash
# flash-long forward / backward bit identity (fwd and bwd separately), then config-5 attention timings
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_gemm_bf16.py -k "flash_long_bwd_dma" > gpurun_out/r6f_test.log 2>&1
rc=$?
grep -E "AssertionError|passed|failed" gpurun_out/r6f_test.log | cut -c1-3000
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2; do
  for b in 1 2; do
    echo "== K3M_FLASH_LONG_FWD,BWD=$b round $r"
    K3M_FLASH_LONG_BWD=$b K3M_FLASH_LONG_FWD=$b timeout -k 10 120 python scripts/attn_bench.py bf16 cfg5 2>/dev/null | grep flash || exit 1
  done
done
