#!/bin/bash
# pair-draw attention dropout: regenerate the flash-long fixture, attention + train-mode parity tests, timings
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python tests/golden/make_flash_long_golden.py && cp tests/golden/flash_long_d96.npz gpurun_out/ || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_gemm_bf16.py tests/test_gpu_attention_long.py tests/test_gpu_train_mode_parity.py tests/test_gpu_kernels.py > gpurun_out/r6i_test.log 2>&1
rc=$?
grep -E "Error|passed|failed" gpurun_out/r6i_test.log | cut -c1-2000
[ $rc -eq 0 ] || exit $rc
for pp in 0.1 0; do
  echo "== ATTN_P=$pp cfg5 bf16"
  ATTN_P=$pp timeout -k 10 120 python scripts/attn_bench.py bf16 cfg5 2>/dev/null | grep flash || exit 1
  echo "== ATTN_P=$pp bs64 both"
  ATTN_P=$pp timeout -k 10 120 python scripts/attn_bench.py both 2>/dev/null || exit 1
done
for t in 5 4 0; do
  echo "== K3M_FLASH_LONG_TPG=$t"
  K3M_FLASH_LONG_TPG=$t timeout -k 10 120 python scripts/attn_bench.py bf16 cfg5 2>/dev/null | grep flash || exit 1
done
