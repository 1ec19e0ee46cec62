#!/bin/bash
# flash-long forward: XCD-aware query-block mapping (K3M_FLASH_LONG_XCD), parity tests then same-box A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out/r6v
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm_bf16.py tests/test_gpu_train_mode_parity.py tests/test_gpu_configs.py -k "long or flash or attn or train or cfg5" > gpurun_out/r6v/tests.txt 2>&1 || { tail -30 gpurun_out/r6v/tests.txt; exit 1; }
tail -2 gpurun_out/r6v/tests.txt
for r in 1 2; do
  for x in 1 0; do
    K3M_FLASH_LONG_XCD=$x timeout -k 10 200 python scripts/attn_bench.py bf16 cfg5 > gpurun_out/r6v/attn_xcd${x}_$r.txt 2>&1 || exit 1
    echo "== xcd=$x round $r"; grep "flash" gpurun_out/r6v/attn_xcd${x}_$r.txt | head -5
  done
done
bash scripts/ab_env_bench.sh 5 K3M_FLASH_LONG_XCD "1 0" 2 r6v || exit 1
