#!/bin/bash
# bf16 grouped-walk tile model (K3M_B16_TILE_MODEL): GEMM / co-attention tests, then same-box A/B on configs 3 and 5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out/r6s
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm_bf16.py tests/test_gpu_gemm_b16_dual.py tests/test_gpu_configs.py > gpurun_out/r6s/tests.txt 2>&1
rc=$?; tail -1 gpurun_out/r6s/tests.txt; [ $rc -eq 0 ] || { grep -E "Error|FAILED" gpurun_out/r6s/tests.txt | head; exit $rc; }
bash scripts/ab_env_bench.sh 3 K3M_B16_TILE_MODEL "1 0" 2 r6s && bash scripts/ab_env_bench.sh 5 K3M_B16_TILE_MODEL "1 0" 2 r6s
