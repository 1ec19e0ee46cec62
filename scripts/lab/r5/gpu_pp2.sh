#!/bin/bash
# ping-pong main loops: kernel tests, then same-box A/B of the fp32 (config 2) and bf16 (config 3) steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_gemm_x6.py tests/test_gpu_gemm_bf16.py -k "not attention and not layernorm" > gpurun_out/pp2_test.log 2>&1 \
  || { tail -40 gpurun_out/pp2_test.log; exit 1; }
tail -3 gpurun_out/pp2_test.log
bash scripts/ab_env.sh K3M_X6_PP "0 31" 2 --steps 10 --warmup 4 > gpurun_out/pp2_ab_cfg2.txt 2>&1 || { cat gpurun_out/pp2_ab_cfg2.txt; exit 1; }
cat gpurun_out/pp2_ab_cfg2.txt
bash scripts/ab_env.sh K3M_B16_PP "0 3" 2 --steps 10 --warmup 4 --config 3 --dtype bf16 > gpurun_out/pp2_ab_cfg3.txt 2>&1 || { cat gpurun_out/pp2_ab_cfg3.txt; exit 1; }
cat gpurun_out/pp2_ab_cfg3.txt
for v in 0 7 0 7; do
  echo "== K3M_B16_PP=$v" >> gpurun_out/pp2_b16_gemm.txt
  K3M_B16_PP=$v timeout -k 10 300 python -u scripts/gemm_bench.py all 20 bf16 >> gpurun_out/pp2_b16_gemm.txt 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/pp2_b16_gemm.txt | head -120
