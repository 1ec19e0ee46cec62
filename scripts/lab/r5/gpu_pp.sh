#!/bin/bash
# round 5 (resumed): ping-pong x6 main loop — correctness, then per-shape A/B against the compiler-scheduled loop
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_gemm_x6.py -k "persistent_walk" > gpurun_out/pp_test.log 2>&1 || { tail -30 gpurun_out/pp_test.log; exit 1; }
tail -3 gpurun_out/pp_test.log
for r in 1 2; do
  for v in 0 31; do
    echo "== K3M_X6_PP=$v round $r" >> gpurun_out/pp_ab.txt
    K3M_X6_PP=$v timeout -k 10 300 python -u scripts/gemm_bench.py all 20 fp32 >> gpurun_out/pp_ab.txt 2>&1 || exit 1
  done
done
cat gpurun_out/pp_ab.txt | grep -v amdgpu.ids
