#!/bin/bash
# LDS-DMA-staged ping-pong loop on the 256x256 forward / input-gradient walks: bit identity, then A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_gemm_x6.py -k "persistent_walk" > gpurun_out/r5d6_test.log 2>&1 || { tail -30 gpurun_out/r5d6_test.log; exit 1; }
tail -2 gpurun_out/r5d6_test.log
for r in 1 2; do
  for v in 31 95; do
    for sh in fwd dgrad; do
      echo "== K3M_X6_PP=$v round $r $sh" >> gpurun_out/r5d6_ab.txt
      K3M_X6_PP=$v timeout -k 10 200 python -u scripts/gemm_bench.py $sh 20 fp32 >> gpurun_out/r5d6_ab.txt 2>&1 || exit 1
    done
  done
done
grep -v amdgpu.ids gpurun_out/r5d6_ab.txt
