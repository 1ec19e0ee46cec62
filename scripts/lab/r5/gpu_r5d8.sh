#!/bin/bash
# input-gradient walk with the FAST epilogue (K3M_X6_PP bit 128): bit identity, then A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
K3M_X6_PP=159 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_gemm_x6.py -k "dgelu or epilogues or beta or accuracy" > gpurun_out/r5d8_test.log 2>&1 || { tail -30 gpurun_out/r5d8_test.log; exit 1; }
tail -2 gpurun_out/r5d8_test.log
for r in 1 2; do
  for v in 31 159; do
    echo "== K3M_X6_PP=$v round $r" >> gpurun_out/r5d8_ab.txt
    K3M_X6_PP=$v timeout -k 10 200 python -u scripts/gemm_bench.py dgrad 20 fp32 >> gpurun_out/r5d8_ab.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/r5d8_ab.txt
