#!/bin/bash
# lab: input-gradient walk on PPDLoop with the branch-free interior epilogue (dGELU shapes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
K3M_LIB=ab/ppdfast.so K3M_X6_PP=127 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_gemm_x6.py -k "dgelu or epilogues or beta or accuracy" > gpurun_out/r5e_ppdfast_test.log 2>&1 || { tail -30 gpurun_out/r5e_ppdfast_test.log; exit 1; }
tail -1 gpurun_out/r5e_ppdfast_test.log
for r in 1 2; do
  for cfg in "k3m_amd/libk3m_hip.so 63" "k3m_amd/libk3m_hip.so 127" "ab/ppdfast.so 127"; do
    set -- $cfg
    echo "== $1 K3M_X6_PP=$2 round $r" >> gpurun_out/r5e_ppdfast.txt
    K3M_LIB=$1 K3M_X6_PP=$2 timeout -k 10 200 python -u scripts/gemm_bench.py dgrad 20 fp32 >> gpurun_out/r5e_ppdfast.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/r5e_ppdfast.txt | grep -E "==|dgrad"
