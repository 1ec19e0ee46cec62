#!/bin/bash
# step A/B: ping-pong default (31) vs + LDS-DMA-staged weight-gradient walk (63); forward shapes on PPDLoop v2 (127)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/ab_env.sh K3M_X6_PP "31 63" 3 --steps 10 --warmup 4 > gpurun_out/r5d9_ab_cfg2.txt 2>&1 || { cat gpurun_out/r5d9_ab_cfg2.txt; exit 1; }
cat gpurun_out/r5d9_ab_cfg2.txt
for r in 1 2; do
  for v in 63 127; do
    for sh in fwd dgrad; do
      echo "== K3M_X6_PP=$v round $r $sh" >> gpurun_out/r5d9_ab_fwd.txt
      K3M_X6_PP=$v timeout -k 10 200 python -u scripts/gemm_bench.py $sh 20 fp32 >> gpurun_out/r5d9_ab_fwd.txt 2>&1 || exit 1
    done
  done
done
grep -v amdgpu.ids gpurun_out/r5d9_ab_fwd.txt | grep -E "==|ffn|qkv|out"
