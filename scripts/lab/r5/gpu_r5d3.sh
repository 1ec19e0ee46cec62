#!/bin/bash
# wgrad tile choice under the ping-pong loop, then a HEAD profile of config 2 and a bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in "15 31" "11 31" "15 63"; do
    set -- $v
    echo "== K3M_X6_TILE256=$1 K3M_X6_PP=$2 round $r" >> gpurun_out/r5d3_wgrad.txt
    K3M_X6_TILE256=$1 K3M_X6_PP=$2 timeout -k 10 200 python -u scripts/gemm_bench.py wgrad 20 fp32 >> gpurun_out/r5d3_wgrad.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/r5d3_wgrad.txt
bash scripts/prof_cfg.sh 2 r5d_cfg2 2 || exit 1
head -25 gpurun_out/prof_r5d_cfg2/step_split.txt
head -3 gpurun_out/prof_r5d_cfg2/gemm_calls.txt
timeout -k 10 600 python bench.py --steps 20 --warmup 8 > gpurun_out/r5d_bench_cfg2.json 2> gpurun_out/r5d_bench_cfg2.err || exit 1
tail -1 gpurun_out/r5d_bench_cfg2.json
