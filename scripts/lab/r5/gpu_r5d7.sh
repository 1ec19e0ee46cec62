#!/bin/bash
# two-workgroups-per-CU 128x256 x6 tiles (K3M_X6_VARIANT 1/2) vs the ping-pong walk on the forward shapes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in 0 1 2; do
    echo "== K3M_X6_VARIANT=$v round $r" >> gpurun_out/r5d7_ab.txt
    K3M_X6_VARIANT=$v timeout -k 10 200 python -u scripts/gemm_bench.py fwd 20 fp32 >> gpurun_out/r5d7_ab.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/r5d7_ab.txt
