#!/bin/bash
# lab A/B: issue-priority variants of the ping-pong phases (per-shape)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for lib in k3m_amd/libk3m_hip.so ab/prio.so ab/priolate.so; do
    echo "== $lib round $r" >> gpurun_out/r5e_prio.txt
    K3M_LIB=$lib timeout -k 10 200 python -u scripts/gemm_bench.py all 20 fp32 >> gpurun_out/r5e_prio.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/r5e_prio.txt | grep -E "==|fwd|dgrad|wgrad ffn|co pv"
