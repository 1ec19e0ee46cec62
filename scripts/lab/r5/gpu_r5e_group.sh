#!/bin/bash
# lab: persistent-walk tile order (row-tiles per N walk 8 = HEAD vs 4 / 16), config 2 interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm_x6.py \
  -k "persistent_walk or splitk or beta" > gpurun_out/r5e_group_test.log 2>&1 || { tail -30 gpurun_out/r5e_group_test.log; exit 1; }
tail -1 gpurun_out/r5e_group_test.log
for r in 1 2 3; do
  for lib in k3m_amd/libk3m_hip.so ab/g4.so ab/g16.so; do
    out=$(K3M_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 4 2>/dev/null | tail -n 1) || exit 1
    echo "$lib $(echo "$out" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["gemm_all"]["ms_per_step"])')"
  done
done
