#!/bin/bash
# lab: persistent-walk tile order (row-tiles per N walk 8 = HEAD vs 4 / 16), config 2 interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for lib in k3m_amd/libk3m_hip.so ab/g4.so ab/g16.so; do
    out=$(K3M_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 4 2>/dev/null | tail -n 1) || exit 1
    echo "$lib $(echo "$out" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["gemm_all"]["ms_per_step"])')"
  done
done
