#!/bin/bash
# Whole-step A/B of the LayerNorm changes (half-wave bf16 kernels on long LayerNorms, 8 rows per backward
# slab): interleaved bench runs, base = K3M_LN_BF16_VEC=0 K3M_LN_ROWS_PER_SLAB=4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {   # label, env..., -- bench args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  out=$(env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline "$@" 2>/dev/null | tail -n 1) || { echo "$label failed"; exit 1; }
  echo "$label $(echo "$out" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
}
echo "## config 3 (bf16)"
for r in 1 2 3; do
  run base K3M_LN_BF16_VEC=0 K3M_LN_ROWS_PER_SLAB=4 -- --config 3 --steps 20
  run new K3M_LN_BF16_VEC=1 K3M_LN_ROWS_PER_SLAB=8 -- --config 3 --steps 20
done
echo "## config 2 (fp32)"
for r in 1 2; do
  run base K3M_LN_BF16_VEC=0 K3M_LN_ROWS_PER_SLAB=4 -- --config 2 --steps 12
  run new K3M_LN_BF16_VEC=1 K3M_LN_ROWS_PER_SLAB=8 -- --config 2 --steps 12
done
