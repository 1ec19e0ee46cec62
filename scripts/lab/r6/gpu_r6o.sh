#!/bin/bash
# non-temporal epilogue stores in the bf16 persistent walk (K3M_B16_LAB bit 2): GEMM shapes, then config 3 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r6o
for r in 1 2; do
  for v in 0 4; do
    echo "== K3M_B16_LAB=$v round $r"
    K3M_B16_LAB=$v timeout -k 10 200 python scripts/gemm_bench.py all 20 bf16 2>/dev/null | grep -E "fwd|dgrad|wgrad ffn|sq4k" || exit 1
  done
done
bash scripts/ab_env_bench.sh 3 K3M_B16_LAB "0 4" 2 r6o
