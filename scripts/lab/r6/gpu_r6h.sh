#!/bin/bash
# attention kernel timings with and without probability dropout (the cost of the counter hash)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for pp in 0.1 0; do
  echo "== ATTN_P=$pp cfg5 bf16"
  ATTN_P=$pp timeout -k 10 120 python scripts/attn_bench.py bf16 cfg5 2>/dev/null | grep flash || exit 1
  echo "== ATTN_P=$pp bs64 both"
  ATTN_P=$pp timeout -k 10 120 python scripts/attn_bench.py both 2>/dev/null || exit 1
done
