#!/bin/bash
# split-K slice cost knobs re-checked on the current kernels (same box, interleaved)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
bash scripts/ab_env_bench.sh 3 K3M_SPLITK_COST_BF16 "0.02 0.05 0.1" 2 r6z || exit 1
bash scripts/ab_env_bench.sh 2 K3M_SPLITK_COST_F32 "0.01 0.03" 2 r6z || exit 1
