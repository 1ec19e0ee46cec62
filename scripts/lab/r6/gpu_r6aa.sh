#!/bin/bash
# fp32 weight-gradient split knobs re-checked on the current kernels (config 2, same box, interleaved)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
bash scripts/ab_env_bench.sh 2 K3M_SPLITK_MINK_F32 "1024 768 1536 2048" 2 r6aa || exit 1
bash scripts/ab_env_bench.sh 2 K3M_SPLITK_FILL "1 0" 2 r6aa || exit 1
