#!/bin/bash
# Re-check of older scheduling knobs on the current build (interleaved bench runs, one box):
# text/image lock step (K3M_GROUP_TV), grouped weight gradients (K3M_GROUP_WGRAD), grouped 256x256 x6 tiles
# (K3M_X6_TILE256 bit 8), side-stream attention branches (K3M_BRANCH_STREAMS).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "## K3M_GROUP_TV, config 2"; bash scripts/ab_env.sh K3M_GROUP_TV "0 1" 2 --config 2 --steps 12
echo "## K3M_GROUP_TV, config 3"; bash scripts/ab_env.sh K3M_GROUP_TV "0 1" 2 --config 3 --steps 20
echo "## K3M_X6_TILE256, config 2"; bash scripts/ab_env.sh K3M_X6_TILE256 "15 7" 2 --config 2 --steps 12
echo "## K3M_GROUP_WGRAD, config 2"; bash scripts/ab_env.sh K3M_GROUP_WGRAD "1 0" 2 --config 2 --steps 12
echo "## K3M_BRANCH_STREAMS, config 3"; bash scripts/ab_env.sh K3M_BRANCH_STREAMS "1 4" 2 --config 3 --steps 20
