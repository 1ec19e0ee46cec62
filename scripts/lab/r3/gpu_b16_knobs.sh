#!/bin/bash
# bf16 tile-policy knobs on the config-3 step, interleaved (scripts/ab_env.sh)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "## K3M_B16_MIN (fewest 256x128 tiles for the large-tile kernel)"
bash scripts/ab_env.sh K3M_B16_MIN "160 80 40" 2 --config 3 --steps 20
echo "## K3M_B16_256 (fewest 256x256 tiles for the 256x256 kernel)"
bash scripts/ab_env.sh K3M_B16_256 "192 128 256" 2 --config 3 --steps 20
echo "## K3M_SPLITK_COST_BF16 (bf16 weight-gradient split-K)"
bash scripts/ab_env.sh K3M_SPLITK_COST_BF16 "0.02 0.2" 2 --config 3 --steps 20
echo "## K3M_SPLITK_COST_F32 (fp32 weight-gradient split-K), config 2"
bash scripts/ab_env.sh K3M_SPLITK_COST_F32 "0.01 0.03" 2 --config 2 --steps 12
