#!/bin/bash
# split-K cost weight re-checked under the ping-pong walks (config 2, interleaved)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/ab_env.sh K3M_SPLITK_COST_F32 "0.01 0.03 0.06" 3 --steps 10 --warmup 4 > gpurun_out/r5e_knob_splitk.txt 2>&1 || { cat gpurun_out/r5e_knob_splitk.txt; exit 1; }
cat gpurun_out/r5e_knob_splitk.txt
