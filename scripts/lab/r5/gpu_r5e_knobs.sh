#!/bin/bash
# tile-policy knobs re-checked under the ping-pong walks (config 2, interleaved)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/ab_env.sh K3M_X6_TILE256 "15 7" 3 --steps 10 --warmup 4 > gpurun_out/r5e_knob_tile256.txt 2>&1 || { cat gpurun_out/r5e_knob_tile256.txt; exit 1; }
cat gpurun_out/r5e_knob_tile256.txt
bash scripts/ab_env.sh K3M_X6_P_MIN "100 50 200" 2 --steps 10 --warmup 4 > gpurun_out/r5e_knob_pmin.txt 2>&1 || { cat gpurun_out/r5e_knob_pmin.txt; exit 1; }
cat gpurun_out/r5e_knob_pmin.txt
