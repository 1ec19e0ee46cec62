#!/bin/bash
# AdamW sweep unroll A/B (K3M_ADAM_UNROLL 1 vs 2) on the config-3 and config-2 steps, plus the optimizer tests
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_trainer.py tests/test_gpu_kernels.py -k "adam or trainer or optim" > gpurun_out/adam_tests.txt 2>&1
echo "## config 3"
bash scripts/ab_env.sh K3M_ADAM_UNROLL "1 2" 3 --config 3 --steps 20
echo "## config 2"
bash scripts/ab_env.sh K3M_ADAM_UNROLL "1 2" 2 --config 2 --steps 12
