#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -q -s --timeout 500 --timeout-method thread > gpurun_out/t_cfgcmp.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainer.py -x -q --timeout 300 --timeout-method thread -k "deterministic" > gpurun_out/t_det.log 2>&1
bash scripts/prof_cfg.sh 5 r5b_cfg5 2
