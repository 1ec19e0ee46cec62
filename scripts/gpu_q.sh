#!/bin/bash
# round-5 GPU step: GEMM + determinism tests, per-call GEMM table, dynamic-queue A/B (configs 2 and 3)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_gemm_x6.py tests/test_gpu_gemm_bf16.py tests/test_gpu_gemm_b16_dual.py tests/test_gpu_gemm_b16_big.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_gemm_q.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest tests/test_gpu_trainer.py -x -q --timeout 300 --timeout-method thread -k "deterministic" > gpurun_out/t_det.log 2>&1
timeout -k 10 400 python scripts/gemm_calls.py --config 2 --top 70 > gpurun_out/gc2_q1.txt 2>&1 || exit $?
timeout -k 10 600 scripts/ab_env.sh K3M_DYN_QUEUE "0 1" 2 --steps 20 --warmup 8 > gpurun_out/ab_q_cfg2.txt 2>&1 || exit $?
timeout -k 10 600 scripts/ab_env.sh K3M_DYN_QUEUE "0 1" 2 --config 3 --steps 20 --warmup 8 > gpurun_out/ab_q_cfg3.txt 2>&1
