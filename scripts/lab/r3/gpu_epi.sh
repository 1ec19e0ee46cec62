#!/bin/bash
# GEMM epilogue rework check: kernel tests, fp32/bf16 GEMM microbenchmarks, bench configs 2 and 3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_x6.py tests/test_gpu_gemm_bf16.py tests/test_gpu_gemm_b16_big.py > gpurun_out/epi_tests.log 2>&1; rc=$?; echo "gemm tests rc=$rc"; tail -2 gpurun_out/epi_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 200 python scripts/gemm_bench.py all 10 fp32 > gpurun_out/epi_gemm_f32.log 2>&1 || exit 1
timeout -k 10 200 python scripts/gemm_bench.py all 10 bf16 > gpurun_out/epi_gemm_b16.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 4 | tail -1 | cut -c1-250
timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --steps 10 --warmup 4 | tail -1 | cut -c1-250
