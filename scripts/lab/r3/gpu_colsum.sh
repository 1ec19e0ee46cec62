#!/bin/bash
# dGELU colsum-slab fusion: kernel tests, goldens, engine-level A/B (K3M_DGRAD_COLSUM)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm_x6.py tests/test_gpu_gemm_bf16.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_ddp_engine.py > gpurun_out/colsum_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/colsum_tests.log
[ $rc -ne 0 ] && exit $rc
K3M_DGRAD_COLSUM=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py > gpurun_out/colsum_tests0.log 2>&1; rc=$?; echo "tests (COLSUM=0) rc=$rc"; tail -1 gpurun_out/colsum_tests0.log
[ $rc -ne 0 ] && exit $rc
for m in 0 1 0 1; do K3M_DGRAD_COLSUM=$m timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 4 | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('fp32 COLSUM=$m', d['value'], d['ms_per_step'], d['coattn']['frac'])"; done
for m in 0 1 0 1; do K3M_DGRAD_COLSUM=$m timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --steps 10 --warmup 4 | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('bf16 COLSUM=$m', d['value'], d['ms_per_step'], d['coattn']['frac'])"; done
