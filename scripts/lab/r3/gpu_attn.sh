#!/bin/bash
# attention x6 check: kernel tests + goldens, then interleaved microbenchmarks K3M_ATTN_X6=0/1
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_train_mode_parity.py > gpurun_out/attn_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/attn_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for r in 1 2; do for x in 0 1; do K3M_ATTN_X6=$x timeout -k 10 200 python scripts/attn_bench.py fp32 2>/dev/null | sed "s/^/X6=$x /"; done; done
