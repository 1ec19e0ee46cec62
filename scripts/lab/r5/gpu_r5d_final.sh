#!/bin/bash
# HEAD: whole GPU suite, smoke, default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5d_gpu_tests.txt 2>&1
rc=$?; tail -5 gpurun_out/r5d_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5d_smoke.txt 2>&1 || { tail -20 gpurun_out/r5d_smoke.txt; exit 1; }
tail -3 gpurun_out/r5d_smoke.txt
