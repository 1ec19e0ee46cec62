#!/bin/bash
# the whole GPU suite + smoke on the current build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r6k
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6k/gpu_tests.txt 2>&1
rc=$?
tail -5 gpurun_out/r6k/gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "Error|FAILED|failed" gpurun_out/r6k/gpu_tests.txt | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6k/smoke.txt 2>&1 || { tail -20 gpurun_out/r6k/smoke.txt; exit 1; }
tail -3 gpurun_out/r6k/smoke.txt
