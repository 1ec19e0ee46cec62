#!/bin/bash
# cheaper GELU forms: GEMM / parity / kernel tests, GEMM shapes, then same-box A/B against the previous build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out/r6r
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm_bf16.py tests/test_gpu_gemm_x6.py tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_gemm_b16_dual.py > gpurun_out/r6r/tests.txt 2>&1
rc=$?; tail -1 gpurun_out/r6r/tests.txt; [ $rc -eq 0 ] || { grep -E "Error|FAILED" gpurun_out/r6r/tests.txt | head; exit $rc; }
for lib in k3m_amd/libk3m_hip.so k3m_amd/lab_prev/libk3m_hip.so k3m_amd/libk3m_hip.so k3m_amd/lab_prev/libk3m_hip.so; do
  echo "== $lib"
  K3M_LIB=$lib timeout -k 10 200 python scripts/gemm_bench.py gelu 20 both 2>/dev/null | grep -i gelu || exit 1
done
bash scripts/ab_lib_bench.sh 3 k3m_amd/lab_prev/libk3m_hip.so 2 r6r && bash scripts/ab_lib_bench.sh 2 k3m_amd/lab_prev/libk3m_hip.so 2 r6r
