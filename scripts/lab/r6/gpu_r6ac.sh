#!/bin/bash
# bf16 flash attention (L <= 128): exp2-domain softmax, one fewer multiply per score, no per-score bounds test in the
# forward's dropout; parity tests then same-box A/B against the previous build (prevlib/)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out/r6ac
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm_bf16.py tests/test_gpu_train_mode_parity.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py > gpurun_out/r6ac/tests.txt 2>&1 || { tail -30 gpurun_out/r6ac/tests.txt; exit 1; }
tail -2 gpurun_out/r6ac/tests.txt
for r in 1 2; do
  for v in new prev; do
    if [ $v = prev ]; then lib=prevlib/libk3m_hip.so; else lib=k3m_amd/libk3m_hip.so; fi
    K3M_LIB=$lib timeout -k 10 200 python scripts/attn_bench.py bf16 > gpurun_out/r6ac/attn_${v}_$r.txt 2>&1 || exit 1
    echo "== $v round $r"; grep "flash" gpurun_out/r6ac/attn_${v}_$r.txt | head -9
  done
done
bash scripts/ab_lib_bench.sh 3 prevlib/libk3m_hip.so 2 r6ac || exit 1
bash scripts/ab_lib_bench.sh 4 prevlib/libk3m_hip.so 2 r6ac || exit 1
