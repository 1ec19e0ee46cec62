#!/bin/bash
# flash-long forward: dropout as a template parameter (no spills at d = 64): parity tests, then same-box timings
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
mkdir -p gpurun_out/r6u
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm_bf16.py tests/test_gpu_train_mode_parity.py -k "long or flash or attn or train" > gpurun_out/r6u/tests.txt 2>&1 || { tail -30 gpurun_out/r6u/tests.txt; exit 1; }
tail -2 gpurun_out/r6u/tests.txt
for r in 1 2; do
  for v in new prev; do
    if [ $v = prev ]; then lib=prevlib/libk3m_hip.so; else lib=k3m_amd/libk3m_hip.so; fi
    K3M_LIB=$lib timeout -k 10 200 python scripts/attn_bench.py bf16 cfg5 > gpurun_out/r6u/attn_${v}_$r.txt 2>&1 || exit 1
    echo "== $v round $r"; grep -i "pv self\|co" gpurun_out/r6u/attn_${v}_$r.txt | head -12
  done
done
bash scripts/ab_lib_bench.sh 5 prevlib/libk3m_hip.so 2 r6u || exit 1
