#!/bin/bash
# PMC: bf16 FFN1 GELU forward on the dual kernel (HEAD default) and on the epilogue-wave kernel; FFN2 forward on the
# 256x256 walk and on the epilogue-wave kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
K3M_B16_WS=0 bash scripts/pmc_gemm.sh r6dual "fwd ffn1 gelu" bf16 || exit 1
python scripts/pmc_table.py r6dual "gemm_dual_kernel<256, 128, 2, 2, true, true, 2" 99052683264 295698432 20992,3072,768 > gpurun_out/r6_pmc_b16_ffn1_dual.json || exit 1
K3M_B16_WS=3 bash scripts/pmc_gemm.sh r6ws "fwd ffn1 gelu" bf16 || exit 1
python scripts/pmc_table.py r6ws "gemm_ws_kernel<2>" 99052683264 295698432 20992,3072,768 > gpurun_out/r6_pmc_b16_ffn1_ws.json || exit 1
K3M_B16_WS=0 bash scripts/pmc_gemm.sh r6f2 "fwd ffn2" bf16 || exit 1
python scripts/pmc_table.py r6f2 "gemm_persist_kernel<256, 256, 2, 4, true, true, 1" 99052683264 165150720 20992,768,3072 > gpurun_out/r6_pmc_b16_ffn2_walk.json || exit 1
K3M_B16_WS=3 bash scripts/pmc_gemm.sh r6f2ws "fwd ffn2" bf16 || exit 1
python scripts/pmc_table.py r6f2ws "gemm_ws_kernel<1>" 99052683264 165150720 20992,768,3072 > gpurun_out/r6_pmc_b16_ffn2_ws.json || exit 1
for f in gpurun_out/r6_pmc_b16_*.json; do
python -c "
import json,sys; d=json.load(open('$f'))
print('$f', {k: (round(v, 4) if isinstance(v, float) else v) for k, v in d.items() if k not in ('counters_mean_per_dispatch', 'dispatches', 'kernel_names')})"
done
