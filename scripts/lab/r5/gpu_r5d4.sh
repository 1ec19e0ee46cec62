#!/bin/bash
# HEAD PMC record of the FFN1 forward (ping-pong loop), and the weight-gradient walk with / without ping-pong
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/pmc_gemm.sh r5dffn1 "fwd ffn1 gelu" fp32 || exit 1
python scripts/pmc_table.py r5dffn1 "gemm_x6_persist_kernel<256, 256, 4, 2, 16, true, true, 2, true, true>" 99052683264 589824000 20992,3072,768 > gpurun_out/r5d_pmc_x6_ffn1_pp.json || exit 1
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD"
for v in 31 63; do
  i=0
  for P in "$P1" "$P2" "FETCH_SIZE"; do
    i=$((i+1))
    K3M_X6_PP=$v timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmc_wg${v}_$i -o run -- python scripts/gemm_bench.py "wgrad ffn1" 3 fp32 > gpurun_out/pmc_wg${v}_$i.log 2>&1
    rc=$?; echo "wg $v pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python scripts/pmc_table.py wg$v "persist_kernel<256, 256, 2, 4, 16, false, false" 99052683264 > gpurun_out/r5d_pmc_wgrad_pp$v.json
done
python - <<'PY'
import json
for f in ["gpurun_out/r5d_pmc_x6_ffn1_pp.json", "gpurun_out/r5d_pmc_wgrad_pp31.json", "gpurun_out/r5d_pmc_wgrad_pp63.json"]:
    d = json.load(open(f))
    print(f, {k: (round(v, 4) if isinstance(v, float) else v) for k, v in d.items() if k not in ("counters_mean_per_dispatch", "dispatches", "kernel_names")})
PY
