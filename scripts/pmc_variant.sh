#!/bin/bash
# One SQ/GRBM counter pass per x6 variant on the FFN1 forward (clock and MFMA busy per variant).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
for v in $1; do
  K3M_X6_VARIANT=$v timeout -s KILL 90 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d gpurun_out/pmc_var${v}_1 -o run -- python scripts/gemm_bench.py "fwd ffn1 gelu" 3 fp32 > gpurun_out/pmc_var${v}.log 2>&1
  rc=$?; echo "variant $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
