#!/bin/bash
# rocprofv3 counter passes over the config-5 PV self-attention (flash-long kernels, bf16), each pass its own run
# usage: scripts/pmc_attn_long.sh <tag> [shape name]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=$1; S=${2:-pv self}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD"
P3="SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_IFETCH SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
P4="FETCH_SIZE"
P5="WRITE_SIZE TCC_HIT_sum"
i=0
for P in "$P1" "$P2" "$P4" "$P5" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmc_${T}_$i -o run -- python scripts/attn_bench.py bf16 cfg5 "$S" > gpurun_out/pmc_${T}_$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
