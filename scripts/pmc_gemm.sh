#!/bin/bash
# rocprofv3 counter passes over one product GEMM shape (scripts/gemm_bench.py -> k3m_gemm), each pass a
# run of its own (per-pass slot limits: 8 SQ, 4 TCC, 2 GRBM).  Summarise with scripts/pmc_table.py.
# usage: scripts/pmc_gemm.sh <tag> "<shape name>" <fp32|bf16>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=$1; S=$2; D=$3
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD"
P3="SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_IFETCH SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
P4="FETCH_SIZE"
P5="WRITE_SIZE TCC_HIT_sum"
i=0
[ -s gpurun_out/pmc_avail.txt ] || timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/pmc_avail.txt 2>&1 || true
for P in "$P1" "$P2" "$P4" "$P5" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmc_${T}_$i -o run -- python scripts/gemm_bench.py "$S" 3 "$D" > gpurun_out/pmc_${T}_$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
