#!/bin/bash
# SQ counter passes over one lab kernel (each pass its own rocprofv3 run; <= 8 SQ counters each).
# usage: scripts/lab/pmc_lab.sh <shape-substring> <variant-substring> <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=$1; V=$2; T=$3
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/pmc_avail.txt 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmc_${T}_$i -o run -- scripts/lab/gemm_lab 3 "$S" "$V" > gpurun_out/pmc_${T}_$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
