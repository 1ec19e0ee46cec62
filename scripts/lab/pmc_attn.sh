#!/bin/bash
# SQ counter passes over the short attention kernels (scripts/lab/attn_stamps, one shape; each pass
# its own rocprofv3 run, <= 8 SQ counters each).  usage: scripts/lab/pmc_attn.sh <shape index> <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
S=$1; T=$2
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD"
P3="SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_EXP SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmc_${T}_$i -o run -- scripts/lab/attn_stamps "$S" > gpurun_out/pmc_${T}_$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
