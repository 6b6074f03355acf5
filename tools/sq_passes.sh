#!/bin/bash
# SQ stall/issue counter passes over a fixed F1 (or F2) decode workload (tools/pmc_run.py),
# one --pmc pass per counter set, no tracing domains.  Usage: tools/sq_passes.sh [F1|F2] [tag]
set -o pipefail
FMT=${1:-F1}; TAG=${2:-sq}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o p$i -- python3 $R/tools/pmc_run.py $FMT 512 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
