#!/bin/bash
# SQ counter passes over the zlib encoder (tools/deflate_profile.py: 512 x 1 MiB smooth f32
# chunks, L4), one --pmc pass per counter set, no tracing domains; summaries per kernel.
# Usage: tools/sq_encode.sh [tag] [lib]
set -o pipefail
TAG=${1:-sq_enc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
LIB=$(realpath ${2:-$R/hsds_amd/libhsds_amd.so})
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  HZ_PROF_LIB=$LIB HSDS_AMD_DEV=1 HSDS_AMD_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o p$i -- python3 $R/tools/deflate_profile.py > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
for k in parse_kernel huff_kernel emit_kernel; do python3 $R/tools/pmc_sum.py $OUT $k; done > $OUT/summary.txt
cat $OUT/summary.txt
