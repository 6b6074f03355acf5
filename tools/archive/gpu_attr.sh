#!/bin/bash
# instruction / time attribution of the inflate kernel by compiling phases out:
# tools/gpu_attr.sh lib1 lib2 ...  (abtmp/*.so from tools/ablib.sh); per lib one SQ pass
# (instructions + cycles) over the bench workload (4096 F1 chunks), statuses unchecked
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/attr
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename $lib .so)
  HZ_NOCHECK=1 HSDS_AMD_DEV=1 HSDS_AMD_LIB=$R/$lib timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_BRANCH \
    --output-format csv -d $OUT/$n -o $n -- python3 $R/tools/pmc_run.py F1 4096 > $OUT/$n.log 2>&1
  rc=$?; echo "$n rc=$rc $(grep 'pmc_run done' $OUT/$n.log)"
  [ $rc -eq 0 ] || { tail -5 $OUT/$n.log; exit $rc; }
done
