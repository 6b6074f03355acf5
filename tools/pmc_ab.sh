#!/bin/bash
# SQ counters of the inflate kernel for several builds: tools/pmc_ab.sh lib1.so lib2.so ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_ab
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY"
for lib in "$@"; do
  b=$(basename $lib .so)
  HSDS_AMD_DEV=1 HSDS_AMD_LIB=$R/$lib timeout -k 10 300 rocprofv3 --pmc $SQ --output-format csv -d $OUT/$b -o $b -- \
    python3 $R/tools/pmc_run.py F1 2048 > $OUT/$b.log 2>&1
  rc=$?; echo "$b rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/$b.log; exit $rc; }
  python3 - $OUT/$b <<'PY'
import csv, glob, sys, collections
tot = collections.Counter(); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "inflate_kernel" in row["Kernel_Name"]:
            tot[row["Counter_Name"]] += float(row["Counter_Value"])
w = tot["SQ_WAVES"] or 1
print("  " + " ".join(f"{k}={v:.4g}" for k, v in sorted(tot.items())))
ins = tot["SQ_INSTS_VALU"] + tot["SQ_INSTS_SALU"] + tot["SQ_INSTS_LDS"] + tot["SQ_INSTS_BRANCH"]
print(f"  per-wave-cycles/instr={tot['SQ_WAVE_CYCLES']/max(1,ins):.2f} wait_any/wave_cycles={tot['SQ_WAIT_ANY']/max(1,tot['SQ_WAVE_CYCLES']):.3f}")
PY
done
