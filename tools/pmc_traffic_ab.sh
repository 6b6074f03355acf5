#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of inflate2_kernel for several builds (traffic attribution by
# compiling phases out): tools/pmc_traffic_ab.sh lib1.so lib2.so ...  (workload: pmc_run.py
# F1 2048, statuses unchecked so that experiment builds can run)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_tab
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  b=$(basename $lib .so)
  for c in FETCH_SIZE WRITE_SIZE; do
    HZ_NOCHECK=1 HSDS_AMD_DEV=1 HSDS_AMD_LIB=$R/$lib timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/$b.$c -o x -- \
      python3 $R/tools/pmc_run.py F1 2048 > $OUT/$b.$c.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$b $c rc=$rc"; tail -5 $OUT/$b.$c.log; exit $rc; }
  done
  python3 - $OUT $b <<'PY'
import csv, glob, sys, collections
out, b = sys.argv[1], sys.argv[2]
res = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    v = collections.defaultdict(float)
    for f in glob.glob(f"{out}/{b}.{c}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "inflate2_kernel" in row["Kernel_Name"] and row["Counter_Name"] == c:
                v[row["Dispatch_Id"]] += float(row["Counter_Value"])
    res[c] = sum(v.values()) / max(1, len(v)) * 1024 / 1e9
print(f"{b:24s} fetch {res['FETCH_SIZE']:8.3f} GB  write {res['WRITE_SIZE']:8.3f} GB  per launch (2048 chunks)")
PY
done
