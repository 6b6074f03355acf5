#!/bin/bash
# WRITE_SIZE / FETCH_SIZE calibration of the access widths inflate2_kernel uses (tools/wcal.hip):
# two separate --pmc passes; prints counter bytes / moved bytes per kernel (2nd repetition)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/wcal
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in WRITE_SIZE FETCH_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o x -- $R/tools/wcal > $OUT/$c.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$c rc=$rc"; tail -5 $OUT/$c.log; exit $rc; }
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
moved = {"st_dword_wave": 1 << 30, "st_byte_wave": 1 << 30, "st_dwordx4_wave": 1 << 30, "st_lane16": 1 << 30,
         "st_lane32": 1 << 30, "ld_dwordx4_wave": 1 << 30, "ld_dword_wave": 1 << 30, "ld_byte_wave": 1 << 30,
         "ld_byte_gather": 4096 * 224 * 16 * 64}
for c in ("WRITE_SIZE", "FETCH_SIZE"):
    v = collections.defaultdict(list)
    for f in glob.glob(f"{out}/{c}/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(float)
        name = {}
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == c:
                per[row["Dispatch_Id"]] += float(row["Counter_Value"])
                name[row["Dispatch_Id"]] = row["Kernel_Name"]
        for d in sorted(per, key=int):
            k = name[d].split("(")[0].split()[-1]
            v[k].append(per[d] * 1024)
    for k, vals in v.items():
        print(f"{c:10s} {k:18s} counter {vals[-1] / 1e9:8.4f} GB  moved {moved.get(k, 0) / 1e9:8.4f} GB  "
              f"ratio {vals[-1] / moved.get(k, 1):6.3f}")
PY
