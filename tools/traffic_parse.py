"""Per-launch HBM bytes of inflate_kernel from the FETCH_SIZE / WRITE_SIZE passes.
FETCH_SIZE and WRITE_SIZE are in KB (rocprofv3 derived counters, 1024 B units);
FETCH_SIZE is doubled per the gfx950 correction (MI355X_MICROARCH.md, HBM section)."""
import csv
import glob
import json
import os
import sys

out = sys.argv[1]


def per_launch(pattern, counter, kernel="inflate_kernel"):
    vals = {}
    for f in glob.glob(os.path.join(out, pattern, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == counter and kernel in row["Kernel_Name"]:
                vals[row["Dispatch_Id"]] = vals.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
    return vals


fetch = per_launch("fetch", "FETCH_SIZE")
write = per_launch("write", "WRITE_SIZE")
if not fetch or not write:
    sys.exit("no inflate_kernel counter rows found")
f_kb = sum(fetch.values()) / len(fetch)
w_kb = sum(write.values()) / len(write)
res = {"kernel": "inflate_kernel", "launches": [len(fetch), len(write)],
       "fetch_size_kb": f_kb, "write_size_kb": w_kb,
       "bytes_per_launch": int(2 * f_kb * 1024 + w_kb * 1024),
       "formula": "2*FETCH_SIZE + WRITE_SIZE (KB -> bytes)",
       "chunks": 4096, "unique": 1024,
       "source": "profiles/r1_traffic.json (tools/pmc_traffic.sh: rocprofv3 --pmc FETCH_SIZE, --pmc WRITE_SIZE)"}
print(json.dumps(res, indent=1))
