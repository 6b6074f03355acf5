"""sum rocprofv3 counter_collection.csv per counter for the inflate kernel dispatches:
python tools/pmc_sum.py DIR [kernel-substring]"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "inflate2_kernel"
tot = defaultdict(float)
disp = set()
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kname not in r.get("Kernel_Name", ""):
            continue
        disp.add(r.get("Dispatch_Id"))
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
n = max(len(disp), 1)
print(f"{d}: {len(disp)} dispatches of {kname}")
for k in sorted(tot):
    print(f"  {k:24s} {tot[k] / n:.4g} per dispatch")
