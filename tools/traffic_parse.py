"""Per-launch HBM bytes from the FETCH_SIZE / WRITE_SIZE passes of tools/pmc_traffic.sh.
FETCH_SIZE and WRITE_SIZE are in KB (rocprofv3 derived counters, 1024 B units);
FETCH_SIZE is doubled per the gfx950 correction (MI355X_MICROARCH.md, HBM section).

    traffic_parse.py OUT [round]        headline: inflate2_kernel, per launch
    traffic_parse.py OUT round cfg3     cfg3 leg: every kernel of the step, per step
                                        (one inflate2_kernel launch per step)"""
import csv
import glob
import json
import os
import sys

out = sys.argv[1]
rnd = sys.argv[2] if len(sys.argv) > 2 else "r2"
mode = sys.argv[3] if len(sys.argv) > 3 else "headline"
KERNEL = "inflate2_kernel"


def rows(pattern, counter):
    per = {}
    for f in glob.glob(os.path.join(out, pattern, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == counter:
                k = (row["Dispatch_Id"], row["Kernel_Name"])
                per[k] = per.get(k, 0.0) + float(row["Counter_Value"])
    return per


def inflate_only(per):
    v = [x for (d, name), x in per.items() if KERNEL in name]
    return v


if mode == "headline":
    fetch = inflate_only(rows("fetch", "FETCH_SIZE"))
    write = inflate_only(rows("write", "WRITE_SIZE"))
    if not fetch or not write:
        sys.exit(f"no {KERNEL} counter rows found")
    f_kb = sum(fetch) / len(fetch)
    w_kb = sum(write) / len(write)
    res = {"kernel": KERNEL, "launches": [len(fetch), len(write)],
           "fetch_size_kb": f_kb, "write_size_kb": w_kb,
           "bytes_per_launch": int(2 * f_kb * 1024 + w_kb * 1024),
           "bytes_per_launch_undoubled": int(f_kb * 1024 + w_kb * 1024),
           "formula": "2*FETCH_SIZE + WRITE_SIZE (KB -> bytes)",
           "chunks": 4096, "unique": 1024,
           "source": f"profiles/{rnd}_traffic.json (tools/pmc_traffic.sh: rocprofv3 --pmc FETCH_SIZE, --pmc WRITE_SIZE)"}
else:
    fp, wp = rows("fetch3", "FETCH_SIZE"), rows("write3", "WRITE_SIZE")
    nf = len(inflate_only(fp))
    nw = len(inflate_only(wp))
    if not nf or not nw:
        sys.exit(f"no {KERNEL} counter rows found in the cfg3 passes")
    by_kernel = {}
    for (d, name), x in fp.items():
        short = name.split("(")[0].split("::")[-1]
        by_kernel.setdefault(short, [0.0, 0.0])[0] += x / nf * 1024
    for (d, name), x in wp.items():
        short = name.split("(")[0].split("::")[-1]
        by_kernel.setdefault(short, [0.0, 0.0])[1] += x / nw * 1024
    f_b = sum(v[0] for v in by_kernel.values())
    w_b = sum(v[1] for v in by_kernel.values())
    res = {"leg": "cfg3", "steps_profiled": [nf, nw],
           "fetch_bytes_per_step": int(f_b), "write_bytes_per_step": int(w_b),
           "bytes_per_step": int(2 * f_b + w_b), "bytes_per_step_undoubled": int(f_b + w_b),
           "per_kernel_fetch_write_bytes": {k: [int(a), int(b)] for k, (a, b) in sorted(by_kernel.items())},
           "formula": "sum over the step's kernels of 2*FETCH_SIZE + WRITE_SIZE (KB -> bytes)",
           "source": f"profiles/{rnd}_traffic_cfg3.json (tools/pmc_traffic.sh cfg3 passes)"}
print(json.dumps(res, indent=1))
