"""Per-launch HBM bytes from the FETCH_SIZE / WRITE_SIZE passes of tools/pmc_traffic.sh.
FETCH_SIZE and WRITE_SIZE are in KB (rocprofv3 derived counters, 1024 B units);
FETCH_SIZE is doubled per the gfx950 correction (MI355X_MICROARCH.md, HBM section).

    traffic_parse.py OUT [round]        headline: inflate2_kernel, per launch
    traffic_parse.py OUT round cfg3     cfg3 leg: every kernel of the step, per step
    traffic_parse.py OUT round cfg4     cfg4 leg: the same over the cfg4 passes
                                        (one inflate2_kernel launch per step)"""
import csv
import glob
import json
import os
import re
import sys

KERNEL = "inflate2_kernel"


def kernel_short_name(name):
    """The function name of a demangled kernel signature: return type, namespaces
    (including '(anonymous namespace)'), template arguments and the parameter list
    removed -- '(anonymous namespace)::inflate2_kernel(Item const*, ...)' -> 'inflate2_kernel',
    'void at::native::elementwise_kernel<128, 4, ...>(int, ...)' -> 'elementwise_kernel'."""
    s = name.strip().replace("(anonymous namespace)", "anon")
    s = re.sub(r"^(void|int|unsigned int)\s+", "", s)
    # cut at the parameter list: the first '(' outside template brackets
    depth, cut = 0, len(s)
    for i, ch in enumerate(s):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            cut = i
            break
    s = s[:cut]
    # drop template arguments, then namespaces
    out, depth = [], 0
    for ch in s:
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif depth == 0:
            out.append(ch)
    s = "".join(out)
    return s.split("::")[-1].strip() or name.strip()


def rows(out, pattern, counter):
    per = {}
    for f in glob.glob(os.path.join(out, pattern, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == counter:
                k = (row["Dispatch_Id"], row["Kernel_Name"])
                per[k] = per.get(k, 0.0) + float(row["Counter_Value"])
    return per


def inflate_only(per):
    return [x for (d, name), x in per.items() if kernel_short_name(name) == KERNEL]


def per_step(out, rnd, leg, fpat, wpat):
    fp, wp = rows(out, fpat, "FETCH_SIZE"), rows(out, wpat, "WRITE_SIZE")
    nf = len(inflate_only(fp))
    nw = len(inflate_only(wp))
    if not nf or not nw:
        sys.exit(f"no {KERNEL} counter rows found in the {leg} passes")
    by_kernel = {}
    for (d, name), x in fp.items():
        by_kernel.setdefault(kernel_short_name(name), [0.0, 0.0])[0] += x / nf * 1024
    for (d, name), x in wp.items():
        by_kernel.setdefault(kernel_short_name(name), [0.0, 0.0])[1] += x / nw * 1024
    f_b = sum(v[0] for v in by_kernel.values())
    w_b = sum(v[1] for v in by_kernel.values())
    return {"leg": leg, "steps_profiled": [nf, nw],
            "fetch_bytes_per_step": int(f_b), "write_bytes_per_step": int(w_b),
            "bytes_per_step": int(2 * f_b + w_b), "bytes_per_step_undoubled": int(f_b + w_b),
            "per_kernel_fetch_write_bytes": {k: [int(a), int(b)] for k, (a, b) in sorted(by_kernel.items())},
            "formula": "sum over the step's kernels of 2*FETCH_SIZE + WRITE_SIZE (KB -> bytes)",
            "source": f"profiles/{rnd}_traffic_{leg}.json (tools/pmc_traffic.sh {leg} passes)"}


def main(argv):
    out = argv[1]
    rnd = argv[2] if len(argv) > 2 else "r2"
    mode = argv[3] if len(argv) > 3 else "headline"
    if mode == "headline":
        fetch = inflate_only(rows(out, "fetch", "FETCH_SIZE"))
        write = inflate_only(rows(out, "write", "WRITE_SIZE"))
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
               "source": f"profiles/{rnd}_traffic.json (tools/pmc_traffic.sh: rocprofv3 --pmc FETCH_SIZE, "
                         f"--pmc WRITE_SIZE)"}
    elif mode == "cfg3":
        res = per_step(out, rnd, "cfg3", "fetch3", "write3")
    else:
        res = per_step(out, rnd, "cfg4", "fetch4", "write4")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv)
