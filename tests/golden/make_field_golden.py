"""Goldens for compound field subsets in chunkReadSelection / chunkWriteSelection
(chunkUtil.py:882-995), from the REFERENCE itself: hsds.util.chunkUtil with
select_dt = hsds.util.hdf5dtype.getSubType(dtype, fields) (hdf5dtype.py:857-876), as
GET_Chunk / PUT_Chunk build it from the `fields` query parameter (chunk_dn.py:112-140,
456-497).  Run in the build container only:  python tests/golden/make_field_golden.py

Outputs: field_cases.json (metadata, dtype descrs, expected flags / errors) and
field_cases.npz (chunk arrays, write data and expected outputs as raw bytes)."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refshim  # noqa: E402,F401  (puts /root/reference on sys.path)

from hsds.util import chunkUtil as cu  # noqa: E402
from hsds.util.hdf5dtype import getSubType  # noqa: E402

DTYPES = {
    "mixed": np.dtype([("a", "<i4"), ("b", "<f8"), ("c", "S3"), ("d", "<f4", (2,)), ("e", "<f2")]),
    "nested": np.dtype([("p", [("x", "<f4"), ("y", "<i2")]), ("q", "u1"), ("r", "<c8")]),
    "aligned": np.dtype({"names": ["u", "v", "w"], "formats": ["u1", "<f8", "<i2"], "offsets": [0, 8, 16],
                         "itemsize": 24}),
}


def fill(dt, shape, rng):
    a = np.zeros(shape, dt)
    raw = a.view(np.uint8)
    raw[...] = rng.integers(0, 256, raw.shape, dtype=np.uint8)
    for name in dt.names:
        f = dt.fields[name][0]
        base = f.base if f.subdtype else f
        if base.kind == "f":
            a[name] = np.round(rng.normal(size=a[name].shape) * 100, 1).astype(base)
        elif base.kind == "c":
            a[name] = (rng.normal(size=a[name].shape) + 1j * rng.normal(size=a[name].shape)).astype(base)
        elif base.kind == "V" and base.names:
            for sub in base.names:
                a[name][sub] = (rng.normal(size=a[name][sub].shape) * 50).astype(base.fields[sub][0])
    return a


def main():
    rng = np.random.default_rng(31)
    meta, arrs = {"read": [], "write": []}, {}
    meta["dtypes"] = {k: np.lib.format.dtype_to_descr(v) for k, v in DTYPES.items()}
    reads = [("mixed", (12, 20), (slice(1, 12, 2), slice(0, 20, 3)), ["b"]),
             ("mixed", (12, 20), (slice(0, 12, 1), slice(5, 17, 1)), ["d", "a"]),
             ("mixed", (12, 20), (slice(3, 4, 1), slice(0, 20, 7)), ["c", "e", "b", "a"]),
             ("mixed", (12, 20), (slice(0, 12, 5), slice(0, 20, 1)), ["a", "b", "c", "d", "e"]),
             ("mixed", (12, 20), (slice(0, 12, 5), slice(0, 20, 1)), ["d"]),
             ("nested", (6, 5, 7), (slice(0, 6, 2), slice(1, 5, 1), slice(0, 7, 3)), ["p"]),
             ("nested", (6, 5, 7), (slice(0, 6, 1), slice(0, 5, 2), slice(2, 7, 1)), ["r", "q"]),
             ("aligned", (40,), (slice(3, 40, 4),), ["w", "u"]),
             ("aligned", (40,), (slice(0, 40, 1),), ["v"])]
    for k, (dn, shape, sl, fields) in enumerate(reads):
        dt = DTYPES[dn]
        arr = fill(dt, shape, rng)
        name = f"read{k}"
        case = {"name": name, "dtype": dn, "shape": list(shape), "slices": [[s.start, s.stop, s.step] for s in sl],
                "fields": fields}
        arrs[name + "__chunk"] = arr.view(np.uint8).reshape(-1)
        try:
            sdt = getSubType(dt, fields)
            out = cu.chunkReadSelection(arr, slices=sl, select_dt=sdt)
            case["out_shape"] = list(out.shape)
            case["out_descr"] = np.lib.format.dtype_to_descr(out.dtype)
            case["out_itemsize"] = out.dtype.itemsize
            arrs[name + "__out"] = np.ascontiguousarray(out).view(np.uint8).reshape(-1)
        except Exception as e:          # noqa: BLE001 - the reference's error is the golden
            case["error"] = type(e).__name__
        meta["read"].append(case)
    writes = [("mixed", (12, 20), (slice(1, 12, 2), slice(0, 20, 3)), ["b"], None),
              ("mixed", (12, 20), (slice(0, 12, 1), slice(5, 17, 1)), ["d", "a"], None),
              ("mixed", (12, 20), (slice(0, 12, 3), slice(0, 20, 2)), ["b", "e"], "same"),
              ("mixed", (12, 20), (slice(0, 12, 3), slice(0, 20, 2)), ["b", "a"], "negzero"),
              ("mixed", (12, 20), (slice(0, 12, 3), slice(0, 20, 2)), ["b"], "nan"),
              ("mixed", (12, 20), (slice(2, 9, 1), slice(1, 20, 6)), None, "negzero"),
              ("mixed", (12, 20), (slice(2, 9, 1), slice(1, 20, 6)), None, "nan"),
              ("mixed", (12, 20), (slice(2, 9, 1), slice(1, 20, 6)), None, None),
              ("nested", (6, 5, 7), (slice(0, 6, 2), slice(1, 5, 1), slice(0, 7, 3)), ["r", "p"], None),
              ("nested", (6, 5, 7), (slice(0, 6, 2), slice(1, 5, 1), slice(0, 7, 3)), ["q"], "same"),
              ("aligned", (40,), (slice(3, 40, 4),), ["w", "v"], None)]
    for k, (dn, shape, sl, fields, mode) in enumerate(writes):
        dt = DTYPES[dn]
        arr = fill(dt, shape, rng)
        sdt = getSubType(dt, fields) if fields else dt
        sel_shape = arr[sl].shape
        data = np.zeros(sel_shape, sdt)
        cur = arr[sl]
        for f in sdt.names:
            data[f] = fill(dt, sel_shape, rng)[f] if mode is None else cur[f]
        if mode == "negzero":
            # 0.0 stored, -0.0 written: equal under ndarray_compare, so not written
            arr["b"][sl] = 0.0
            data["b"] = -0.0
            if fields and "a" in fields:
                data["a"] = cur["a"] + 1          # field a differs: written; b stays +0.0
        elif mode == "nan":
            arr["b"][sl] = np.nan
            data["b"] = np.nan                    # NaN != NaN: the field counts as updated
        name = f"write{k}"
        case = {"name": name, "dtype": dn, "shape": list(shape), "slices": [[s.start, s.stop, s.step] for s in sl],
                "fields": fields, "mode": mode}
        arrs[name + "__chunk"] = arr.view(np.uint8).reshape(-1).copy()
        arrs[name + "__data"] = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
        a2 = arr.copy()
        upd = cu.chunkWriteSelection(chunk_arr=a2, slices=sl, data=data)
        upd2 = cu.chunkWriteSelection(chunk_arr=a2, slices=sl, data=data)
        case["updated"], case["updated_again"] = bool(upd), bool(upd2)
        arrs[name + "__out"] = a2.view(np.uint8).reshape(-1)
        meta["write"].append(case)
    with open(os.path.join(HERE, "field_cases.json"), "w") as f:
        json.dump(meta, f, indent=1)
    np.savez_compressed(os.path.join(HERE, "field_cases.npz"), **arrs)
    print(len(meta["read"]), "read cases,", len(meta["write"]), "write cases")
    for c in meta["read"]:
        print(c["name"], c["fields"], c.get("error"), c.get("out_itemsize"))
    for c in meta["write"]:
        print(c["name"], c["fields"], c["mode"], c["updated"], c["updated_again"])


if __name__ == "__main__":
    main()
