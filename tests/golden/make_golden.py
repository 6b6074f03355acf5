"""Generate the golden vectors under tests/golden/ from the REFERENCE itself.

Run in the build container only (needs /root/reference and
/opt/conda/lib/libblosc.so.1):   python tests/golden/make_golden.py

Everything expected here is an output of the reference's own code:
  * hsds.util.storUtil._compress / _uncompress / _shuffle / _unshuffle
    (storUtil.py:94-281) with numcodecs re-expressed over c-blosc 1.21.0
    (tests/golden/refshim.py), and
  * hsds.util.chunkUtil / dsetUtil / idUtil selection and partition functions.
Inputs are synthetic (numpy default_rng seeds recorded next to each case) or copied
from the reference's unit tests (shuffle_test.py:26-41 KAT, compression_test.py).

Outputs:
  codec_cases.npz   -- compressed inputs + decoded outputs (small) or sha256 (large)
  codec_cases.json  -- per-case metadata (filter ops, expected status / sha256)
  selection_cases.json -- selection math goldens (a13-a22 of SURVEY.md section 8a)
"""
import hashlib
import json
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refshim  # noqa: E402  (installs the numcodecs stand-in, puts /root/reference on sys.path)

from hsds.util import storUtil as su  # noqa: E402
from hsds.util import chunkUtil as cu  # noqa: E402
from hsds.util import dsetUtil as du  # noqa: E402
from hsds.util import idUtil as iu  # noqa: E402
from hsds.util.dsetUtil import getFilterOps  # noqa: E402

BIG = 64 * 1024  # outputs above this size are stored as sha256 only


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def smooth(n, dtype, seed):
    rng = np.random.default_rng(seed)
    x = np.round(np.cumsum(rng.normal(size=n)), 2)
    if np.dtype(dtype).kind in "iu":
        return (np.cumsum(rng.normal(size=n)) * 100).astype(dtype)
    return x.astype(dtype)


def filters_json(shuffle, level):
    f = []
    if shuffle:
        f.append({"class": "H5Z_FILTER_SHUFFLE", "id": 2, "name": "shuffle"})
    if level is not None:
        f.append({"class": "H5Z_FILTER_DEFLATE", "id": 1, "level": level, "name": "deflate"})
    return f


def run_uncompress(blob, ops):
    try:
        return su._uncompress(blob, **ops)
    except Exception as e:  # HTTPInternalServerError / ValueError
        return e


def main():
    arrays = {}
    cases = []

    def add_case(name, blob, ops, note, seed=None, raw=None):
        out = run_uncompress(blob, ops)
        case = {"name": name, "note": note, "seed": seed,
                "compressor": ops.get("compressor"), "shuffle": ops.get("shuffle", 0),
                "level": ops.get("level"), "dtype": np.dtype(ops["dtype"]).str if ops.get("dtype") is not None else None,
                "chunk_shape": list(ops["chunk_shape"]) if ops.get("chunk_shape") is not None else None,
                "in_len": len(blob)}
        arrays[name + "__in"] = np.frombuffer(blob, np.uint8)
        if isinstance(out, Exception):
            case["status"] = "error"
            case["error"] = type(out).__name__
        else:
            case["status"] = "ok"
            case["out_len"] = len(out)
            case["out_sha256"] = sha(out)
            if raw is not None:
                assert raw == out, name
            if len(out) <= BIG:
                arrays[name + "__out"] = np.frombuffer(out, np.uint8)
        cases.append(case)

    app = {"filter_map": {}}
    # ---- F1: HSDS-native Blosc-zlib objects, produced by the reference _compress
    f1 = [("f1_f32_1m_L4", np.float32, (512, 512), 4, 1, 20261015),
          ("f1_f32_256k_L1", np.float32, (256, 256), 1, 1, 11),
          ("f1_f32_256k_L3", np.float32, (256, 256), 3, 1, 12),
          ("f1_f32_256k_L5", np.float32, (256, 256), 5, 1, 13),
          ("f1_f32_256k_L9", np.float32, (256, 256), 9, 1, 14),
          ("f1_f32_16k_L4", np.float32, (64, 64), 4, 1, 15),
          ("f1_i16_256k_L4", np.int16, (16, 64, 128), 4, 1, 16),
          ("f1_f64_64k_L4_noshuf", np.float64, (8192,), 4, 0, 17),
          ("f1_f32_leftover_L4", np.float32, (65536 + 250,), 4, 1, 18)]
    for name, dt, shape, level, shuf, seed in f1:
        arr = smooth(int(np.prod(shape)), dt, seed).reshape(shape)
        ops = getFilterOps(app, "d-" + name, filters_json(shuf, level), dtype=arr.dtype, chunk_shape=shape)
        app["filter_map"].clear()
        blob = su._compress(arr.tobytes(), **ops)
        add_case(name, blob, ops, "reference _compress -> _uncompress", seed, arr.tobytes())
    # zeros / random-bits (memcpyed) / tiny
    for name, data, shape, level in (
            ("f1_zeros_1m_L4", bytes(1 << 20), (262144,), 4),
            ("f1_random_64k_L4", np.random.default_rng(7).integers(0, 256, 65536, np.uint8).tobytes(), (16384,), 4),
            ("f1_tiny_12b_L4", bytes(range(12)), (3,), 4),
            ("f1_f32_64k_L0", smooth(16384, np.float32, 19).tobytes(), (16384,), 0)):
        ops = getFilterOps(app, "d-" + name, filters_json(1, level), dtype=np.dtype(np.float32), chunk_shape=shape)
        app["filter_map"].clear()
        blob = su._compress(data, **ops)
        add_case(name, blob, ops, "reference _compress -> _uncompress", None, data)

    # ---- Blosc frames from other writers: typesize > 1 with in-frame shuffle
    for ts, dt, n, seed in ((2, np.int16, 131072, 21), (4, np.float32, 65536, 22), (8, np.float64, 32768, 23),
                            (4, np.float32, 262144 + 1000, 24), (16, np.float32, 8192, 25), (32, np.float32, 8192, 26)):
        data = smooth(n // np.dtype(dt).itemsize + (1 if n % np.dtype(dt).itemsize else 0), dt, seed).tobytes()[:n]
        blob = refshim.blosc_compress_raw(data, 4, 1, ts)
        ops = {"compressor": "zlib", "shuffle": 1, "level": 4, "dtype": np.dtype(dt),
               "chunk_shape": (n // np.dtype(dt).itemsize,)}
        add_case(f"f1_ts{ts}_{n}", blob, ops, "libblosc typesize>1 frame -> reference _uncompress", seed, data)

    # ---- F2: HDF5 chunk = zlib stream of HDF5-byte-shuffled data
    for dt, shape, level, seed in ((np.int16, (16, 64, 128), 4, 31), (np.int32, (128, 128), 4, 32),
                                   (np.float32, (512, 512), 4, 33), (np.float64, (64, 128), 6, 34),
                                   (np.float32, (100, 100), 1, 35), (np.uint8, (4096,), 9, 36)):
        arr = smooth(int(np.prod(shape)), dt, seed).reshape(shape)
        shuffled = refshim.Shuffle(arr.dtype.itemsize).encode(arr.tobytes()).tobytes()
        blob = zlib.compress(shuffled, level)
        ops = {"compressor": "zlib", "shuffle": 1, "level": level, "dtype": arr.dtype, "chunk_shape": shape}
        add_case(f"f2_{np.dtype(dt).name}_{'x'.join(map(str, shape))}_L{level}", blob, ops,
                 "zlib.compress(Shuffle.encode) -> reference _uncompress", seed, arr.tobytes())
    # F2 with stored blocks (level 0) and plain zlib without shuffle (compression_test.py:70-79)
    arr = np.random.default_rng(4).integers(0, 200, 20000).astype("<i4")
    add_case("zlib_i4_noshuffle", zlib.compress(arr.tobytes()), {"compressor": "zlib", "shuffle": 0,
             "dtype": arr.dtype, "chunk_shape": arr.shape}, "compression_test.testZLibCompression", 4, arr.tobytes())
    arr = smooth(30000, np.float32, 41)
    add_case("f2_f32_stored_L0", zlib.compress(refshim.Shuffle(4).encode(arr.tobytes()).tobytes(), 0),
             {"compressor": "zlib", "shuffle": 1, "dtype": arr.dtype, "chunk_shape": arr.shape},
             "stored deflate blocks", 41, arr.tobytes())
    # ---- error cases
    good = zlib.compress(smooth(10000, np.float32, 51).tobytes(), 4)
    bad = bytearray(good)
    bad[-1] ^= 0x55
    ops = {"compressor": "zlib", "shuffle": 0, "dtype": np.dtype(np.float32), "chunk_shape": (10000,)}
    add_case("err_adler32", bytes(bad), ops, "adler32 mismatch -> 500")
    add_case("err_truncated", good[:-20], ops, "truncated stream -> 500")
    bad = bytearray(good)
    bad[2] = (bad[2] & ~0x06) | 0x06  # BTYPE=3 reserved
    add_case("err_btype3", bytes(bad), ops, "invalid block type -> 500")
    blob = bytearray(su._compress(smooth(65536, np.float32, 52).tobytes(), compressor="zlib", level=4,
                                  shuffle=1, dtype=np.dtype(np.float32), chunk_shape=(65536,)))
    blob[40] ^= 0xFF
    ops = {"compressor": "zlib", "shuffle": 1, "dtype": np.dtype(np.float32), "chunk_shape": (65536,)}
    add_case("err_f1_corrupt", bytes(blob), ops, "corrupt split stream -> 500")
    # ---- no compressor, shuffle only (storUtil.py:225-226)
    arr = smooth(4096, np.float64, 61)
    add_case("shuffle_only_f64", refshim.Shuffle(8).encode(arr.tobytes()).tobytes(),
             {"compressor": None, "shuffle": 1, "dtype": arr.dtype, "chunk_shape": arr.shape},
             "_uncompress(compressor=None, shuffle=1)", 61, arr.tobytes())

    # ---- shuffle KAT (tests/unit/shuffle_test.py:26-41)
    kat = np.array([1, 2, 3], dtype="<u2")
    sh = su._shuffle(1, kat.tobytes(), chunk_shape=kat.shape, dtype=kat.dtype)
    un = su._unshuffle(1, sh, chunk_shape=kat.shape, dtype=kat.dtype)
    shuffle_kat = {"in": kat.tobytes().hex(), "shuffled": bytes(sh).hex(), "unshuffled": bytes(un).hex()}
    sh_cases = []
    for dt, n, seed in (("<u2", 3, None), ("<f4", 1000, 71), ("<f8", 777, 72), ("<i2", 4096, 73), ("|u1", 50, 74)):
        a = np.arange(n).astype(dt) if seed is None else smooth(n, dt, seed)
        s = su._shuffle(1, a.tobytes(), chunk_shape=a.shape, dtype=a.dtype)
        sh_cases.append({"dtype": dt, "n": n, "seed": seed, "in": a.tobytes().hex(), "shuffled": bytes(s).hex()})

    np.savez_compressed(os.path.join(HERE, "codec_cases.npz"), **arrays)
    with open(os.path.join(HERE, "codec_cases.json"), "w") as f:
        json.dump({"cases": cases, "shuffle_kat": shuffle_kat, "shuffle_cases": sh_cases}, f, indent=1)

    make_selection_cases()
    print("wrote", len(cases), "codec cases")


def enc_sel(sel):
    out = []
    for s in sel:
        if isinstance(s, slice):
            out.append({"slice": [s.start, s.stop, s.step]})
        else:
            out.append({"coords": [int(x) for x in s]})
    return out


def make_selection_cases():
    dset_id = "d-be8e2c7c-2a6b1dbd-8c64-d1a5e6-4c4d8e"
    cases = {"getSelectionList": [], "getChunkIds": [], "coverage": [], "pagination": [],
             "partition": [], "s3key": [], "readSelection": [], "writeSelection": []}
    sel_strs = [("[1000:3000,500:3500]", [4096, 4096]), ("[0:512:2,3:2048:5,1:2048:3]", [512, 2048, 2048]),
                ("[::4,::4]", [131072, 131072]), ("[5,:]", [10, 20]), ("[:,3:17:4]", [10, 20]),
                ("[2:9]", [10]), ("[[1,4,7],2:5]", [10, 10]), (":", [7]), ("[0:4:2,0:4:2]", [10, 10]),
                ("[3:4]", [10]), ("[1:10:10]", [10]), ("[ 2 : 8 : 3 , 1:2 ]", [10, 5]), ("", [4, 5]),
                ("[0:10,0:10]", [10, 5]), ("[a:3]", [10]), ("[1:2:0]", [10]), ("[7:3]", [10]), ("[1,2]", [10]),
                ("[0:12]", [10]), ("[[1,12]]", [10])]
    for s, dims in sel_strs:
        try:
            r = du.getSelectionList(s, dims)
            cases["getSelectionList"].append({"select": s, "dims": dims, "result": enc_sel(r),
                                              "shape": du.getSelectionShape(r)})
        except ValueError as e:
            cases["getSelectionList"].append({"select": s, "dims": dims, "error": "ValueError", "msg": str(e)})
    # chunk ids + coverage goldens (chunk_util_test.py:851-1047 style)
    sels = [((slice(1000, 3000, 1), slice(500, 3500, 1)), (64, 64), [4096, 4096]),
            ((slice(0, 512, 2), slice(3, 2048, 5), slice(1, 2048, 3)), (16, 64, 128), [512, 2048, 2048]),
            ((slice(0, 100, 1),), (10,), [100]),
            ((slice(5, 95, 7),), (10,), [100]),
            ((slice(3, 97, 30),), (10,), [100]),
            ((slice(0, 40, 3), slice(2, 40, 1)), (10, 12), [40, 40]),
            ((slice(4, 5, 1), slice(0, 10, 1), slice(17, 33, 2)), (2, 5, 8), [10, 10, 40]),
            ((slice(0, 1024, 1), slice(0, 1024, 4)), (512, 512), [1024, 1024]),
            (((1, 4, 17), slice(2, 30, 3)), (10, 10), [20, 40])]
    for sel, layout, dims in sels:
        ids = cu.getChunkIds(dset_id, sel, layout)
        num = cu.getNumChunks(sel, layout)
        entry = {"selection": enc_sel(sel), "layout": list(layout), "dims": dims, "num_chunks": num,
                 "chunk_ids": ids}
        cov = []
        for cid in ids[:96]:
            cs = cu.getChunkSelection(cid, sel, layout)
            cc = cu.getChunkCoverage(cid, sel, layout)
            dc = cu.getDataCoverage(cid, sel, layout)
            cov.append({"chunk_id": cid, "chunk_sel": enc_sel(cs) if cs else None,
                        "chunk_cov": enc_sel(cc) if cc else None, "data_cov": enc_sel(dc),
                        "query": du.getSliceQueryParam(cc) if cc else None})
        entry["coverage"] = cov
        cases["getChunkIds"].append(entry)
    # pagination (dsetUtil.py:689-800)
    for sel, itemsize, maxreq in (((slice(0, 131072, 1), slice(0, 131072, 1)), 4, 100 * 1024 * 1024),
                                  ((slice(0, 1000, 3), slice(0, 50, 1)), 8, 10000),
                                  ((slice(5, 6, 1), slice(0, 100000, 1)), 4, 100000),
                                  (((1, 2, 3, 4, 5, 6, 7, 8), slice(0, 1000, 1)), 4, 9000),
                                  ((slice(0, 10, 1),), 4, 1000)):
        dims = [s.stop if isinstance(s, slice) else 100 for s in sel]
        try:
            pages = du.getSelectionPagination(sel, dims, itemsize, maxreq)
            cases["pagination"].append({"selection": enc_sel(sel), "dims": dims, "itemsize": itemsize,
                                        "max_request_size": maxreq, "pages": [enc_sel(p) for p in pages]})
        except ValueError as e:
            cases["pagination"].append({"selection": enc_sel(sel), "dims": dims, "itemsize": itemsize,
                                        "max_request_size": maxreq, "error": str(e)})
    # md5 partition (idUtil.py:481-486) and storage keys (idUtil.py:174-251)
    for i in range(64):
        cid = f"c-{dset_id[2:]}_{i // 8}_{i % 8}"
        cases["partition"].append({"id": cid, "p8": iu.getObjPartition(cid, 8), "p4": iu.getObjPartition(cid, 4),
                                   "p2": iu.getObjPartition(cid, 2), "p3": iu.getObjPartition(cid, 3)})
    for cid in (f"c-{dset_id[2:]}_0_0", f"c-{dset_id[2:]}_12_7_3", f"c5-{dset_id[2:]}_1_2"):
        cases["s3key"].append({"id": cid, "key": iu.getS3Key(cid)})
    # chunkReadSelection / chunkWriteSelection (chunkUtil.py:882-995)
    rng = np.random.default_rng(99)
    for shape, dt, sl in (((16, 64, 128), "<i2", (slice(1, 16, 2), slice(3, 64, 5), slice(1, 128, 3))),
                          ((512, 512), "<f4", (slice(0, 512, 4), slice(0, 512, 4))),
                          ((10, 12), "<f8", (slice(2, 9, 1), slice(0, 12, 5))),
                          ((7,), "|u1", (slice(0, 7, 1),))):
        arr = (rng.integers(-1000, 1000, size=shape)).astype(dt)
        out = cu.chunkReadSelection(arr, slices=sl)
        cases["readSelection"].append({"shape": list(shape), "dtype": dt, "seed": 99,
                                       "slices": enc_sel(sl), "out_shape": list(out.shape),
                                       "out_sha256": sha(out.tobytes())})
        data = (rng.integers(-1000, 1000, size=out.shape)).astype(dt)
        a2 = arr.copy()
        upd = cu.chunkWriteSelection(chunk_arr=a2, slices=sl, data=data)
        upd2 = cu.chunkWriteSelection(chunk_arr=a2, slices=sl, data=data)
        cases["writeSelection"].append({"shape": list(shape), "dtype": dt, "slices": enc_sel(sl),
                                        "updated": bool(upd), "updated_again": bool(upd2),
                                        "out_sha256": sha(a2.tobytes())})
    with open(os.path.join(HERE, "selection_cases.json"), "w") as f:
        json.dump(cases, f, indent=0)


if __name__ == "__main__":
    main()
