"""Golden vectors for the Blosc inner codecs other than zlib:
lz4, lz4hc, blosclz (decoded by the engine) and zstd (recorded; outside the engine).

Run in the build container only (needs /root/reference and /opt/conda/lib/libblosc.so.1):
    python tests/golden/make_codec2_golden.py

Every expected output comes from the reference's own code: getFilterOps
(dsetUtil.py:159-212) turns an HDF5 filter list into filter ops, storUtil._compress
(storUtil.py:238-281) writes the object with Blosc(cname=<compressor>), and
storUtil._uncompress (storUtil.py:182-235) decodes it, with numcodecs re-expressed over
c-blosc 1.21.0 (tests/golden/refshim.py).  Frames with typesize > 1 (as an HDF5 Blosc
filter writes them for linked chunks) come from libblosc directly and are decoded by the
reference's _uncompress.  Corrupted frames record whatever the reference returns.

Outputs: codec2_cases.npz / codec2_cases.json (same schema as codec_cases.*).
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refshim  # noqa: E402

from hsds.util import storUtil as su  # noqa: E402
from hsds.util.dsetUtil import getFilterOps  # noqa: E402

BIG = 64 * 1024
FILTER = {"lz4": ("H5Z_FILTER_LZ4", 32004), "lz4hc": ("H5Z_FILTER_LZ4HC", 32005),
          "blosclz": ("H5Z_FILTER_BLOSC", 32001), "zstd": ("H5Z_FILTER_ZSTD", 32015)}


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def data(kind, n, dtype, seed):
    rng = np.random.default_rng(seed)
    dt = np.dtype(dtype)
    if kind == "smooth":
        if dt.kind in "iu":
            return (np.cumsum(rng.normal(size=n)) * 100).astype(dt)
        return np.round(np.cumsum(rng.normal(size=n)), 2).astype(dt)
    if kind == "steps":      # long runs: long matches, overlapping copies
        return np.repeat(rng.integers(0, 50, n // 97 + 1), 97)[:n].astype(dt)
    if kind == "text":
        t = np.frombuffer((b"hsds chunk %d; the quick brown fox jumps over the lazy dog. " * (n // 40 + 2))[:n * dt.itemsize], np.uint8)
        return t.view(dt)[:n]
    if kind == "zeros":
        return np.zeros(n, dt)
    if kind == "lowent":     # 4 symbols: short matches everywhere
        return rng.integers(0, 4, n).astype(dt)
    raise ValueError(kind)


def main():
    arrays, cases = {}, []

    def run_uncompress(blob, ops):
        try:
            return su._uncompress(blob, **ops)
        except Exception as e:
            return e

    def add(name, blob, ops, note, seed=None, raw=None):
        out = run_uncompress(blob, ops)
        case = {"name": name, "note": note, "seed": seed, "compressor": ops.get("compressor"),
                "shuffle": ops.get("shuffle", 0), "level": ops.get("level"),
                "dtype": np.dtype(ops["dtype"]).str if ops.get("dtype") is not None else None,
                "chunk_shape": list(ops["chunk_shape"]) if ops.get("chunk_shape") is not None else None,
                "in_len": len(blob), "codec": int(blob[2] >> 5) if len(blob) >= 16 else None,
                "memcpyed": bool(blob[2] & 2) if len(blob) >= 16 else None}
        arrays[name + "__in"] = np.frombuffer(blob, np.uint8)
        if isinstance(out, Exception):
            case["status"], case["error"] = "error", type(out).__name__
        else:
            case["status"], case["out_len"], case["out_sha256"] = "ok", len(out), sha(out)
            if raw is not None:
                assert raw == out, name
            if len(out) <= BIG:
                arrays[name + "__out"] = np.frombuffer(out, np.uint8)
        cases.append(case)

    app = {"filter_map": {}}
    seed = 900
    # ---- HSDS-written objects: reference getFilterOps + _compress (typesize 1)
    for comp in ("lz4", "lz4hc", "blosclz", "zstd"):
        for kind, dt, shape, level, shuf in (("smooth", "<f4", (512, 512), 5, 1), ("smooth", "<f4", (256, 256), 9, 1),
                                             ("smooth", "<i2", (16, 64, 128), 5, 1), ("steps", "<i4", (300, 301), 5, 0),
                                             ("text", "|u1", (100003,), 1, 0), ("zeros", "<f8", (8192,), 5, 1),
                                             ("lowent", "|u1", (70001,), 3, 0), ("lowent", "|u1", (200,), 5, 0)):
            seed += 1
            arr = data(kind, int(np.prod(shape)), dt, seed).reshape(shape)
            f = [{"class": "H5Z_FILTER_SHUFFLE", "id": 2, "name": "shuffle"}] if shuf else []
            cls, fid = FILTER[comp]
            f.append({"class": cls, "id": fid, "level": level, "name": comp})
            ops = getFilterOps(app, f"d-{comp}-{seed}", f, dtype=arr.dtype, chunk_shape=shape)
            app["filter_map"].clear()
            blob = su._compress(arr.tobytes(), **ops)
            add(f"{comp}_{kind}_{np.dtype(dt).name}_{'x'.join(map(str, shape))}_L{level}", blob, ops,
                "reference getFilterOps + _compress -> _uncompress", seed, arr.tobytes())
    # ---- zstd at every level (block types, literal modes and table modes vary)
    for level in range(1, 10):
        for kind, dt, shape in (("smooth", "<f4", (256, 512)), ("lowent", "|u1", (150000,)), ("steps", "<i2", (70000,))):
            seed += 1
            arr = data(kind, int(np.prod(shape)), dt, seed).reshape(shape)
            f = [{"class": "H5Z_FILTER_SHUFFLE", "id": 2, "name": "shuffle"},
                 {"class": "H5Z_FILTER_ZSTD", "id": 32015, "level": level, "name": "zstd"}]
            ops = getFilterOps(app, f"d-zstd-{seed}", f, dtype=arr.dtype, chunk_shape=shape)
            app["filter_map"].clear()
            blob = su._compress(arr.tobytes(), **ops)
            add(f"zstd_L{level}_{kind}_{np.dtype(dt).name}", blob, ops, "reference getFilterOps + _compress -> _uncompress",
                seed, arr.tobytes())
    # ---- frames with typesize > 1 and in-frame shuffle (HDF5 Blosc filter writers)
    for comp in ("lz4", "lz4hc", "blosclz", "zstd"):
        for kind, dt, n, level in (("smooth", "<f4", 65536, 5), ("smooth", "<i2", 131072, 9), ("smooth", "<f8", 40000, 5),
                                   ("steps", "<i4", 262144 + 333, 5), ("lowent", "<f4", 8192 + 3, 5)):
            seed += 1
            arr = data(kind, n, dt, seed)
            raw = arr.tobytes()
            blob = refshim.blosc_compress_raw(raw, level, 1, arr.dtype.itemsize, cname=comp)
            ops = {"compressor": comp, "shuffle": 1, "level": level, "dtype": arr.dtype, "chunk_shape": (n,)}
            add(f"{comp}_ts{arr.dtype.itemsize}_{kind}_{n}_L{level}", blob, ops,
                "libblosc typesize>1 frame -> reference _uncompress", seed, raw)
    # ---- corrupted frames: whatever the reference does (error, or decoded bytes)
    rng = np.random.default_rng(77)
    for comp, kind in (("lz4", "lowent"), ("blosclz", "steps"), ("zstd", "lowent"), ("zstd", "text")):
        arr = data(kind, 65536, "|u1", 4242)
        ops = {"compressor": comp, "shuffle": 0, "level": 5, "dtype": np.dtype("u1"), "chunk_shape": (65536,)}
        good = su._compress(arr.tobytes(), **ops)
        assert not good[2] & 2
        for k in range(8):
            bad = bytearray(good)
            pos = int(rng.integers(40, len(bad)))
            bad[pos] ^= int(rng.integers(1, 256))
            add(f"err_{comp}_{kind}_flip{k}", bytes(bad), ops, f"byte {pos} corrupted")
        # c-blosc 1.21 blosc_decompress takes no source size and reads past the end of a
        # truncated object; the engine rejects it (header cbytes > object length)
        add(f"err_{comp}_{kind}_trunc", good[:-7], ops, "truncated frame: reference reads past the object end")
    # ---- c-blosc 1.21 frame header fields per codec (compute_blocksize, split flag)
    hdr = []
    base = data("smooth", 1 << 20, "<i4", 5).tobytes()
    for cname in ("lz4", "lz4hc", "blosclz", "zlib"):
        for lv in range(10):
            for ts in (1, 2, 4, 8, 16, 32):
                for nb in (1 << 22, 1 << 20, 262144, 100000, 40000, 32768, 5000, 100):
                    f = refshim.blosc_compress_raw(base[:nb], lv, 1, ts, cname=cname)
                    hdr.append({"cname": cname, "clevel": lv, "typesize": ts, "nbytes": nb, "flags": f[2],
                                "blocksize": int(np.frombuffer(f[8:12], "<u4")[0])})
    np.savez_compressed(os.path.join(HERE, "codec2_cases.npz"), **arrays)
    with open(os.path.join(HERE, "codec2_cases.json"), "w") as fh:
        json.dump({"cases": cases, "headers": hdr}, fh, indent=1)
    print("wrote", len(cases), "cases;", sum(c["status"] == "error" for c in cases), "errors")


if __name__ == "__main__":
    main()
