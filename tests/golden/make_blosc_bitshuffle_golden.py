"""Golden vectors for Blosc frames carrying the bitshuffle flag (0x04), as HDF5 Blosc-filter
writers produce them (Blosc(shuffle=BITSHUFFLE)); HSDS reads them through
storUtil._uncompress -> numcodecs Blosc().decode (storUtil.py:195-208).

Run in the build container only (needs /root/reference and /opt/conda/lib/libblosc.so.1):
    python tests/golden/make_blosc_bitshuffle_golden.py

Frames come from libblosc 1.21.0 itself (blosc_compress_ctx with doshuffle = 2), plus
hand-built frames with stored (raw) splits that pin the block rules the writer never
exercises on its own (a block whose element count is not a multiple of 8 stays as
decoded; tail bytes past the last whole element; typesize 1).  Every expected output is
the reference's _uncompress of the frame, with numcodecs re-expressed over c-blosc 1.21.0
(tests/golden/refshim.py).

Outputs: blosc_bitshuffle_cases.npz / blosc_bitshuffle_cases.json.
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

BIG = 64 * 1024


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def data(kind, n, dtype, seed):
    rng = np.random.default_rng(seed)
    dt = np.dtype(dtype)
    if kind == "smooth":
        if dt.kind in "iu":
            return (np.cumsum(rng.normal(size=n)) * 100).astype(dt)
        return np.round(np.cumsum(rng.normal(size=n)), 2).astype(dt)
    if kind == "steps":
        return np.repeat(rng.integers(0, 50, n // 97 + 1), 97)[:n].astype(dt)
    if kind == "random":
        return rng.integers(0, 256, n * dt.itemsize, dtype=np.uint8).view(dt)[:n]
    raise ValueError(kind)


def raw_frame(ts, blocks, nbytes, bs, flags):
    """Blosc1 frame (version 2) whose blocks are lists of stored splits."""
    hdr = 16 + 4 * len(blocks)
    body, starts = b"", []
    for splits in blocks:
        starts.append(hdr + len(body))
        for sp in splits:
            body += len(sp).to_bytes(4, "little") + sp
    f = bytes([2, 1, flags, ts]) + nbytes.to_bytes(4, "little") + bs.to_bytes(4, "little")
    f += (hdr + len(body)).to_bytes(4, "little")
    return f + b"".join(x.to_bytes(4, "little") for x in starts) + body


def main():
    arrays, cases = {}, []

    def add(name, blob, ops, note, raw=None):
        try:
            out = su._uncompress(blob, **ops)
        except Exception as e:
            out = e
        case = {"name": name, "note": note, "compressor": ops["compressor"], "shuffle": ops.get("shuffle", 0),
                "dtype": np.dtype(ops["dtype"]).str, "chunk_shape": list(ops["chunk_shape"]), "in_len": len(blob),
                "flags": int(blob[2]), "typesize": int(blob[3])}
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

    seed = 3100
    # ---- libblosc-written BITSHUFFLE frames: every codec, typesizes 1-16
    for comp in ("zlib", "lz4", "blosclz", "zstd"):
        for kind, dt, n, level, bsz in (("smooth", "<f4", 65536, 5, 0), ("smooth", "<i2", 131072 + 5, 9, 0),
                                        ("smooth", "<f8", 40000, 4, 0), ("steps", "<i4", 70001, 5, 16384),
                                        ("random", "|u1", 50000, 5, 0), ("smooth", "<f4", 30000 + 3, 1, 4096),
                                        ("smooth", "<c16", 4000, 5, 0)):
            seed += 1
            arr = data(kind, n, dt, seed) if dt != "<c16" else data("smooth", 2 * n, "<f8", seed).view("<c16")
            raw = arr.tobytes()
            ts = arr.dtype.itemsize
            blob = refshim.blosc_compress_raw(raw, level, 2, ts, cname=comp, blocksize=bsz)
            assert blob[2] & 0x04 or blob[2] & 0x02, (comp, blob[2])
            ops = {"compressor": comp, "shuffle": 0, "level": level, "dtype": arr.dtype, "chunk_shape": (n,)}
            add(f"{comp}_bit_ts{ts}_{kind}_{n}_L{level}_bs{bsz}", blob, ops, "libblosc BITSHUFFLE frame -> _uncompress",
                raw)
    # ---- hand-built frames with stored splits: the decoder's block rules
    rng = np.random.default_rng(91)
    for ts, nel, bs, split in ((4, 1000, 0, False), (4, 1003, 0, False), (2, 1001, 0, False), (8, 1004, 0, False),
                               (1, 1000, 0, False), (1, 1005, 0, False), (3, 1000, 0, False), (4, 2000, 4000, False),
                               (4, 2000, 4000, True), (2, 4096, 2048, True)):
        nb = ts * nel
        bsz = bs or nb
        payload = rng.integers(0, 256, nb, dtype=np.uint8).tobytes()
        blocks = []
        for b0 in range(0, nb, bsz):
            blk = payload[b0:b0 + bsz]
            isleft = len(blk) < bsz
            nspl = ts if split and not isleft and ts <= 16 and bsz // ts >= 128 else 1
            ne = len(blk) // nspl
            blocks.append([blk[j * ne:(j + 1) * ne] for j in range(nspl)])
        flags = 0x04 | (0 if split else 0x10)
        blob = raw_frame(ts, blocks, nb, bsz, flags)
        ops = {"compressor": "blosclz", "shuffle": 0, "level": 5, "dtype": np.dtype("u1"), "chunk_shape": (nb,)}
        add(f"raw_bit_ts{ts}_n{nel}_bs{bsz}{'_split' if split else ''}", blob, ops, "hand-built stored-split frame")
    # tail bytes past the last whole element (nbytes not a multiple of ts)
    payload = rng.integers(0, 256, 4003, dtype=np.uint8).tobytes()
    add("raw_bit_ts4_tail3", raw_frame(4, [[payload]], 4003, 4003, 0x14),
        {"compressor": "blosclz", "shuffle": 0, "level": 5, "dtype": np.dtype("u1"), "chunk_shape": (4003,)},
        "hand-built frame, 3 tail bytes")
    # byte shuffle wins over the bit flag when both are set (typesize > 1)
    payload = rng.integers(0, 256, 4000, dtype=np.uint8).tobytes()
    add("raw_bytebit_ts4", raw_frame(4, [[payload]], 4000, 4000, 0x15),
        {"compressor": "blosclz", "shuffle": 0, "level": 5, "dtype": np.dtype("u1"), "chunk_shape": (4000,)},
        "hand-built frame, flags 0x01 | 0x04")
    np.savez_compressed(os.path.join(HERE, "blosc_bitshuffle_cases.npz"), **arrays)
    with open(os.path.join(HERE, "blosc_bitshuffle_cases.json"), "w") as fh:
        json.dump({"cases": cases}, fh, indent=1)
    print("wrote", len(cases), "cases;", sum(c["status"] == "error" for c in cases), "errors")


if __name__ == "__main__":
    main()
