"""Golden vectors for the bitshuffle+LZ4 chunk format (shuffle=2).

Run in the build container with the image's conda Python (imagecodecs lives there):
    env -u PYTHONPATH -u PYTHONHOME /opt/conda/bin/python3.9 tests/golden/make_bitshuffle_golden.py

The reference writes a bitshuffle chunk in storUtil._shuffle (storUtil.py:103-131):
bitshuffle.compress_lz4(arr, block_size) behind a 12-byte header (u64 BE chunk bytes,
u32 BE block_size * itemsize); storUtil._unshuffle (storUtil.py:144-174) checks the
header and calls bitshuffle.decompress_lz4.  bitshuffle 0.5.2 is not in the image.
What pins these vectors:
  * the bit transposition comes from the bitshuffle C core that imagecodecs 2021.8.26
    vendors (bitshuffle 0.3.5: bshuf_bitshuffle, the same transposition 0.5.2 keeps
    stable for HDF5 files); the script checks imagecodecs' blocked layout against the
    per-block composition below;
  * each block's LZ4 block comes from the image's liblz4 1.9.3 LZ4_compress_default,
    the call bshuf_compress_lz4_block makes;
  * the framing (per block: u32 BE compressed size + LZ4 block; a last block of the
    remaining elements rounded down to a multiple of 8; the size % 8 leftover elements
    copied raw) is bitshuffle's published bshuf_compress_lz4 layout, restated here.
Every case's expected result (bytes, or HTTPInternalServerError) comes from ref_decode:
_unshuffle's checks with decompress_lz4's block walk over liblz4's LZ4_decompress_safe
and imagecodecs' inverse transposition.  A corrupted LZ4 byte may still decode.

Outputs: bitshuffle_cases.npz (arrays <name>__in, <name>__raw) / bitshuffle_cases.json.
"""
import ctypes
import hashlib
import json
import os
import struct

import numpy as np
from imagecodecs import _bitshuffle as ibs

HERE = os.path.dirname(os.path.abspath(__file__))
LZ4 = ctypes.CDLL("/opt/conda/lib/liblz4.so.1")
LZ4.LZ4_compressBound.restype = ctypes.c_int
LZ4.LZ4_compress_default.restype = ctypes.c_int
LZ4.LZ4_compress_default.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
LZ4.LZ4_decompress_safe.restype = ctypes.c_int
LZ4.LZ4_decompress_safe.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]


def lz4_block(b):
    src = np.frombuffer(b, np.uint8).copy() if len(b) else np.zeros(1, np.uint8)
    cap = LZ4.LZ4_compressBound(len(b))
    out = np.zeros(max(cap, 1), np.uint8)
    n = LZ4.LZ4_compress_default(src.ctypes.data, out.ctypes.data, len(b), cap)
    assert n > 0
    return out[:n].tobytes()


def default_block(es):
    # bshuf_default_block_size: 8192-byte target, multiple of 8, at least 128 elements
    bs = (8192 // es) // 8 * 8
    return max(bs, 128)


def transpose(arr):
    """bshuf_trans_bit_elem of one block (element count a multiple of 8)"""
    return ibs.bitshuffle_encode(arr, blocksize=arr.size).tobytes()


def compress_lz4(arr, block):
    """bitshuffle.compress_lz4(arr, block) composed from the transposition + liblz4"""
    flat = arr.reshape(-1)
    es, n = flat.dtype.itemsize, flat.size
    bs = block if block else default_block(es)
    out = bytearray()
    tpos = 0
    ref = ibs.bitshuffle_encode(flat, blocksize=bs).tobytes()   # imagecodecs' blocked layout
    for i in range(n // bs):
        t = transpose(flat[i * bs:(i + 1) * bs])
        assert t == ref[tpos:tpos + len(t)]
        tpos += len(t)
        c = lz4_block(t)
        out += struct.pack(">I", len(c)) + c
    last = (n % bs) - (n % bs) % 8
    if last:
        s = (n // bs) * bs
        t = transpose(flat[s:s + last])
        assert t == ref[tpos:tpos + len(t)]
        tpos += len(t)
        c = lz4_block(t)
        out += struct.pack(">I", len(c)) + c
    left = flat[n - n % 8:].tobytes()
    assert left == ref[tpos:]
    out += left
    return bytes(out)


def ref_decode(blob, chunk_bytes, dtype):
    """storUtil._unshuffle(codec=2) (storUtil.py:144-174) over the image's libraries:
    bitshuffle.decompress_lz4's block walk with liblz4's LZ4_decompress_safe and
    imagecodecs' bitshuffle core for the inverse transposition.  Returns bytes or None
    (HTTPInternalServerError)."""
    es = dtype.itemsize
    if len(blob) < 12:
        return None
    if int.from_bytes(blob[:8], "big") != chunk_bytes:
        return None
    bs = int.from_bytes(blob[8:12], "big") // es
    if bs == 0:
        bs = default_block(es)
    if bs % 8:
        return None
    n = chunk_bytes // es
    out = bytearray()
    p, e = 12, 0
    while e + 8 <= n:
        cnt = bs if n - e >= bs else (n - e) // 8 * 8
        if p + 4 > len(blob):
            return None
        nb = int.from_bytes(blob[p:p + 4], "big")
        p += 4
        if nb > len(blob) - p or nb >= 1 << 31:
            return None
        src = np.frombuffer(blob[p:p + nb], np.uint8).copy() if nb else np.zeros(1, np.uint8)
        dst = np.zeros(cnt * es + 1, np.uint8)
        r = LZ4.LZ4_decompress_safe(src.ctypes.data, dst.ctypes.data, nb, cnt * es)
        if r != cnt * es:
            return None
        t = np.frombuffer(dst[:cnt * es].tobytes(), dtype)
        out += ibs.bitshuffle_decode(t, blocksize=cnt, out=np.empty_like(t)).tobytes()
        p += nb
        e += cnt
    left = (n - e) * es
    if p + left > len(blob):
        return None
    out += blob[p:p + left]
    p += left
    if p != len(blob):          # decompress_lz4: consumed bytes != input size
        return None
    return bytes(out)


def hsds_frame(arr, block):
    """storUtil._shuffle(codec=2) (storUtil.py:103-131)"""
    es = arr.dtype.itemsize
    return struct.pack(">Q", arr.size * es) + struct.pack(">I", block * es) + compress_lz4(arr, block)


def data(kind, n, dtype, seed):
    rng = np.random.default_rng(seed)
    dt = np.dtype(dtype)
    if kind == "smooth" and dt.kind == "f":
        return (np.cumsum(rng.standard_normal(n)) * 0.01).astype(dt)
    if kind == "smooth" and dt.kind in "iu":
        return (np.arange(n) // 7 + 3).astype(dt)
    return np.frombuffer(rng.integers(0, 256, n * dt.itemsize, dtype=np.uint8).tobytes(), dt).copy()


def main():
    cases = []
    arrays = {}

    def add(name, raw, blob, block, note=""):
        want = ref_decode(blob, len(raw), raw_dtype[name])
        arrays[name + "__in"] = np.frombuffer(blob, np.uint8)
        arrays[name + "__raw"] = np.frombuffer(raw, np.uint8)
        cases.append({"name": name, "itemsize": int(raw_dtype[name].itemsize), "nbytes": len(raw),
                      "block": block, "status": "ok" if want is not None else "error", "in_len": len(blob),
                      "raw_sha256": hashlib.sha256(raw).hexdigest(),
                      "out_sha256": hashlib.sha256(want).hexdigest() if want is not None else None,
                      "note": note})
        return want

    raw_dtype = {}
    specs = [
        ("f4_1MiB_b2048", "smooth", 262144, "<f4", 2048),      # the HSDS default block (config)
        ("f4_1MiB_rand_b2048", "rand", 262144, "<f4", 2048),
        ("u1_1000_b2048", "smooth", 1000, "u1", 2048),         # one partial block only
        ("i2_1003_b256", "smooth", 1003, "<i2", 256),          # full + last + 3 leftover
        ("f8_777_b64", "smooth", 777, "<f8", 64),
        ("u4_5_b2048", "smooth", 5, "<u4", 2048),              # leftover only
        ("f4_4096_b0", "smooth", 4096, "<f4", 0),              # header block 0: default block
        ("c16_100_b16", "rand", 100, "<c16", 16),
        ("s3_999_b128", "rand", 999, "S3", 128),               # 3-byte elements
        ("i8_65536_b2048", "smooth", 65536, "<i8", 2048),
        ("u2_131072_b8", "smooth", 131072, "<u2", 8),          # many tiny blocks
        ("f4_262143_b2048", "smooth", 262143, "<f4", 2048),    # ragged tail
    ]
    for k, (name, kind, n, dt, block) in enumerate(specs):
        a = data(kind, n, dt, 100 + k)
        raw = a.tobytes()
        raw_dtype[name] = a.dtype
        blob = hsds_frame(a, block)
        if block == 0:
            # the header carries block 0; bitshuffle then uses its default block
            blob = blob[:8] + struct.pack(">I", 0) + blob[12:]
        assert add(name, raw, blob, block) == raw
        # imagecodecs' own decoder agrees on the transposition
        dec = ibs.bitshuffle_decode(ibs.bitshuffle_encode(a, blocksize=block if block else 0),
                                    blocksize=block if block else 0, out=np.empty_like(a))
        assert dec.tobytes() == raw

    # corrupted frames
    base = arrays["i2_1003_b256__in"].tobytes()
    raw = arrays["i2_1003_b256__raw"].tobytes()
    bad = {
        "bad_total": struct.pack(">Q", len(raw) + 2) + base[8:],             # storUtil.py:160-164
        "bad_short_header": base[:11],                                        # storUtil.py:148-152
        "bad_block_not_mult8": base[:8] + struct.pack(">I", 2 * 100) + base[12:],
        "bad_trunc": base[:len(base) // 2],
        "bad_trailing": base + b"\x00\x01",
        "bad_lz4_size": base[:12] + struct.pack(">I", 0x7FFFFFF0) + base[16:],
    }
    p = 12 + 4 + 5
    corrupt = bytearray(base)
    corrupt[p] ^= 0xFF
    bad["bad_lz4_bytes"] = bytes(corrupt)
    for name, blob in bad.items():
        raw_dtype[name] = np.dtype("<i2")
        add(name, raw, blob, 256)
    np.savez_compressed(os.path.join(HERE, "bitshuffle_cases.npz"), **arrays)
    meta = {"generator": "tests/golden/make_bitshuffle_golden.py",
            "bitshuffle_core": ibs.bitshuffle_version(), "lz4": "liblz4 1.9.3 (/opt/conda/lib)",
            "cases": cases}
    with open(os.path.join(HERE, "bitshuffle_cases.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(len(cases), "cases")


if __name__ == "__main__":
    main()
