"""ctypes wrapper around oracle/liboracle.so -- the CPU restatement of HSDS's
chunk codec (see oracle.c for the reference file:line each function follows).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  The product package (hsds_amd) never imports it.

Selection copies (chunkReadSelection / chunkWriteSelection / the SN slab scatter,
hsds/util/chunkUtil.py:882-995, hsds/chunk_crawl.py:418) are numpy slicing in the
reference; the oracle for those is numpy slicing itself (`select_gather`,
`select_scatter` below).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

OK = 0
ERR_FRAME = -1
ERR_DATA = -2
ERR_TRUNC = -3
ERR_SIZE = -4
ERR_UNSUPPORTED = -5
ERR_ARG = -6

_lib = None


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P, I64, I = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        L.orc_zlib_decode.argtypes = [P, I64, P, I64]
        L.orc_zlib_decode.restype = I64
        L.orc_lz4_decode.argtypes = [P, I64, P, I64]
        L.orc_lz4_decode.restype = I64
        L.orc_zstd_decode.argtypes = [P, I64, P, I64]
        L.orc_zstd_decode.restype = I64
        L.orc_blosclz_decode.argtypes = [P, I64, P, I64]
        L.orc_blosclz_decode.restype = I64
        L.orc_blosc_decode.argtypes = [P, I64, P, I64]
        L.orc_blosc_decode.restype = I64
        L.orc_is_blosc.argtypes = [P, I64]
        L.orc_is_blosc.restype = I
        L.orc_uncompress.argtypes = [P, I64, I, I, I, P, I64]
        L.orc_uncompress.restype = I64
        L.orc_blosc_encode_zlib.argtypes = [P, I64, I, I, I, P, I64]
        L.orc_blosc_encode_zlib.restype = I64
        L.orc_blosc_encode_lz4.argtypes = [P, I64, I, I64, I, P, I64]
        L.orc_blosc_encode_lz4.restype = I64
        L.orc_lz4_encode.argtypes = [P, I64, P, I64]
        L.orc_lz4_encode.restype = I64
        L.orc_blosc_blocksize_codec.argtypes = [I, I, I64, I]
        L.orc_blosc_blocksize_codec.restype = I64
        L.orc_blosc_blocksize.argtypes = [I, I, I64]
        L.orc_blosc_blocksize.restype = I64
        L.orc_zlib_encode.argtypes = [P, I64, I, P, I64]
        L.orc_zlib_encode.restype = I64
        L.orc_shuffle.argtypes = [P, I64, I, P]
        L.orc_unshuffle.argtypes = [P, I64, I, P]
        L.orc_adler32.argtypes = [P, I64]
        L.orc_adler32.restype = ctypes.c_uint32
        L.orc_bitshuffle_decode.argtypes = [P, I64, P, I64, I64]
        L.orc_bitshuffle_decode.restype = I64
        L.orc_bitshuffle_encode.argtypes = [P, I64, I64, I64, P, I64]
        L.orc_bitshuffle_encode.restype = I64
        L.orc_bshuf_trans.argtypes = [P, P, I64, I64]
        L.orc_bshuf_untrans.argtypes = [P, P, I64, I64]
        L.orc_uncompress_batch.argtypes = [P, P, P, P, I64, I, I, I, I, P]
        L.orc_encode_batch.argtypes = [I, P, P, P, P, I64, I, I, I, I, P]
        _lib = L
    return _lib


def _u8(b):
    return np.frombuffer(b, dtype=np.uint8) if not isinstance(b, np.ndarray) else b.view(np.uint8).reshape(-1)


def compressor_code(compressor):
    """storUtil._uncompress compressor argument -> oracle code."""
    if not compressor or compressor == "scaleoffset":
        return 0
    if compressor in ("gzip", "deflate", "zlib"):
        return 1
    return 2


def zlib_decode(data, cap):
    s = _u8(data)
    out = np.empty(max(cap, 1), np.uint8)
    n = lib().orc_zlib_decode(s.ctypes.data, s.size, out.ctypes.data, cap)
    return n if n < 0 else out[:n].tobytes()


def _split_decode(fn, data, n):
    """one Blosc split: exactly n bytes (c-blosc rejects any other size) or a status"""
    s = _u8(data)
    if s.size == 0:
        s = np.zeros(1, np.uint8)[:0]
    out = np.empty(max(n, 1), np.uint8)
    r = fn(s.ctypes.data, len(data), out.ctypes.data, n)
    if r < 0:
        return r
    return out[:n].tobytes() if r == n else ERR_SIZE


def lz4_decode(data, n):
    return _split_decode(lib().orc_lz4_decode, data, n)


def zstd_decode(data, n):
    return _split_decode(lib().orc_zstd_decode, data, n)


def blosclz_decode(data, n):
    return _split_decode(lib().orc_blosclz_decode, data, n)


def blosc_decode(data, cap):
    s = _u8(data)
    out = np.empty(max(cap, 1), np.uint8)
    n = lib().orc_blosc_decode(s.ctypes.data, s.size, out.ctypes.data, cap)
    return n if n < 0 else out[:n].tobytes()


def is_blosc(data):
    s = _u8(data)
    return bool(lib().orc_is_blosc(s.ctypes.data, s.size))


def uncompress(data, compressor=None, shuffle=0, itemsize=1, expected=None):
    """_uncompress restatement; returns bytes, or a negative status int."""
    s = _u8(data)
    if expected is None:
        raise ValueError("expected output size required")
    out = np.empty(max(expected, 1), np.uint8)
    n = lib().orc_uncompress(s.ctypes.data, s.size, compressor_code(compressor), int(shuffle),
                             int(itemsize), out.ctypes.data, expected)
    return n if n < 0 else out[:n].tobytes()


def blosc_encode(data, typesize=1, clevel=5, shuffle=1):
    """numcodecs Blosc(cname='zlib', clevel, shuffle).encode(buf) with buf itemsize = typesize."""
    s = _u8(data)
    out = np.empty(s.size + 16, np.uint8)
    n = lib().orc_blosc_encode_zlib(s.ctypes.data, s.size, typesize, clevel, shuffle,
                                    out.ctypes.data, out.size)
    if n < 0:
        raise RuntimeError(f"blosc encode error {n}")
    return out[:n].tobytes()


def blosc_encode_lz4(data, typesize=1, blocksize=131072, shuffle=1):
    """Blosc1 frame with LZ4 splits (corpus writer for lz4 tests and the bench)."""
    s = _u8(data)
    out = np.empty(s.size + 16, np.uint8)
    n = lib().orc_blosc_encode_lz4(s.ctypes.data, s.size, typesize, blocksize, shuffle, out.ctypes.data, out.size)
    if n < 0:
        raise RuntimeError(f"blosc lz4 encode error {n}")
    return out[:n].tobytes()


def lz4_encode(data):
    s = _u8(data)
    out = np.empty(s.size + s.size // 255 + 64, np.uint8)
    n = lib().orc_lz4_encode(s.ctypes.data, s.size, out.ctypes.data, out.size)
    if n < 0:
        raise RuntimeError(f"lz4 encode error {n}")
    return out[:n].tobytes()


def blosc_blocksize_codec(clevel, typesize, nbytes, cname):
    """c-blosc 1.21 compute_blocksize for cname (zlib / lz4hc / zstd are HCR codecs)"""
    return lib().orc_blosc_blocksize_codec(clevel, typesize, nbytes, 0 if cname in ("lz4", "blosclz") else 1)


def blosc_blocksize(clevel, typesize, nbytes):
    return lib().orc_blosc_blocksize(clevel, typesize, nbytes)


def zlib_encode(data, level):
    s = _u8(data)
    cap = s.size + s.size // 100 + 1024
    out = np.empty(cap, np.uint8)
    n = lib().orc_zlib_encode(s.ctypes.data, s.size, level, out.ctypes.data, cap)
    if n < 0:
        raise RuntimeError("zlib encode error")
    return out[:n].tobytes()


def shuffle(data, n):
    s = _u8(data)
    out = np.empty(s.size, np.uint8)
    lib().orc_shuffle(s.ctypes.data, s.size, n, out.ctypes.data)
    return out.tobytes()


def unshuffle(data, n):
    s = _u8(data)
    out = np.empty(s.size, np.uint8)
    lib().orc_unshuffle(s.ctypes.data, s.size, n, out.ctypes.data)
    return out.tobytes()


def adler32(data):
    s = _u8(data)
    return int(lib().orc_adler32(s.ctypes.data, s.size))


def _ptr_array(arrs):
    return np.array([a.ctypes.data for a in arrs], dtype=np.uint64)


def uncompress_batch(blobs, expected, compressor="zlib", shuffle=0, itemsize=1, nthreads=1,
                     out=None):
    """Threaded _uncompress over many chunks (bench cpu_baseline). blobs: list of uint8 arrays."""
    n = len(blobs)
    if out is None:
        out = [np.empty(e, np.uint8) for e in expected]
    srcp = _ptr_array(blobs)
    dstp = _ptr_array(out)
    lens = np.array([b.size for b in blobs], np.int64)
    exp = np.array(expected, np.int64)
    status = np.zeros(n, np.int64)
    lib().orc_uncompress_batch(srcp.ctypes.data, lens.ctypes.data, dstp.ctypes.data, exp.ctypes.data,
                               n, compressor_code(compressor), shuffle, itemsize, nthreads,
                               status.ctypes.data)
    return out, status


def encode_batch(chunks, op="blosc", typesize=1, clevel=4, shuffle=1, nthreads=1):
    """Threaded F1 (op='blosc') or F2 (op='zlib') encode of uint8 arrays; returns list of arrays."""
    n = len(chunks)
    caps = [c.size + c.size // 100 + 1024 for c in chunks]
    out = [np.empty(cap, np.uint8) for cap in caps]
    srcp = _ptr_array(chunks)
    dstp = _ptr_array(out)
    lens = np.array([c.size for c in chunks], np.int64)
    capa = np.array(caps, np.int64)
    status = np.zeros(n, np.int64)
    lib().orc_encode_batch(1 if op == "blosc" else 2, srcp.ctypes.data, lens.ctypes.data,
                           dstp.ctypes.data, capa.ctypes.data, n, typesize, clevel, shuffle,
                           nthreads, status.ctypes.data)
    if (status < 0).any():
        raise RuntimeError("encode error")
    return [o[:s] for o, s in zip(out, status)]


def select_gather(chunk_arr, slices):
    """chunkReadSelection (chunkUtil.py:909-927) for plain dtypes: chunk_arr[slices]."""
    return chunk_arr[tuple(slices)]


def select_scatter(arr, slices, data):
    """np_arr[data_sel] = chunk_arr (chunk_crawl.py:418) / chunkWriteSelection copy."""
    arr[tuple(slices)] = data
    return arr


# ---- bitshuffle + LZ4 (shuffle = 2; storUtil.py:103-131,144-174) ----

def bitshuffle_decode(data, chunk_bytes, itemsize):
    """storUtil._unshuffle(codec=2): the chunk bytes, or a negative status"""
    s = _u8(data)
    if s.size == 0:
        s = np.zeros(1, np.uint8)[:0]
    out = np.empty(max(chunk_bytes, 1), np.uint8)
    r = lib().orc_bitshuffle_decode(s.ctypes.data, s.size, out.ctypes.data, chunk_bytes, itemsize)
    return r if r < 0 else out[:chunk_bytes].tobytes()


def bitshuffle_encode(data, itemsize, block=2048):
    """storUtil._shuffle(codec=2) with block = config bit_shuffle_default_blocksize"""
    s = _u8(data)
    cap = s.size + s.size // 8 + 4 * (s.size // max(block * itemsize, 8) + 2) + 64
    out = np.empty(cap, np.uint8)
    n = lib().orc_bitshuffle_encode(s.ctypes.data, s.size, itemsize, block, out.ctypes.data, cap)
    if n < 0:
        raise ValueError(f"bitshuffle encode failed: {n}")
    return out[:n].tobytes()


def bshuf_trans(data, itemsize):
    s = _u8(data)
    out = np.empty(s.size, np.uint8)
    lib().orc_bshuf_trans(s.ctypes.data, out.ctypes.data, s.size // itemsize, itemsize)
    return out.tobytes()
