"""Drop-in mirror of the HSDS chunk-codec functions (hsds/util/storUtil.py:48-281).

Same names, argument meaning and error behaviour as the reference:
  * `_uncompress(data, compressor, shuffle, level, dtype, chunk_shape)` (storUtil.py:182)
    detects Blosc frames (cbuffer_metainfo typesize > 0, storUtil.py:195-196),
    decodes them (in-frame unshuffle, the external shuffle is then skipped,
    storUtil.py:203-204) or inflates a zlib stream (storUtil.py:209-220) and
    byte-unshuffles it (storUtil.py:225-226).  Any codec failure raises
    HTTPInternalServerError, an unknown shuffle code raises ValueError.
  * `_shuffle` / `_unshuffle` codec 1 = numcodecs.Shuffle(itemsize) (storUtil.py:94-143);
    `_unshuffle` codec 2 = bitshuffle+LZ4 behind HSDS's 12-byte header
    (storUtil.py:144-174), decoded by bshuf_kernel; `_shuffle` codec 2 writes it
    (storUtil.py:103-131) through the bitshuffle encode kernels.

All byte work runs on the MI355X through the C ABI (include/hsds_amd.h); there is
no CPU fallback.  The snappy codec raises NotImplementedError.
"""
import numpy as np

from . import _native as nat

try:  # the reference raises aiohttp's HTTP exceptions from the codec layer
    from aiohttp.web_exceptions import HTTPInternalServerError
except Exception:  # pragma: no cover - aiohttp is in the image
    class HTTPInternalServerError(Exception):
        pass

BYTE_SHUFFLE = 1
BIT_SHUFFLE = 2
# config bit_shuffle_default_blocksize (storUtil.py:110), elements per bitshuffle block
BIT_SHUFFLE_BLOCK = 2048


def getCompressors():
    """Compressor names this engine decodes (storUtil.getCompressors naming: zlib is
    reported as gzip, plus the deflate synonym, storUtil.py:52-66)."""
    return ["gzip", "deflate"]


def getSupportedFilters(include_compressors=True):
    filters = ["shuffle", "fletcher32", "nbit", "scaleoffset"]
    if include_compressors:
        filters.extend(getCompressors())
    return filters


def _compressor_code(compressor):
    if not compressor or compressor == "scaleoffset":
        return nat.COMP_NONE
    if compressor in ("gzip", "deflate", "zlib"):
        return nat.COMP_ZLIB
    return nat.COMP_OTHER


def _as_bytes(data):
    if isinstance(data, (bytes, bytearray, memoryview)):
        return np.frombuffer(data, dtype=np.uint8)
    return np.ascontiguousarray(data).view(np.uint8).reshape(-1)


def _itemsize(dtype):
    return 1 if dtype is None else np.dtype(dtype).itemsize


def _shuffle(codec, data, chunk_shape=None, dtype=None):
    """storUtil._shuffle (storUtil.py:94): codec 1 = byte shuffle."""
    if codec == BYTE_SHUFFLE:
        src = _as_bytes(data)
        out = np.empty(src.size, np.uint8)
        rc = nat.lib().hsds_shuffle(nat.engine().h, src.ctypes.data, src.size, _itemsize(dtype),
                                    out.ctypes.data)
        if rc != nat.OK:
            raise nat.NativeError(rc, "hsds_shuffle")
        return out.tobytes()
    if codec == BIT_SHUFFLE:
        # bitshuffle.compress_lz4 of data.reshape(chunk_shape) behind the 12-byte header
        # (storUtil.py:103-131); the reshape's ValueError on a size mismatch is kept
        itemsize = dtype.itemsize if isinstance(dtype, np.dtype) else np.dtype(dtype).itemsize \
            if dtype is not None else None.itemsize        # AttributeError without a dtype, as there
        chunk_size = int(np.prod(chunk_shape)) * itemsize
        src = _as_bytes(data)
        if src.size != chunk_size or src.size % itemsize:
            raise ValueError(f"cannot reshape array of size {src.size // max(itemsize, 1)} into shape {chunk_shape}")
        block = BIT_SHUFFLE_BLOCK
        cap = int(nat.lib().hsds_bitshuffle_bound(src.size, itemsize, block))
        if cap < 0:
            raise nat.NativeError(cap, "hsds_bitshuffle_bound")
        out = np.empty(cap, np.uint8)
        n = nat.lib().hsds_bitshuffle_compress(nat.engine().h, src.ctypes.data, src.size, itemsize, block,
                                               out.ctypes.data, cap)
        if n < 0:
            raise nat.NativeError(n, "hsds_bitshuffle_compress")
        return out[:n].tobytes()
    raise ValueError()


def _unshuffle(codec, data, dtype=None, chunk_shape=None):
    """storUtil._unshuffle (storUtil.py:136): codec 1 = byte unshuffle, codec 2 =
    bitshuffle+LZ4 (storUtil.py:144-174: a short buffer, a header whose chunk bytes
    differ from prod(chunk_shape) * itemsize, and any decode failure raise
    HTTPInternalServerError)."""
    if codec == BYTE_SHUFFLE:
        src = _as_bytes(data)
        out = np.empty(src.size, np.uint8)
        rc = nat.lib().hsds_unshuffle(nat.engine().h, src.ctypes.data, src.size, _itemsize(dtype),
                                      out.ctypes.data)
        if rc != nat.OK:
            raise nat.NativeError(rc, "hsds_unshuffle")
        return out.tobytes()
    if codec == BIT_SHUFFLE:
        itemsize = _itemsize(dtype)
        chunk_size = int(np.prod(chunk_shape)) * itemsize      # TypeError without a shape, as there
        src = _as_bytes(data)
        if src.size < 12:
            raise HTTPInternalServerError()
        out = np.empty(max(chunk_size, 1), np.uint8)
        n = nat.lib().hsds_uncompress(nat.engine().h, src.ctypes.data, src.size, nat.COMP_NONE, BIT_SHUFFLE,
                                      itemsize, out.ctypes.data, chunk_size)
        if n < 0:
            if n in (nat.ERR_ARG, nat.ERR_DEVICE):
                raise nat.NativeError(n, "hsds_uncompress")
            raise HTTPInternalServerError()
        return out[:n].tobytes()
    raise ValueError()


def _blosc_nbytes(src):
    """Decoded size recorded in a Blosc1 header, or None when `src` is not a Blosc frame."""
    if src.size >= 16 and src[0] <= 2 and src[3] > 0:
        return int(src[4]) | (int(src[5]) << 8) | (int(src[6]) << 16) | (int(src[7]) << 24)
    return None


def _uncompress(data, compressor=None, shuffle=0, level=None, dtype=None, chunk_shape=None):
    """storUtil._uncompress (storUtil.py:182-235) on the GPU."""
    if shuffle not in (0, BYTE_SHUFFLE, BIT_SHUFFLE) and shuffle:
        raise ValueError()
    comp = _compressor_code(compressor)
    src = _as_bytes(data)
    itemsize = _itemsize(dtype)
    if comp == nat.COMP_NONE and not shuffle:
        return bytes(src)
    if shuffle == BIT_SHUFFLE:
        # the outer codec first (its output is the bitshuffle object), then _unshuffle
        # codec 2 (storUtil.py:189-227)
        if comp != nat.COMP_NONE:
            data = _uncompress(data, compressor, 0, level, dtype, None)
        return _unshuffle(BIT_SHUFFLE, data, dtype=dtype, chunk_shape=chunk_shape)
    if comp != nat.COMP_NONE and _blosc_nbytes(src) is not None and (src[2] >> 5) not in (0, 1, 3, 4):
        # snappy inner codec: not built into the numcodecs the reference pins either
        raise NotImplementedError(f"Blosc inner codec {int(src[2] >> 5)} (snappy) is outside the hsds_amd engine scope")
    if comp == nat.COMP_NONE:
        expected = src.size              # shuffle only: _unshuffle of the bytes as given
    elif chunk_shape is not None:
        expected = int(np.prod(chunk_shape)) * itemsize
    else:
        nb = _blosc_nbytes(src) if comp != nat.COMP_NONE else None
        if nb is not None:
            expected = nb
        elif comp == nat.COMP_NONE:
            expected = src.size
        else:
            expected = None
    if expected is None:
        # size unknown (zlib.decompress semantics): grow the capacity until it fits
        cap = max(1 << 16, src.size * 8)
        while True:
            out = np.empty(cap, np.uint8)
            n = nat.lib().hsds_uncompress(nat.engine().h, src.ctypes.data, src.size, comp, int(shuffle),
                                          itemsize, out.ctypes.data, -cap)
            if n == nat.ERR_SIZE and cap < (1 << 31):
                cap *= 4
                continue
            break
    else:
        out = np.empty(max(expected, 1), np.uint8)
        n = nat.lib().hsds_uncompress(nat.engine().h, src.ctypes.data, src.size, comp, int(shuffle),
                                      itemsize, out.ctypes.data, expected)
    if n < 0:
        if n in (nat.ERR_ARG, nat.ERR_DEVICE):
            raise nat.NativeError(n, "hsds_uncompress")
        raise HTTPInternalServerError()
    return out[:n].tobytes()


def _compress(data, compressor=None, level=5, shuffle=0, dtype=None, chunk_shape=None):
    """storUtil._compress (storUtil.py:238-281) on the GPU: a Blosc1 frame with the
    inner codec cname = compressor (gzip/deflate/zlib are all Blosc "zlib",
    storUtil.py:255-257; lz4 and lz4hc carry LZ4 blocks, blosclz BloscLZ), typesize 1 because the
    reference always hands Blosc a bytes object, and the byte-shuffle flag from
    `shuffle`.  Differences from the reference, by design:
      * zstd splits are the GPU writer's frames (raw literals, predefined sequence
        tables, one block per 8 KiB; zstd_enc.h), not libzstd's bytes: any valid frame
        decodes identically through c-blosc;
      * bitshuffle (shuffle=2) objects carry the GPU LZ4 writer's blocks, not liblz4's
        (any valid block: bitshuffle.decompress_lz4 reads both);
      * an encoder failure raises instead of silently storing the raw bytes
        (storUtil.py:266-279 logs and returns `data`, which its own reader then
        rejects: SURVEY.md section 8b)."""
    if not compressor and shuffle != BIT_SHUFFLE:
        return data
    if shuffle == BIT_SHUFFLE:
        # bitshuffle first, then Blosc without its own shuffle (storUtil.py:243-251); a
        # bitshuffle failure is logged there and the bytes go on unshuffled
        try:
            data = _shuffle(BIT_SHUFFLE, data, dtype=dtype, chunk_shape=chunk_shape)
        except (ValueError, TypeError, AttributeError):
            pass
        shuffle = 0
        if not compressor or compressor == "scaleoffset":
            return data
    if shuffle not in (0, BYTE_SHUFFLE):
        raise ValueError()
    if not compressor or compressor == "scaleoffset":
        return data        # no compressor, nothing shuffled: the bytes as given
    cname = nat.cname_code(compressor)
    if cname is None:
        raise NotImplementedError(f"Blosc codec {compressor!r} has no encoder in the hsds_amd engine")
    if level is None:
        level = 5
    src = _as_bytes(data)
    cap = src.size + 16
    out = np.empty(cap, np.uint8)
    n = nat.lib().hsds_compress_codec(nat.engine().h, src.ctypes.data, src.size, int(level), int(shuffle), 1, cname,
                                      out.ctypes.data, cap)
    if n < 0:
        raise nat.NativeError(n, "hsds_compress_codec")
    return out[:n].tobytes()
