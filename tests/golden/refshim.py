"""Import shim that lets the reference's own codec / selection modules run in the
build container, so that golden vectors can be generated from them.

FIXTURE GENERATION ONLY.  Never imported by the product, by `-m gpu` tests, by
`smoke()` or by `bench.py` (the reference does not exist on the GPU box).

numcodecs (pinned 0.12.1-0.15.1 by the reference: requirements.txt:27,
Pipfile.lock, pyproject.toml:46) is not installed here.  It is re-expressed over
the C library /opt/conda/lib/libblosc.so.1 (c-blosc 1.21.0, "Zlib 1.2.11"),
which is the same c-blosc 1.21.x frame codec numcodecs vendors.  Recipe:
SURVEY.md Appendix A.
"""
import ctypes
import importlib.resources as ir
import sys
import types

import numpy as np

REFERENCE = "/root/reference"

_b = ctypes.CDLL("/opt/conda/lib/libblosc.so.1")
_b.blosc_compress_ctx.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                  ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
_b.blosc_decompress_ctx.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
_b.blosc_cbuffer_sizes.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t),
                                   ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
_b.blosc_cbuffer_metainfo.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t),
                                      ctypes.POINTER(ctypes.c_int)]
_b.blosc_list_compressors.restype = ctypes.c_char_p
_nthreads = [1]


def _buf(x):
    if isinstance(x, (bytes, bytearray, memoryview)):
        return np.ascontiguousarray(np.frombuffer(x, dtype=np.uint8))
    return np.ascontiguousarray(x)


def cbuffer_metainfo(src):
    a = _buf(src)
    ts = ctypes.c_size_t()
    fl = ctypes.c_int()
    _b.blosc_cbuffer_metainfo(a.ctypes.data, ctypes.byref(ts), ctypes.byref(fl))
    return (ts.value, fl.value & 1 and 1 or (2 if fl.value & 4 else 0), bool(fl.value & 2))


class Blosc:
    def __init__(self, cname="lz4", clevel=5, shuffle=1, blocksize=0):
        self.cname, self.clevel, self.shuffle, self.blocksize = cname, clevel, shuffle, blocksize

    def encode(self, buf):
        a = _buf(buf)  # numcodecs: ensure_contiguous_ndarray -> typesize = itemsize
        dst = np.empty(a.nbytes + 16, np.uint8)
        n = _b.blosc_compress_ctx(self.clevel, self.shuffle, a.itemsize, a.nbytes, a.ctypes.data,
                                  dst.ctypes.data, dst.nbytes, self.cname.encode(),
                                  self.blocksize, _nthreads[0])
        if n <= 0:
            raise RuntimeError("blosc compress error")
        return dst[:n].tobytes()

    def decode(self, buf, out=None):
        a = _buf(buf)
        nb, cb, bs = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        _b.blosc_cbuffer_sizes(a.ctypes.data, ctypes.byref(nb), ctypes.byref(cb), ctypes.byref(bs))
        dst = np.empty(nb.value, np.uint8)
        n = _b.blosc_decompress_ctx(a.ctypes.data, dst.ctypes.data, dst.nbytes, _nthreads[0])
        if n < 0:
            raise RuntimeError("blosc decompress error")
        return dst.tobytes()


class Shuffle:
    def __init__(self, elementsize):
        self.elementsize = elementsize

    def encode(self, buf):
        a = _buf(buf)
        n = self.elementsize
        return a.reshape(-1, n).T.copy().reshape(-1) if n > 1 else a.copy()

    def decode(self, buf):
        a = _buf(buf)
        n = self.elementsize
        return a.reshape(n, -1).T.copy().reshape(-1) if n > 1 else a.copy()


def blosc_compress_raw(data, clevel, shuffle, typesize, cname="zlib", blocksize=0):
    """Direct libblosc call with an explicit typesize (frames other writers produce)."""
    a = _buf(data)
    dst = np.empty(a.nbytes + 16, np.uint8)
    n = _b.blosc_compress_ctx(clevel, shuffle, typesize, a.nbytes, a.ctypes.data, dst.ctypes.data,
                              dst.nbytes, cname.encode(), blocksize, 1)
    if n <= 0:
        raise RuntimeError("blosc compress error")
    return dst[:n].tobytes()


def blosc_decompress_raw(frame):
    """libblosc decode; returns bytes or None when libblosc reports an error."""
    a = _buf(frame)
    nb, cb, bs = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
    _b.blosc_cbuffer_sizes(a.ctypes.data, ctypes.byref(nb), ctypes.byref(cb), ctypes.byref(bs))
    dst = np.empty(max(nb.value, 1), np.uint8)
    n = _b.blosc_decompress_ctx(a.ctypes.data, dst.ctypes.data, nb.value, 1)
    if n < 0:
        return None
    return dst[:n].tobytes()


blosc = types.SimpleNamespace(
    list_compressors=lambda: _b.blosc_list_compressors().decode().split(","),
    cbuffer_metainfo=cbuffer_metainfo,
    set_nthreads=lambda n: _nthreads.__setitem__(0, n),
    get_nthreads=lambda: _nthreads[0])
sys.modules["numcodecs"] = types.SimpleNamespace(blosc=blosc, Blosc=Blosc, Shuffle=Shuffle)
sys.modules["bitshuffle"] = types.SimpleNamespace()
sys.modules["importlib_resources"] = types.SimpleNamespace(files=ir.files)
for _m in ["aiobotocore", "aiobotocore.config", "aiobotocore.session", "botocore",
           "botocore.exceptions"]:
    sys.modules[_m] = types.ModuleType(_m)
sys.modules["aiobotocore.config"].AioConfig = object
sys.modules["aiobotocore.session"].get_session = lambda: None
sys.modules["botocore.exceptions"].ClientError = Exception
sys.modules["botocore"].UNSIGNED = None
if REFERENCE not in sys.path:
    sys.path.insert(0, REFERENCE)

from hsds import hsds_logger as _log  # noqa: E402

_log.setLogConfig("ERROR")
