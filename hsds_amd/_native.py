"""ctypes binding of the in-tree C-ABI library hsds_amd/libhsds_amd.so (include/hsds_amd.h).

The product path has no CPU fallback: if the library is missing or no GPU is
visible, the calls raise.
"""
import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# The product always loads the in-tree build.  A/B timing of experiment builds (tools/*.sh)
# swaps it with HSDS_AMD_LIB, honoured only together with the development flag
# HSDS_AMD_DEV=1, which nothing in the product or its tests sets.
LIB_PATH = os.path.join(_HERE, "libhsds_amd.so")
if os.environ.get("HSDS_AMD_DEV") == "1" and os.environ.get("HSDS_AMD_LIB"):
    LIB_PATH = os.environ["HSDS_AMD_LIB"]
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "hsds_amd.h")

OK = 0
ERR_FRAME = -1
ERR_DATA = -2
ERR_TRUNC = -3
ERR_SIZE = -4
ERR_UNSUPPORTED = -5
ERR_ARG = -6
ERR_DEVICE = -7

COMP_NONE, COMP_ZLIB, COMP_OTHER = 0, 1, 2
CNAME_ZLIB, CNAME_LZ4, CNAME_LZ4HC, CNAME_BLOSCLZ, CNAME_ZSTD = 0, 1, 2, 3, 4


def cname_code(compressor):
    """storUtil._compress compressor -> HSDS_CNAME_* (None when the engine has no encoder for it)"""
    if compressor in ("gzip", "deflate", "zlib"):
        return CNAME_ZLIB
    return {"lz4": CNAME_LZ4, "lz4hc": CNAME_LZ4HC, "blosclz": CNAME_BLOSCLZ, "zstd": CNAME_ZSTD}.get(compressor)
SHUFFLE_NONE, SHUFFLE_BYTE, SHUFFLE_BIT = 0, 1, 2
MAX_RANK = 8
KIND_BYTES, KIND_F16, KIND_F32, KIND_F64, KIND_C64, KIND_C128 = 0, 1, 2, 3, 4, 5


class NativeError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        super().__init__(f"{what}: {strerror(code)} ({code})" if what else f"{strerror(code)} ({code})")


class ChunkDesc(ctypes.Structure):
    _fields_ = [("src_off", ctypes.c_uint64), ("src_len", ctypes.c_uint64),
                ("dst_off", ctypes.c_uint64), ("dst_len", ctypes.c_uint64)]


class CopyDesc(ctypes.Structure):
    _fields_ = [("src_off", ctypes.c_uint64), ("dst_off", ctypes.c_uint64),
                ("src_stride", ctypes.c_int64 * MAX_RANK), ("dst_stride", ctypes.c_int64 * MAX_RANK),
                ("count", ctypes.c_int64 * MAX_RANK), ("rank", ctypes.c_int32), ("itemsize", ctypes.c_int32)]


PLAN_PACK, PLAN_PLACE, PLAN_GATHER, PLAN_APPLY, PLAN_APPLY_BCAST, PLAN_DIRECT = 0, 1, 2, 3, 4, 5


class PlanGeom(ctypes.Structure):
    _fields_ = [("rank", ctypes.c_int32), ("itemsize", ctypes.c_int32), ("mode", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("nk", ctypes.c_int64 * MAX_RANK),
                ("chunk_stride", ctypes.c_int64 * MAX_RANK), ("slab_stride", ctypes.c_int64 * MAX_RANK),
                ("step", ctypes.c_int64 * MAX_RANK), ("slab_base", ctypes.c_int64)]


_lib = None


def lib():
    """Load the native library (raises when it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    # torch ships its own libamdhip64; load it first so that this library binds to
    # the same HIP runtime instance (one runtime per process)
    import torch  # noqa: F401
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(LIB_PATH)
    P, I, I64, U32, U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint32, ctypes.c_uint64
    sig = {
        "hsds_engine_create": (I, [I, ctypes.POINTER(P)]),
        "hsds_engine_destroy": (None, [P]),
        "hsds_version": (ctypes.c_char_p, []),
        "hsds_strerror": (ctypes.c_char_p, [I]),
        "hsds_set_tuning": (I, [P, U32, U32, U32, ctypes.c_int32]),
        "hsds_decode_batch": (I, [P, P, P, I64, P, U64, P, I, I, I, P]),
        "hsds_uncompress": (I64, [P, P, I64, I, I, I, P, I64]),
        "hsds_last_inflate_ms": (I, [P, ctypes.POINTER(ctypes.c_float)]),
        "hsds_shuffle_device": (I, [P, P, I64, I, P, P]),
        "hsds_unshuffle_device": (I, [P, P, I64, I, P, P]),
        "hsds_shuffle": (I, [P, P, I64, I, P]),
        "hsds_unshuffle": (I, [P, P, I64, I, P]),
        "hsds_copy_batch": (I, [P, P, P, P, I64, P]),
        "hsds_compare_batch": (I, [P, P, P, P, I64, I, P, P]),
        "hsds_copy_batch_if": (I, [P, P, P, P, I64, P, P]),
        "hsds_encode_batch": (I, [P, P, P, I64, P, U64, P, P, I, I, I, P]),
        "hsds_encode_batch_codec": (I, [P, P, P, I64, P, U64, P, P, I, I, I, I, P]),
        "hsds_compress": (I64, [P, P, I64, I, I, I, P, I64]),
        "hsds_compress_codec": (I64, [P, P, I64, I, I, I, I, P, I64]),
        "hsds_last_deflate_ms": (I, [P, ctypes.POINTER(ctypes.c_float)]),
        "hsds_encode_bitshuffle_batch": (I, [P, P, U64, U64, P, I64, P, U64, P, P, I, I, P]),
        "hsds_bitshuffle_bound": (I64, [I64, I, I]),
        "hsds_bitshuffle_compress": (I64, [P, P, I64, I, I, P, I64]),
        "hsds_partition_ids": (I, [ctypes.c_char_p, I, P, I64, I, P]),
        "hsds_plan_descs": (I, [P, P, P, P, P, P, I64, P, P]),
        "hsds_host_map": (I, [P, P, U64, ctypes.POINTER(ctypes.c_void_p)]),
        "hsds_host_unmap": (I, [P, P]),
        "hsds_stage_upload": (I, [P, P, P, P, I64, P, P, U64, I, P]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def strerror(code):
    names = {OK: "ok", ERR_FRAME: "malformed Blosc frame", ERR_DATA: "corrupt deflate stream",
             ERR_TRUNC: "truncated stream", ERR_SIZE: "decoded size mismatch",
             ERR_UNSUPPORTED: "unsupported codec or layout", ERR_ARG: "invalid argument",
             ERR_DEVICE: "HIP runtime error"}
    return names.get(code, "unknown status")


def declared_functions():
    """Function names declared in include/hsds_amd.h (the C ABI contract)."""
    txt = open(HEADER_PATH).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(hsds_[a-z0-9_]+)\s*\(", txt)))


_engines = {}


class Engine:
    """One engine per device (an opaque hsds_engine*)."""

    def __init__(self, device=0):
        self.device = device
        h = ctypes.c_void_p()
        rc = lib().hsds_engine_create(device, ctypes.byref(h))
        if rc != OK:
            raise NativeError(rc, "hsds_engine_create")
        self.h = h

    def close(self):
        if self.h:
            lib().hsds_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_tuning(self, seg_over16=None, warmup_bits=None, rounds=None, waves_per_stream=None):
        """Inflate tuning; a setting left at None keeps the engine's current value
        (hsds_engine_create's defaults: the GPU-swept ones).  waves_per_stream: 0 by batch
        size, 1, 2, 4 or 8 wavefronts per zlib stream (None: keep)."""
        keep = 0xFFFFFFFF
        rc = lib().hsds_set_tuning(self.h, keep if seg_over16 is None else seg_over16,
                                   keep if warmup_bits is None else warmup_bits,
                                   keep if waves_per_stream is None else waves_per_stream,
                                   -1 if rounds is None else rounds)
        if rc != OK:
            raise NativeError(rc, "hsds_set_tuning")

    def last_inflate_ms(self):
        v = ctypes.c_float()
        rc = lib().hsds_last_inflate_ms(self.h, ctypes.byref(v))
        if rc != OK:
            raise NativeError(rc, "hsds_last_inflate_ms")
        return v.value

    def last_deflate_ms(self):
        v = ctypes.c_float()
        rc = lib().hsds_last_deflate_ms(self.h, ctypes.byref(v))
        if rc != OK:
            raise NativeError(rc, "hsds_last_deflate_ms")
        return v.value


def engine(device=None):
    """Process-wide engine for `device` (default: torch's current device)."""
    if device is None:
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("hsds_amd needs a ROCm GPU (torch.cuda.is_available() is False)")
        device = torch.cuda.current_device()
    e = _engines.get(device)
    if e is None:
        e = Engine(device)
        _engines[device] = e
    return e
