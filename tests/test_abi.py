"""The C-ABI library (include/hsds_amd.h) loads and exports every declared entry point.
CPU-only: no compute call is made without a GPU."""
import ctypes
import os
import subprocess

import pytest

from hsds_amd import _native


@pytest.fixture(scope="module")
def native_lib():
    if not os.path.exists(_native.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build()
    return ctypes.CDLL(_native.LIB_PATH)


def test_header_declares_the_boundary():
    names = _native.declared_functions()
    for must in ("hsds_engine_create", "hsds_engine_destroy", "hsds_decode_batch", "hsds_uncompress",
                 "hsds_shuffle", "hsds_unshuffle", "hsds_copy_batch", "hsds_compare_batch",
                 "hsds_copy_batch_if"):
        assert must in names


def test_library_exports_every_declared_symbol(native_lib):
    missing = [n for n in _native.declared_functions() if not hasattr(native_lib, n)]
    assert not missing, missing


def test_exports_are_c_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    for n in _native.declared_functions():
        assert n in exported, n          # unmangled: extern "C"


def test_ctypes_signatures_cover_header():
    # every declared function has a ctypes prototype in the binding (so argument
    # widths are never defaulted to int)
    L = _native.lib()
    for n in _native.declared_functions():
        assert getattr(L, n).argtypes is not None, n


def test_version_and_strerror(native_lib):
    L = _native.lib()
    assert L.hsds_version().startswith(b"hsds_amd")
    assert L.hsds_strerror(-2)
    assert _native.strerror(_native.ERR_DATA) == "corrupt deflate stream"


def test_no_silent_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU visible")
    with pytest.raises(RuntimeError):
        _native.engine()
    from hsds_amd import codec
    with pytest.raises(Exception):
        codec._uncompress(b"\x78\x9c\x03\x00\x00\x00\x00\x01", compressor="zlib", dtype=None)
