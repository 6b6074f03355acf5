"""CPU emulation of the GPU LZ4 write path (parse phase of deflate_wave.h, then the
wave-parallel token walk of lz4_enc.h, tests/emu/deflate_emu.cpp): every block
decodes to its input through the oracle's LZ4 decoder (oracle.c orc_lz4_decode,
pinned by the reference goldens), for all levels and the data shapes that stress
literal runs crossing lanes and segments, long runs and the block-end rules."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU = os.path.join(ROOT, "tests", "emu", "libdeflate_emu.so")
SRC = os.path.join(ROOT, "tests", "emu", "deflate_emu.cpp")


@pytest.fixture(scope="module")
def emu():
    hdrs = [os.path.join(ROOT, "hsds_amd", "csrc", h) for h in ("lz4_enc.h", "deflate_wave.h", "lz_wave.h",
                                                               "inflate_wave.h")]
    if not os.path.exists(EMU) or os.path.getmtime(EMU) < max(os.path.getmtime(p) for p in [SRC] + hdrs):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", EMU, SRC])
    L = ctypes.CDLL(EMU)
    L.emu_lz4_block.restype = ctypes.c_int64
    L.emu_lz4_block.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int]
    return L


def block(L, data, level):
    src = np.frombuffer(data, np.uint8).copy() if data else np.zeros(1, np.uint8)
    dst = np.zeros(len(data) + len(data) // 255 + 64, np.uint8)
    r = L.emu_lz4_block(src.ctypes.data, len(data), dst.ctypes.data, dst.size, level)
    assert r >= 0, r
    return dst[:r].tobytes()


def inputs():
    rng = np.random.default_rng(3)
    return {
        "smooth_f32": np.round(np.cumsum(rng.normal(size=65536)), 2).astype(np.float32).tobytes(),
        "zeros": bytes(200000),
        "text": (b"hsds chunk, the quick brown fox " * 4000)[:100003],
        "steps": np.repeat(rng.integers(0, 50, 3000), 97).astype("<i4").tobytes(),
        "random": rng.integers(0, 256, 50000, dtype=np.uint8).tobytes(),
        "lowent": rng.integers(0, 4, 131072, dtype=np.uint8).tobytes(),
        "sparse": (rng.random(120000) < 0.01).astype(np.uint8).tobytes(),   # long literal-free runs, rare literals
        "tiny": b"abcdefghijklm",
        "one": b"x",
        "end_rules": bytes(30) + b"0123456789abcdefghij" * 3,
    }


@pytest.mark.parametrize("name", sorted(inputs()))
@pytest.mark.parametrize("level", [1, 4, 5, 9])
def test_lz4_blocks_decode(emu, oracle_lib, name, level):
    data = inputs()[name]
    comp = block(emu, data, level)
    assert oracle_lib.lz4_decode(comp, len(data)) == data


def blz_block(L, data, level):
    L.emu_blosclz_block.restype = ctypes.c_int64
    L.emu_blosclz_block.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int]
    src = np.frombuffer(data, np.uint8).copy() if data else np.zeros(1, np.uint8)
    dst = np.zeros(len(data) + len(data) // 16 + 64, np.uint8)
    r = L.emu_blosclz_block(src.ctypes.data, len(data), dst.ctypes.data, dst.size, level)
    assert r >= 0, r
    return dst[:r].tobytes()


@pytest.mark.parametrize("name", sorted(inputs()))
@pytest.mark.parametrize("level", [1, 5, 9])
def test_blosclz_blocks_decode(emu, oracle_lib, name, level):
    data = inputs()[name]
    comp = blz_block(emu, data, level)
    assert oracle_lib.blosclz_decode(comp, len(data)) == data
