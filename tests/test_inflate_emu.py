"""CPU emulation of the GPU inflate kernel (hsds_amd/csrc/inflate_wave.h compiled with
LANE_LOOP iterating the 64 lanes) checked against libz / the oracle.  This runs the
kernel's exact orchestration (speculative segments, continuation, repair rounds,
LDS source map) on CPU; `-m gpu` tests run the same code on the MI355X."""
import ctypes
import os
import subprocess
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU = os.path.join(ROOT, "tests", "emu", "libinflate_emu.so")
SRC = os.path.join(ROOT, "tests", "emu", "inflate_emu.cpp")


@pytest.fixture(scope="module")
def emu():
    hdr = os.path.join(ROOT, "hsds_amd", "csrc", "inflate_wave.h")
    if not os.path.exists(EMU) or os.path.getmtime(EMU) < max(os.path.getmtime(SRC), os.path.getmtime(hdr)):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", EMU, SRC])
    L = ctypes.CDLL(EMU)
    L.emu_inflate.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                              ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                              ctypes.c_int, ctypes.c_void_p]
    return L


def run(L, comp, n, tune=(384, 96, 1, 192, 4)):
    src = np.frombuffer(comp, np.uint8).copy()
    if src.size == 0:
        src = np.zeros(1, np.uint8)
    dst = np.zeros(max(n, 1), np.uint8)
    st = np.zeros(14, np.uint64)
    r = L.emu_inflate(src.ctypes.data, len(comp), dst.ctypes.data, n, *tune, st.ctypes.data)
    return r, dst[:n].tobytes()


def corpus():
    rng = np.random.default_rng(123)
    sm = np.round(np.cumsum(rng.normal(size=80000)), 2).astype(np.float32).tobytes()
    out = {
        "smooth_f32": sm,
        "smooth_f32_shuffled": np.frombuffer(sm, np.uint8).reshape(-1, 4).T.copy().tobytes(),
        "int16": (np.cumsum(rng.normal(size=60000)) * 100).astype("<i2").tobytes(),
        "zeros": bytes(150000),
        "random": rng.integers(0, 256, 70000, dtype=np.uint8).tobytes(),
        "text": b"".join(b"row %d: the quick brown fox %d\n" % (i, i * 7 % 13) for i in range(3000)),
        "lowcard": rng.integers(0, 3, 90000, dtype=np.uint8).tobytes(),
        "empty": b"",
        "one": b"x",
        "runs": b"".join(bytes([i % 251]) * (i % 300 + 1) for i in range(700)),
    }
    return out


@pytest.mark.parametrize("level", [0, 1, 4, 6, 9])
def test_levels_match_zlib(emu, level):
    for name, data in corpus().items():
        c = zlib.compress(data, level)
        r, out = run(emu, c, len(data))
        assert r == 0, (name, level, r)
        assert out == data, (name, level)


@pytest.mark.parametrize("strategy", [zlib.Z_FILTERED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FIXED])
def test_strategies(emu, strategy):
    for name, data in corpus().items():
        co = zlib.compressobj(5, zlib.DEFLATED, 15, 8, strategy)
        c = co.compress(data) + co.flush()
        r, out = run(emu, c, len(data))
        assert r == 0 and out == data, (name, strategy, r)


def test_small_window_bits_and_memlevel(emu):
    data = corpus()["text"] * 3
    for wbits, mem in ((9, 1), (10, 9), (12, 4), (15, 1)):
        co = zlib.compressobj(6, zlib.DEFLATED, wbits, mem)
        c = co.compress(data) + co.flush()
        r, out = run(emu, c, len(data))
        assert r == 0 and out == data, (wbits, mem)


@pytest.mark.parametrize("tune", [(64, 0, 1, 0, 0), (512, 1024, 0, 256, 8), (128, 32, 1, 64, 1), (256, 200, 1, 256, 2)])
def test_tunings_do_not_change_output(emu, tune):
    for name in ("smooth_f32", "smooth_f32_shuffled", "zeros", "text"):
        data = corpus()[name]
        c = zlib.compress(data, 4)
        r, out = run(emu, c, len(data), tune)
        assert r == 0 and out == data, (name, tune)


def test_corruptions_fail_like_libz(emu):
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as orc
    rng = np.random.default_rng(9)
    base = corpus()["smooth_f32"][:40000]
    good = zlib.compress(base, 4)
    for t in range(120):
        b = bytearray(good)
        k = t % 5
        if k == 0:
            b = b[:int(rng.integers(1, len(b)))]
        elif k == 1:
            i = int(rng.integers(0, len(b)))
            b[i] ^= 1 << int(rng.integers(0, 8))
        elif k == 2:
            i = int(rng.integers(2, min(len(b), 300)))      # header / first block header area
            b[i] ^= 1 << int(rng.integers(0, 8))
        elif k == 3:
            b[-1 - int(rng.integers(0, 4))] ^= 0x40          # adler32
        else:
            b = b + bytes(rng.integers(0, 256, 7, dtype=np.uint8))   # trailing garbage is ignored
        n = len(base)
        ref = orc.uncompress(bytes(b), "zlib", 0, 1, n)
        r, out = run(emu, bytes(b), n)
        if isinstance(ref, int):
            assert r < 0, (t, k, ref, r)
        else:
            assert r == 0 and out == ref, (t, k, r)


def test_wrong_expected_size(emu):
    data = corpus()["text"]
    c = zlib.compress(data, 4)
    assert run(emu, c, len(data) - 1)[0] < 0
    assert run(emu, c, len(data) + 1)[0] < 0


def test_deep_codes_use_second_level_tables(emu):
    # Fibonacci symbol frequencies make zlib build length-limited codes that reach
    # 15 bits for both literals and distances: the longest codes and the largest
    # second-level table usage the LDS tables are sized for (LL_SUB / D_SUB).
    import zlib
    rng = np.random.default_rng(77)
    fib = [1, 1]
    while len(fib) < 40:
        fib.append(fib[-1] + fib[-2])
    lits = np.concatenate([np.full(min(f, 20000), s % 256, np.uint8) for s, f in enumerate(fib[:24])])
    rare = rng.permutation(256).astype(np.uint8)          # every other byte value once
    data = np.concatenate([rng.permutation(lits), rare]).tobytes()
    # matches at Fibonacci-distributed distances
    parts = [data]
    for k, f in enumerate(fib[:20]):
        d = 1 + (k * 1543) % 30000
        parts.append(data[-d:][:8] * max(1, min(f, 50)))
    data = b"".join(parts)[:400000]
    for level in (1, 6, 9):
        comp = zlib.compress(data, level)
        r, out = run(emu, comp, len(data))
        assert r == 0 and out == data, (level, r)
