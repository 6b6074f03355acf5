"""CPU emulation of the GPU bitshuffle+LZ4 chunk decoder (hsds_amd/csrc/bshuf.h, compiled
for CPU by tests/emu/bshuf_emu.cpp) against the golden frames of
tests/golden/make_bitshuffle_golden.py (expected results from liblz4 1.9.3 and
imagecodecs' bitshuffle 0.3.5 core) and against the oracle (oracle.c
orc_bitshuffle_decode) on frames with the oracle's own LZ4 writer."""
import ctypes
import hashlib
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU = os.path.join(ROOT, "tests", "emu", "libbshuf_emu.so")
SRC = os.path.join(ROOT, "tests", "emu", "bshuf_emu.cpp")


@pytest.fixture(scope="module")
def emu():
    hdrs = [os.path.join(ROOT, "hsds_amd", "csrc", h) for h in ("bshuf.h", "lz_wave.h", "inflate_wave.h")]
    if not os.path.exists(EMU) or os.path.getmtime(EMU) < max(os.path.getmtime(p) for p in [SRC] + hdrs):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", EMU, SRC])
    L = ctypes.CDLL(EMU)
    L.emu_bshuf_chunk.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
    L.emu_bshuf_untrans.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
    L.emu_bshuf_trans.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
    return L


def decode(L, blob, nbytes, es, off=0):
    src = np.frombuffer(blob, np.uint8).copy() if blob else np.zeros(1, np.uint8)
    dst = np.zeros(max(nbytes, 1) + 8, np.uint8)
    st = L.emu_bshuf_chunk(src.ctypes.data, len(blob), dst.ctypes.data + off, nbytes, es)
    return st, dst[off:off + nbytes].tobytes()


def test_untrans_matches_oracle(emu, oracle_lib):
    rng = np.random.default_rng(3)
    for es in (1, 2, 3, 4, 8, 16, 17):
        for cnt in (8, 64, 2048, 520):
            raw = rng.integers(0, 256, cnt * es, dtype=np.uint8).tobytes()
            t = np.frombuffer(oracle_lib.bshuf_trans(raw, es), np.uint8).copy()
            out = np.zeros(cnt * es, np.uint8)
            emu.emu_bshuf_untrans(t.ctypes.data, out.ctypes.data, cnt, es)
            assert out.tobytes() == raw, (es, cnt)


@pytest.mark.parametrize("off", [0, 1])
def test_bshuf_goldens(emu, bshuf_golden, off):
    meta, arrs = bshuf_golden
    for c in meta["cases"]:
        blob = arrs[c["name"] + "__in"].tobytes()
        st, got = decode(emu, blob, c["nbytes"], c["itemsize"], off)
        if c["status"] == "error":
            assert st < 0, c["name"]
        else:
            assert st == 0, (c["name"], st)
            assert hashlib.sha256(got).hexdigest() == c["out_sha256"], c["name"]


def test_bshuf_oracle_frames(emu, oracle_lib):
    rng = np.random.default_rng(11)
    for es, n, block in ((4, 262144, 2048), (2, 100003, 512), (8, 4099, 2048), (1, 70001, 0), (5, 1234, 64)):
        raw = (np.cumsum(rng.integers(-3, 4, n * es)) % 256).astype(np.uint8).tobytes()
        blob = oracle_lib.bitshuffle_encode(raw, es, block)
        st, got = decode(emu, blob, len(raw), es)
        assert st == 0 and got == raw, (es, n, block, st)
        # a truncated and an over-long frame are errors, as in the oracle
        for bad in (blob[:-1], blob + b"\0"):
            assert decode(emu, bad, len(raw), es)[0] < 0
            assert isinstance(oracle_lib.bitshuffle_decode(bad, len(raw), es), int)


@pytest.mark.parametrize("es", [1, 2, 3, 4, 5, 8, 16, 32])
@pytest.mark.parametrize("cnt", [8, 64, 2048])
def test_forward_transposition_matches_oracle(emu, es, cnt):
    """bs::trans_group (the write path's transposition) equals the oracle's
    bshuf_trans_bit_elem restatement, and untrans_block inverts it."""
    from oracle import oracle as orc
    rng = np.random.default_rng(es * 1000 + cnt)
    for kind in ("random", "smooth"):
        if kind == "random":
            x = rng.integers(0, 256, cnt * es, dtype=np.uint8)
        else:
            x = np.frombuffer(np.round(np.cumsum(rng.normal(size=cnt * es // 4 + 1)), 2).astype("<f4").tobytes(),
                              np.uint8)[:cnt * es].copy()
        # aligned and unaligned element bases (the f32 fast path needs 4-byte alignment)
        for off in (0, 1):
            buf = np.zeros(cnt * es + 8, np.uint8)
            buf[off:off + cnt * es] = x
            out = np.zeros(cnt * es, np.uint8)
            emu.emu_bshuf_trans(buf.ctypes.data + off, out.ctypes.data, cnt, es)
            ref = np.frombuffer(orc.bshuf_trans(x.tobytes(), es), np.uint8)
            assert out.tobytes() == ref.tobytes()
            back = np.zeros(cnt * es, np.uint8)
            emu.emu_bshuf_untrans(out.ctypes.data, back.ctypes.data, cnt, es)
            assert back.tobytes() == x.tobytes()
