"""CPU emulation of the GPU zstd split decoder (hsds_amd/csrc/zstd_lane.h, the code
each lane runs, compiled for CPU by tests/emu/zstd_emu.cpp): every zstd object of the
reference goldens (tests/golden/codec2_cases: the reference's _compress at levels 1-9,
typesize 2-8 frames, corrupted frames) against the reference's sha256 and errors, and
every split against the oracle's independent restatement (oracle.c orc_zstd_decode)."""
import ctypes
import hashlib
import os
import struct
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU = os.path.join(ROOT, "tests", "emu", "libzstd_emu.so")
SRC = os.path.join(ROOT, "tests", "emu", "zstd_emu.cpp")


@pytest.fixture(scope="module")
def emu():
    hdrs = [os.path.join(ROOT, "hsds_amd", "csrc", h) for h in ("zstd_lane.h", "zstd_wave.h", "inflate_wave.h")]
    if not os.path.exists(EMU) or os.path.getmtime(EMU) < max(os.path.getmtime(p) for p in [SRC] + hdrs):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", EMU, SRC])
    L = ctypes.CDLL(EMU)
    L.emu_zstd_frame.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]
    L.emu_zstd_frame_wave.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]
    return L


WAVE = [False]


def split(L, comp, n):
    src = np.frombuffer(comp, np.uint8).copy() if comp else np.zeros(1, np.uint8)
    dst = np.zeros(max(n, 1) + 3, np.uint8)
    o = 1 if WAVE[0] else 0                   # the wave decoder also at an odd destination
    fn = L.emu_zstd_frame_wave if WAVE[0] else L.emu_zstd_frame
    r = fn(src.ctypes.data, len(comp), dst.ctypes.data + o, n)
    return r, dst[o:o + n].tobytes()


def frame_decode(L, f, oracle_lib=None):
    if len(f) < 16:
        return -1
    flags, ts = f[2], f[3]
    nb, bs, cb = struct.unpack("<III", f[4:16])
    if cb > len(f):
        return -1
    if flags & 2:
        return f[16:16 + nb]
    nblocks = (nb + bs - 1) // bs
    left = nb % bs
    out = bytearray()
    for b in range(nblocks):
        isl = b == nblocks - 1 and left
        bsz = left if isl else bs
        nspl = ts if (not flags & 0x10 and ts <= 16 and bs // ts >= 128 and not isl) else 1
        ne = bsz // nspl
        p = struct.unpack("<i", f[16 + 4 * b:20 + 4 * b])[0]
        blk = bytearray()
        for _ in range(nspl):
            cs = struct.unpack("<i", f[p:p + 4])[0]
            p += 4
            if cs == ne:
                blk += f[p:p + cs]
            else:
                r, d = split(L, f[p:p + cs], ne)
                if oracle_lib is not None:
                    want = oracle_lib.zstd_decode(f[p:p + cs], ne)
                    assert (r != 0) == isinstance(want, int) and (r != 0 or d == want)
                if r != 0:
                    return r
                blk += d
            p += cs
        if flags & 1 and ts > 1:
            cnt = bsz // ts
            blk = np.frombuffer(bytes(blk[:cnt * ts]), np.uint8).reshape(ts, cnt).T.tobytes() + bytes(blk[cnt * ts:])
        out += blk
    return bytes(out)


@pytest.mark.parametrize("wave", [False, True])
def test_zstd_reference_goldens(emu, golden2, oracle_lib, wave):
    """the lane decoder (zstd_lane.h) and the wavefront decoder (zstd_wave.h)"""
    WAVE[0] = wave
    meta, arrs = golden2
    checked = 0
    for c in meta["cases"]:
        if c["codec"] != 4 or c["memcpyed"]:
            continue
        blob = arrs[c["name"] + "__in"].tobytes()
        got = frame_decode(emu, blob, oracle_lib if not c["name"].endswith("_trunc") else None)
        if c["status"] == "error" or c["name"].endswith("_trunc"):
            assert isinstance(got, int), c["name"]
            continue
        assert not isinstance(got, int), (c["name"], got)
        assert hashlib.sha256(got).hexdigest() == c["out_sha256"], c["name"]
        checked += 1
    assert checked >= 35


@pytest.mark.parametrize("wave", [False, True])
def test_zstd_bench_corpus(emu, wave):
    """libblosc 1.21 zstd frames of the bench corpus (128 KiB blocks with ~37K sequences
    each, repeat offsets, multi-window decodes): decoded bytes equal the raw chunk"""
    if not os.path.exists("/opt/conda/lib/libblosc.so.1"):
        pytest.skip("the image's libblosc is absent")
    import sys
    sys.path.insert(0, ROOT)
    from bench import make_corpus
    WAVE[0] = wave
    raw, blobs = make_corpus("ZSTD", 2, 20261016, 2)
    for r, b in zip(raw, blobs):
        got = frame_decode(emu, bytes(np.asarray(b, np.uint8)))
        assert not isinstance(got, int), got
        assert got == np.ascontiguousarray(r).view(np.uint8).tobytes()


def test_zstd_wave_literal_streams(emu):
    """The wave decoder's Huffman literals on every lane (zstd_wave.h huf_streams_wave):
    libblosc 1.21 zstd frames of literal-heavy data -- skewed random bytes (Huffman codes of
    many lengths), short and long blocks (one-stream and four-stream literal sections),
    levels 1-9 -- decode to their input, as the one-lane-per-stream decoder's do"""
    if not os.path.exists("/opt/conda/lib/libblosc.so.1"):
        pytest.skip("the image's libblosc is absent")
    lb = ctypes.CDLL("/opt/conda/lib/libblosc.so.1")
    lb.blosc_compress_ctx.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
    rng = np.random.default_rng(61)
    cases = []
    for n in (40, 300, 1500, 5000, 40000, 131072, 300000):
        for kind in range(3):
            if kind == 0:      # geometric bytes: a few very short codes, a long tail of 11-bit ones
                a = np.minimum(rng.geometric(0.08, n), 255).astype(np.uint8)
            elif kind == 1:    # near-uniform bytes with a little structure (codes of 7-9 bits)
                a = (rng.integers(0, 200, n) + (np.arange(n) % 7)).astype(np.uint8)
            else:              # text-like runs mixed with noise: matches and literals
                a = np.frombuffer((b"the quick brown fox %d jumps " * (n // 20 + 1))[:n], np.uint8).copy()
                a[rng.integers(0, n, n // 5)] = rng.integers(0, 256, n // 5).astype(np.uint8)
            cases.append(a)
    checked = 0
    for wave in (False, True):
        WAVE[0] = wave
        for a in cases:
            for level in (1, 5, 9):
                out = np.zeros(a.size + 64, np.uint8)
                k = lb.blosc_compress_ctx(level, 0, 1, a.size, a.ctypes.data, out.ctypes.data, out.size, b"zstd", 0, 1)
                assert k > 0
                got = frame_decode(emu, out[:k].tobytes())
                assert not isinstance(got, int), (a.size, level, got)
                assert got == a.tobytes(), (a.size, level)
                checked += 1
    assert checked == 2 * len(cases) * 3
