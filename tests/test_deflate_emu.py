"""CPU emulation of the wave deflate encoder (hsds_amd/csrc/deflate_wave.h compiled
for the host with LANE_LOOP iterating the 64 lanes).  Every stream must inflate
through libz (CPython zlib, the library storUtil._uncompress calls for F2 and
c-blosc calls per split for F1) to exactly the input; sizes are checked against
zlib's at the same level.  Test infrastructure: the product runs the same source
as a HIP kernel."""
import ctypes
import os
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tests", "emu", "libdeflate_emu.so")


@pytest.fixture(scope="module")
def emu():
    if not os.path.exists(LIB):
        pytest.skip("emulator not built (python -c 'import __graft_entry__ as g; g.build()')")
    L = ctypes.CDLL(LIB)
    L.emu_deflate.restype = ctypes.c_int64
    L.emu_deflate.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int,
                              ctypes.c_int]
    L.emu_deflate_shuffled.restype = ctypes.c_int64
    L.emu_deflate_shuffled.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                       ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
    return L


def enc(emu, b, level=4, cap=None, chain=0):
    a = np.frombuffer(b, np.uint8) if len(b) else np.zeros(1, np.uint8)
    cap = len(b) + 1024 if cap is None else cap
    out = np.zeros(cap // 4 + 8, np.uint32)
    r = emu.emu_deflate(a.ctypes.data, len(b), out.ctypes.data, cap, level, chain)
    return None if r < 0 else out.view(np.uint8)[:r].tobytes()


def smooth(rng, n):
    return np.round(np.cumsum(rng.normal(size=n // 4)), 2).astype(np.float32).tobytes()


CASES = {
    "empty": lambda r: b"",
    "one": lambda r: b"x",
    "three": lambda r: b"abc",
    "zeros_8192": lambda r: bytes(8192),
    "zeros_8193": lambda r: bytes(8193),
    "zeros_70000": lambda r: bytes(70000),
    "text": lambda r: (b"the quick brown fox jumps over the lazy dog. " * 2000)[:65537],
    "random_20000": lambda r: r.integers(0, 256, 20000, dtype=np.uint8).tobytes(),
    "runs": lambda r: np.repeat(r.integers(0, 4, 3000, dtype=np.uint8), r.integers(1, 40, 3000)).tobytes(),
    "smooth_f32_64k": lambda r: smooth(r, 1 << 16),
    "int16_cumsum": lambda r: (np.cumsum(r.normal(size=40000)) * 100).astype("<i2").tobytes(),
    "seg_edge_minus1": lambda r: smooth(r, 8188) + b"\x01\x02\x03",
    "two_segments_plus": lambda r: smooth(r, 16384) + b"abcabcabcabc",
}


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("level", [0, 1, 4, 5, 9])
def test_roundtrip_through_libz(emu, name, level):
    rng = np.random.default_rng(abs(hash(name)) % (1 << 31))
    b = CASES[name](rng)
    c = enc(emu, b, level)
    assert c is not None
    assert zlib.decompress(c) == b
    assert c[0] == 0x78 and (c[0] * 256 + c[1]) % 31 == 0
    # zlib's FLEVEL bits for the level (deflate.c)
    lf = 0 if level < 2 else 1 if level < 6 else 2 if level == 6 else 3
    assert c[1] >> 6 == lf


def test_ratio_close_to_zlib_on_smooth_f32(emu):
    # headline data: 256 KiB Blosc splits of smooth float32
    rng = np.random.default_rng(20261015)
    ours = ref = 0
    for _ in range(4):
        b = smooth(rng, 1 << 18)
        c = enc(emu, b, 4)
        assert zlib.decompress(c) == b
        ours += len(c)
        ref += len(zlib.compress(b, 4))
    assert ours / ref < 1.06, ours / ref


def test_capacity_overflow_reports_raw(emu):
    rng = np.random.default_rng(3)
    b = rng.integers(0, 256, 50000, dtype=np.uint8).tobytes()
    # c-blosc stores a split raw when the codec output is not smaller than the split
    assert enc(emu, b, 4, cap=len(b) - 1) is None
    c = enc(emu, b, 4, cap=len(b) + 64)
    assert c is not None and zlib.decompress(c) == b
    small = bytes(1000)
    assert enc(emu, small, 4, cap=4) is None


@pytest.mark.parametrize("ts", [2, 4, 8])
def test_shuffled_block_gather(emu, ts):
    # a Blosc block with typesize > 1: split j is byte plane j of the block
    rng = np.random.default_rng(ts)
    bsz = 4096 * ts + 3
    block = np.frombuffer(smooth(rng, bsz - 3) + b"xyz", np.uint8).copy()
    neb = bsz // ts
    body = block[:neb * ts].reshape(neb, ts).T.reshape(-1)
    shuffled = np.concatenate([body, block[neb * ts:]]).tobytes()
    for off, n in ((0, neb), (neb, neb), ((ts - 1) * neb, neb), (0, bsz)):
        out = np.zeros((n + 1024) // 4 + 8, np.uint32)
        r = emu.emu_deflate_shuffled(block.ctypes.data, n, out.ctypes.data, n + 1024, 4, ts, neb, off)
        assert r > 0
        assert zlib.decompress(out.view(np.uint8)[:r].tobytes()) == shuffled[off:off + n]


def enc_far(emu, b, level, far, chain=0):
    emu.emu_deflate_far.restype = ctypes.c_int64
    emu.emu_deflate_far.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int]
    a = np.frombuffer(b, np.uint8)
    out = np.zeros(len(b) // 4 + 300, np.uint32)
    r = emu.emu_deflate_far(a.ctypes.data, len(b), out.ctypes.data, len(b) + 1024, level, chain, far)
    assert r > 0
    return out.view(np.uint8)[:r].tobytes()


@pytest.mark.parametrize("level", [4, 6, 9])
def test_far_ring_reaches_the_32k_window(emu, level):
    # a 20 000-byte random block repeated: its copy lies beyond the LDS ring (8 KiB) but
    # inside zlib's 32 KiB window, so only the far chains find it
    rng = np.random.default_rng(11)
    blk = rng.integers(0, 256, 20000, dtype=np.uint8).tobytes()
    b = blk + blk + blk[:5000]
    near, far = enc_far(emu, b, level, 0), enc_far(emu, b, level, 1)
    assert zlib.decompress(near) == b and zlib.decompress(far) == b
    assert len(far) < 0.8 * len(near), (len(far), len(near))
    if level >= 6:    # the levels that use the far ring: chains deep enough past the 11-bit
        #              hash collisions of 20 000 random positions
        assert len(far) < 1.07 * len(zlib.compress(b, level)), (len(far), len(zlib.compress(b, level)))
        assert enc(emu, b, level) == far


def test_far_ring_with_deep_chains_on_row_walks(emu):
    # cfg5's worst chunks (row random walks from 0): deep chains gain only with the far ring
    rng = np.random.default_rng(5)
    a = np.round(np.cumsum(rng.normal(size=(128, 512)), axis=1), 2).astype(np.float32).tobytes()
    near, far = enc_far(emu, a, 4, 0, 32), enc_far(emu, a, 4, 1, 32)
    assert zlib.decompress(far) == a
    assert len(far) < 0.97 * len(near), (len(far), len(near))
