"""CPU emulation of the zstd block writer (hsds_amd/csrc/zstd_enc.h, the GPU source
compiled for the host): frames of the emulated parse + per-segment zstd blocks must decode
to the input through libzstd 1.4.9 (the image's /opt/conda library; numcodecs' c-blosc
vendors a zstd of the same format) and through the oracle's RFC 8878 restatement
(orc_zstd_decode, pinned by the reference's zstd objects).  The Blosc-zstd frame geometry
(HCR block size, never split) is pinned against libblosc 1.21 headers.  Test
infrastructure only."""
import ctypes
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tests", "emu", "libdeflate_emu.so")
LIBZSTD = "/opt/conda/lib/libzstd.so.1"
LIBBLOSC = "/opt/conda/lib/libblosc.so.1"


@pytest.fixture(scope="module")
def emu():
    if not os.path.exists(LIB):
        pytest.skip("emulator not built")
    L = ctypes.CDLL(LIB)
    L.emu_zstd_frame.restype = ctypes.c_int64
    L.emu_zstd_frame.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int]
    return L


@pytest.fixture(scope="module")
def zstd():
    if not os.path.exists(LIBZSTD):
        pytest.skip("libzstd absent")
    Z = ctypes.CDLL(LIBZSTD)
    Z.ZSTD_decompress.restype = ctypes.c_size_t
    Z.ZSTD_decompress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
    Z.ZSTD_isError.argtypes = [ctypes.c_size_t]
    Z.ZSTD_compress.restype = ctypes.c_size_t
    Z.ZSTD_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    return Z


def frame(emu, a, level):
    a = np.ascontiguousarray(a, np.uint8)
    out = np.zeros(a.size + a.size // 64 + 1024, np.uint8)
    k = emu.emu_zstd_frame(a.ctypes.data if a.size else 0, a.size, out.ctypes.data, out.size, level)
    assert k > 0
    return out[:k].tobytes()


def unzstd(Z, f, n):
    s = np.frombuffer(f, np.uint8)
    out = np.zeros(n + 16, np.uint8)
    r = Z.ZSTD_decompress(out.ctypes.data, out.size, s.ctypes.data, len(f))
    assert not Z.ZSTD_isError(r), r
    return out[:r].tobytes()


def _smooth(rng, n):
    return np.round(np.cumsum(rng.normal(size=n // 4)), 2).astype(np.float32).view(np.uint8)


CASES = {
    "smooth_256k": lambda r: _smooth(r, 1 << 18),
    "smooth_odd": lambda r: np.concatenate([_smooth(r, 70000), np.arange(3, dtype=np.uint8)]),
    "zeros_100k": lambda r: np.zeros(100000, np.uint8),
    "random_30k": lambda r: r.integers(0, 256, 30000, dtype=np.uint8),
    "runs": lambda r: np.repeat(r.integers(0, 4, 3000, dtype=np.uint8), r.integers(1, 40, 3000)),
    "int16": lambda r: (np.cumsum(r.normal(size=40000)) * 100).astype("<i2").view(np.uint8),
    "text": lambda r: np.frombuffer((b"the quick brown fox jumps over the lazy dog. " * 3000)[:70001], np.uint8),
    "tiny": lambda r: np.frombuffer(b"abcabcabcabcabcXYZ" * 3, np.uint8),
    "one_seg_edge": lambda r: np.concatenate([_smooth(r, 8192), np.zeros(1, np.uint8)]),
}


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("level", [1, 5, 9])
def test_frames_decode_through_libzstd_and_oracle(emu, zstd, name, level):
    from oracle import oracle as orc
    rng = np.random.default_rng(sum(map(ord, name)))
    a = np.ascontiguousarray(CASES[name](rng), np.uint8)
    f = frame(emu, a, level)
    assert f[:4] == b"\x28\xb5\x2f\xfd"
    assert unzstd(zstd, f, a.size) == a.tobytes()
    assert orc.zstd_decode(f, a.size) == a.tobytes()


def test_ratio_on_smooth_f32(emu, zstd):
    # the frame's own FSE_Compressed_Mode sequence tables against the predefined ones
    # (round 4: 1.29x libzstd level 5 here); the bounds document both (zstd writer)
    emu.emu_zstd_frame_t.restype = ctypes.c_int64
    emu.emu_zstd_frame_t.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                     ctypes.c_int, ctypes.c_int]
    rng = np.random.default_rng(20261015)
    ours = pre = ref = 0
    for _ in range(2):
        a = _smooth(rng, 1 << 18)
        ours += len(frame(emu, a, 5))
        o2 = np.zeros(a.size + 4096, np.uint8)
        k = emu.emu_zstd_frame_t(a.ctypes.data, a.size, o2.ctypes.data, o2.size, 5, 0)
        assert k > 0 and unzstd(zstd, o2[:k].tobytes(), a.size) == a.tobytes()
        pre += k
        out = np.zeros(a.size + 1024, np.uint8)
        ref += zstd.ZSTD_compress(out.ctypes.data, out.size, a.ctypes.data, a.size, 5)
    assert ours / ref < 1.05, ours / ref
    assert pre / ref > 1.2 and ours < 0.85 * pre, (ours / ref, pre / ref)


def _blosc_zstd_header(lb, a, level, ts):
    out = np.empty(a.size + 64, np.uint8)
    k = lb.blosc_compress_ctx(level, 1, ts, a.size, a.ctypes.data, out.ctypes.data, out.size, b"zstd", 0, 1)
    assert k > 0
    return int(out[2]), int(out[8:12].view("<u4")[0])


def hcr_blocksize_nosplit(level, ts, nbytes):
    """c-blosc 1.21 compute_blocksize for zstd as hsds_amd restates it (engine.hip
    enc_blocksize, splittable = 0): HCR base, no split enlargement."""
    if nbytes < ts:
        return 1
    bs = nbytes
    if nbytes >= 32 * 1024:
        bs = 64 * 1024
        bs = {0: bs // 4, 1: bs // 2, 2: bs, 3: bs * 2, 4: bs * 4, 5: bs * 4}.get(level, bs * (8 if level < 9 else 16))
    bs = min(bs, nbytes)
    return bs // ts * ts if bs > ts else bs


def test_blosc_zstd_geometry_against_libblosc():
    if not os.path.exists(LIBBLOSC):
        pytest.skip("libblosc absent")
    lb = ctypes.CDLL(LIBBLOSC)
    lb.blosc_compress_ctx.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
    rng = np.random.default_rng(0)
    n = 0
    for nbytes in (200, 5000, 40000, 70000, 200000, 1 << 20, 3 << 20):
        a = np.zeros(nbytes, np.uint8)          # the geometry does not depend on the bytes
        a[::7] = rng.integers(0, 4, a[::7].size, dtype=np.uint8)
        for level in range(10):
            for ts in ((1, 2, 4, 8, 16, 17, 32) if nbytes < (1 << 20) else (1, 17)):
                flags, bs = _blosc_zstd_header(lb, a, level, ts)
                assert bs == hcr_blocksize_nosplit(level, ts, nbytes), (nbytes, level, ts, bs)
                assert flags & 0x10 and flags >> 5 == 4, (nbytes, level, ts, flags)
                n += 1
    assert n == 5 * 70 + 2 * 20


def _long_literal_runs(r):
    # random stretches (literals that run across many parse lanes) between short repeats
    parts = []
    for _ in range(12):
        parts.append(r.integers(0, 256, int(r.integers(2000, 9000)), dtype=np.uint8))
        parts.append(np.tile(np.frombuffer(b"0123456789", np.uint8), int(r.integers(1, 30))))
    return np.concatenate(parts)


@pytest.mark.parametrize("name", sorted(CASES) + ["long_literal_runs", "sparse_matches"])
@pytest.mark.parametrize("level", [1, 5])
def test_count_kernel_lane_algorithm_matches_sequence_walk(name, level):
    """zstd_count_kernel builds each frame's FSE tables from a per-lane count (the
    first match's literal run from an add scan and a max scan over the lanes), while
    encode_segment emits codes from a serial backward walk.  The kernel's per-lane algorithm
    (hze::lane_count + first_run, run lane by lane) must count exactly what the walk emits."""
    L = ctypes.CDLL(LIB)
    L.emu_zstd_counts.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    r = np.random.default_rng(11)
    if name == "long_literal_runs":
        a = _long_literal_runs(r)
    elif name == "sparse_matches":
        a = r.integers(0, 256, 200000, dtype=np.uint8)
        for k in range(0, a.size - 64, 9000):
            a[k + 32:k + 40] = a[k:k + 8]          # one 8-byte repeat per 9000 literals
    else:
        a = np.ascontiguousarray(CASES[name](r), np.uint8)
    cw = np.zeros(121, np.uint32)
    cl = np.zeros(121, np.uint32)
    nseg = L.emu_zstd_counts(a.ctypes.data if a.size else 0, a.size, level, cw.ctypes.data, cl.ctypes.data)
    assert nseg >= 1
    assert np.array_equal(cw, cl), (name, np.nonzero(cw != cl))


@pytest.mark.parametrize("name", sorted(CASES) + ["long_literal_runs"])
@pytest.mark.parametrize("level", [1, 5, 9])
def test_compact_sequence_path_writes_the_same_frames(emu, name, level):
    """zstd_seq_kernel's path (round 6): the segment's sequences extracted once into a compact
    array over its token slots and its raw literals written into the block scratch first, then
    encode_segment in seq mode -- the frames must equal the slot-walking path's byte for byte"""
    L = ctypes.CDLL(LIB)
    L.emu_zstd_set_seqs.argtypes = [ctypes.c_int]
    r = np.random.default_rng(3)
    a = _long_literal_runs(r) if name == "long_literal_runs" else np.ascontiguousarray(CASES[name](r), np.uint8)
    try:
        L.emu_zstd_set_seqs(0)
        f0 = frame(L_frame(L), a, level)
        L.emu_zstd_set_seqs(1)
        f1 = frame(L_frame(L), a, level)
    finally:
        L.emu_zstd_set_seqs(0)
    assert f0 == f1, (name, level, len(f0), len(f1))


def L_frame(L):
    L.emu_zstd_frame.restype = ctypes.c_int64
    L.emu_zstd_frame.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int]
    return L
