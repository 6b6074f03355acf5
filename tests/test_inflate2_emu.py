"""CPU emulation of the GPU two-pass inflate (hsds_amd/csrc/inflate2.h compiled with LANE_LOOP
iterating the 64 lanes) checked against libz and the oracle: the kernel's exact orchestration
(long segments, recorded-start sync, repairs, emit, batched match resolve through the match
ring, fused byte unshuffle) runs on CPU; `-m gpu` tests run the same source on the MI355X."""
import ctypes
import hashlib
import os
import subprocess
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU = os.path.join(ROOT, "tests", "emu", "libinflate2_emu.so")
SRC = os.path.join(ROOT, "tests", "emu", "inflate2_emu.cpp")
STATS = ("windows blocks stored tokens matches lanes_valid repairs repair_lanes cuts batches hops "
         "steps_a steps_e extra_windows fill_max fill_sum span_sum src_in far256 far1536 far4096 farmore hangs").split()


@pytest.fixture(scope="module")
def emu():
    # HZ2_EMU_FLAGS="-DHZ2_RGRP=4 ...": the same tests over an experiment build of the kernel
    flags = os.environ.get("HZ2_EMU_FLAGS", "").split()
    tag = hashlib.sha1(" ".join(flags).encode()).hexdigest()[:10]
    lib = EMU if not flags else os.path.join("/tmp", f"libinflate2_emu_{tag}.so")
    hdrs = [os.path.join(ROOT, "hsds_amd", "csrc", h) for h in ("inflate2.h", "inflate2_stream.inc", "inflate_wave.h")]
    if not os.path.exists(lib) or os.path.getmtime(lib) < max(os.path.getmtime(p) for p in [SRC] + hdrs):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-pthread"] + flags + ["-o", lib, SRC])
    L = ctypes.CDLL(lib)
    L.emu_inflate2.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                               ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    L.emu_inflate2_nw.argtypes = L.emu_inflate2.argtypes + [ctypes.c_int]
    return L


def run(L, comp, n, W=384, rounds=4, over16=1, perm_n=1, dst_off=0, nwaves=1):
    src = np.frombuffer(comp, np.uint8).copy()
    if src.size == 0:
        src = np.zeros(1, np.uint8)
    guard = 0xA5
    dst = np.full(max(n, 1) + dst_off + 8, guard, np.uint8)
    st = np.zeros(len(STATS), np.uint64)
    r = L.emu_inflate2_nw(src.ctypes.data, len(comp), dst.ctypes.data, n, W, rounds, over16, perm_n, dst_off,
                          st.ctypes.data, nwaves)
    assert (dst[:dst_off] == guard).all() and (dst[dst_off + n:] == guard).all(), "write outside the output"
    return r, dst[dst_off:dst_off + n].tobytes(), dict(zip(STATS, st.tolist()))


def corpus():
    rng = np.random.default_rng(123)
    sm = np.round(np.cumsum(rng.normal(size=80000)), 2).astype(np.float32).tobytes()
    return {
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


@pytest.mark.parametrize("level", [0, 1, 4, 6, 9])
def test_levels_match_zlib(emu, level):
    for name, data in corpus().items():
        c = zlib.compress(data, level)
        r, out, _ = run(emu, c, len(data))
        assert r == 0, (name, level, r)
        assert out == data, (name, level)


@pytest.mark.parametrize("strategy", [zlib.Z_FILTERED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FIXED])
def test_strategies(emu, strategy):
    for name, data in corpus().items():
        co = zlib.compressobj(5, zlib.DEFLATED, 15, 8, strategy)
        c = co.compress(data) + co.flush()
        r, out, _ = run(emu, c, len(data))
        assert r == 0 and out == data, (name, strategy, r)


def test_small_window_bits_and_memlevel(emu):
    data = corpus()["text"] * 3
    for wbits, mem in ((9, 1), (10, 9), (12, 4), (15, 1)):
        co = zlib.compressobj(6, zlib.DEFLATED, wbits, mem)
        c = co.compress(data) + co.flush()
        r, out, _ = run(emu, c, len(data))
        assert r == 0 and out == data, (wbits, mem)


@pytest.mark.parametrize("W,rounds,over16", [(0, 0, 0), (0, 8, 0), (64, 1, 4), (384, 4, 1), (1024, 2, 8)])
def test_tunings_do_not_change_output(emu, W, rounds, over16):
    """no warm-up / no repairs / over-provisioned segments only change the work split"""
    for name in ("smooth_f32", "smooth_f32_shuffled", "zeros", "text", "runs"):
        data = corpus()[name]
        c = zlib.compress(data, 4)
        r, out, _ = run(emu, c, len(data), W=W, rounds=rounds, over16=over16)
        assert r == 0 and out == data, (name, W, rounds, over16)


def test_repairs_and_cuts_are_exercised(emu):
    """W = 0 forces unsynced lanes (repairs); zeros force the per-lane match cap (cuts)"""
    data = corpus()["smooth_f32"]
    r, out, st = run(emu, zlib.compress(data, 4), len(data), W=0, rounds=64)
    assert r == 0 and out == data and st["repairs"] > 0
    z = bytes(1 << 20)
    r, out, st = run(emu, zlib.compress(z, 9), len(z))
    assert r == 0 and out == z


def test_hsds_f1_stream_stats(emu):
    """a 256 KiB split of the bench's smooth f32 chunk: one decode pass (HZ2_FUSE: phase A emits,
    no phase E) whose warm-ups stay small (about 2.3 tokens per match here), one window per
    block (plus at most one extra), few repairs"""
    import sys
    sys.path.insert(0, ROOT)
    from bench import smooth_chunk
    raw = smooth_chunk(20261015).view(np.uint8)[:262144].tobytes()
    c = zlib.compress(raw, 4)
    r, out, st = run(emu, c, len(raw))
    assert r == 0 and out == raw
    assert st["windows"] <= st["blocks"] + 2
    assert st["steps_e"] == 0 and st["steps_a"] < 2.7 * st["matches"]
    assert st["repair_lanes"] < 0.05 * st["lanes_valid"]


def test_fused_unshuffle(emu):
    """F2: the inflated byte planes land unshuffled (numcodecs.Shuffle.decode) for itemsizes
    2..16, including a tail that is not a whole element"""
    rng = np.random.default_rng(5)
    for n in (2, 3, 4, 8, 16):
        for count, tail in ((4096, 0), (1001, 0), (777, 0)):
            arr = (np.cumsum(rng.normal(size=count * n)) * 50).astype(np.int64).astype(np.uint8)
            want = arr.tobytes()
            shuffled = arr.reshape(-1, n).T.copy().tobytes()
            r, out, _ = run(emu, zlib.compress(shuffled, 4), len(want), perm_n=n)
            assert r == 0 and out == want, (n, count)
    # a span that is not a multiple of n: trailing bytes are copied as they are
    data = bytes(rng.integers(0, 4, 4003, dtype=np.uint8))
    body = 4003 // 4 * 4
    shuffled = np.frombuffer(data[:body], np.uint8).reshape(-1, 4).T.copy().tobytes() + data[body:]
    r, out, _ = run(emu, zlib.compress(shuffled, 6), len(data), perm_n=4)
    assert r == 0 and out == data


def test_corruptions_fail_like_libz(emu):
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as orc
    rng = np.random.default_rng(9)
    base = corpus()["smooth_f32"][:40000]
    good = zlib.compress(base, 4)
    for t in range(200):
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
        r, out, _ = run(emu, bytes(b), n)
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
    rng = np.random.default_rng(77)
    fib = [1, 1]
    while len(fib) < 40:
        fib.append(fib[-1] + fib[-2])
    lits = np.concatenate([np.full(min(f, 20000), s % 256, np.uint8) for s, f in enumerate(fib[:24])])
    rare = rng.permutation(256).astype(np.uint8)
    data = np.concatenate([rng.permutation(lits), rare]).tobytes()
    parts = [data]
    for k, f in enumerate(fib[:20]):
        d = 1 + (k * 1543) % 30000
        parts.append(data[-d:][:8] * max(1, min(f, 50)))
    data = b"".join(parts)[:400000]
    for level in (1, 6, 9):
        comp = zlib.compress(data, level)
        r, out, _ = run(emu, comp, len(data))
        assert r == 0 and out == data, (level, r)


@pytest.mark.parametrize("off", [1, 2, 3, 5])
def test_unaligned_output(emu, off):
    """the resolve's dword path at every output alignment (the first / last dwords of the
    stream reach outside it and must be written bytewise), plain and unshuffled output"""
    for name in ("smooth_f32", "text", "runs", "zeros"):
        data = corpus()[name][:50001]
        c = zlib.compress(data, 6)
        r, out, _ = run(emu, c, len(data), dst_off=off)
        assert r == 0 and out == data, (name, off)
    data = corpus()["int16"][:40000]
    shuffled = np.frombuffer(data, np.uint8).reshape(-1, 2).T.copy().tobytes()
    r, out, _ = run(emu, zlib.compress(shuffled, 4), len(data), perm_n=2, dst_off=off)
    assert r == 0 and out == data


def test_long_overlapping_matches_and_far_distances(emu):
    """matches whose sources overlap themselves (distance < length) and chains of matches
    inside one resolve batch, plus distances up to 32 KiB"""
    rng = np.random.default_rng(3)
    pat = rng.integers(0, 256, 40000, dtype=np.uint8).tobytes()
    data = b"".join([b"ab" * 300, pat[:5000], b"xyz" * 1000, pat[:32000], pat[100:20000], b"\x00" * 70000,
                     pat[:32768] + pat[:32768]])
    for level in (1, 9):
        c = zlib.compress(data, level)
        r, out, _ = run(emu, c, len(data))
        assert r == 0 and out == data, level


# ---- two and four wavefronts per stream (inflate2w_kernel's window pipeline, one thread each) ----
@pytest.mark.parametrize("nw", [2, 4, 8])
@pytest.mark.parametrize("level", [0, 1, 4, 9])
def test_two_wavefronts_match_zlib(emu, level, nw):
    for name, data in corpus().items():
        c = zlib.compress(data, level)
        r, out, st = run(emu, c, len(data), nwaves=nw)
        assert r == 0, (name, level, r)
        assert out == data, (name, level)


@pytest.mark.parametrize("nw", [2, 4, 8])
def test_two_wavefronts_strategies_and_stored_blocks(emu, nw):
    for strategy in (zlib.Z_FILTERED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FIXED):
        for name in ("smooth_f32", "text", "random", "runs"):
            data = corpus()[name]
            co = zlib.compressobj(5, zlib.DEFLATED, 15, 8, strategy)
            c = co.compress(data) + co.flush()
            r, out, _ = run(emu, c, len(data), nwaves=nw)
            assert r == 0 and out == data, (name, strategy, r)
    # many small blocks of each type: a full flush after every piece
    rng = np.random.default_rng(4)
    co = zlib.compressobj(6)
    data, c = b"", b""
    for i in range(60):
        piece = rng.integers(0, 256 if i % 3 == 0 else 4, int(rng.integers(1, 3000)), dtype=np.uint8).tobytes()
        data += piece
        c += co.compress(piece) + co.flush(zlib.Z_FULL_FLUSH)
    c += co.flush()
    for n in (1, nw):
        r, out, st = run(emu, c, len(data), nwaves=n)
        assert r == 0 and out == data, n
    assert st["stored"] > 0


@pytest.mark.parametrize("nw", [2, 4, 8])
def test_two_wavefronts_continuation_windows_and_f1_stream(emu, nw):
    """one block over several windows (the continuation copies the other wavefront's tables),
    and a 256 KiB split of the bench chunk (7 blocks: both wavefronts alternate)"""
    import sys
    sys.path.insert(0, ROOT)
    from bench import smooth_chunk
    raw = smooth_chunk(20261015).view(np.uint8)[:262144].tobytes()
    r, out, st = run(emu, zlib.compress(raw, 4), len(raw), nwaves=nw)
    assert r == 0 and out == raw and st["windows"] >= st["blocks"]
    z = bytes(1 << 20)
    r, out, st = run(emu, zlib.compress(z, 9), len(z), nwaves=nw)
    assert r == 0 and out == z
    data = corpus()["smooth_f32"]
    r, out, st = run(emu, zlib.compress(data, 4), len(data), over16=0, W=64, nwaves=nw)
    assert r == 0 and out == data


@pytest.mark.parametrize("nw", [2, 4, 8])
@pytest.mark.parametrize("off", [1, 3])
def test_two_wavefronts_unaligned_output(emu, off, nw):
    data = corpus()["smooth_f32"][:50001]
    r, out, _ = run(emu, zlib.compress(data, 4), len(data), dst_off=off, nwaves=nw)
    assert r == 0 and out == data


@pytest.mark.parametrize("nw", [2, 4, 8])
def test_two_wavefronts_corruptions_fail_like_libz(emu, nw):
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as orc
    rng = np.random.default_rng(19)
    base = corpus()["smooth_f32"][:60000]
    good = zlib.compress(base, 4)
    for t in range(120):
        b = bytearray(good)
        k = t % 4
        if k == 0:
            b = b[:int(rng.integers(1, len(b)))]
        elif k == 1:
            i = int(rng.integers(0, len(b)))
            b[i] ^= 1 << int(rng.integers(0, 8))
        elif k == 2:
            b[-1 - int(rng.integers(0, 4))] ^= 0x40
        else:
            b = b + bytes(rng.integers(0, 256, 5, dtype=np.uint8))
        n = len(base)
        ref = orc.uncompress(bytes(b), "zlib", 0, 1, n)
        r, out, _ = run(emu, bytes(b), n, nwaves=nw)
        if isinstance(ref, int):
            assert r < 0 and r != -100, (t, k, ref, r)
        else:
            assert r == 0 and out == ref, (t, k, r)
    data = corpus()["text"]
    c = zlib.compress(data, 4)
    assert run(emu, c, len(data) - 1, nwaves=nw)[0] not in (0, -100)
    assert run(emu, c, len(data) + 1, nwaves=nw)[0] not in (0, -100)


@pytest.mark.parametrize("nw", [2, 4, 8])
def test_pipeline_timeout_redecodes_with_one_wavefront(emu, nw):
    """A window-pipeline wait that gives up (Tune::spin_max; inflate2.h inflate_stream /
    inflate_stream_pipe) is not reported as corrupt data: wavefront 0 decodes the stream
    again alone, so valid streams still come out bit-exact and corrupt ones keep libz's
    verdict.  spin_max = 1 makes nearly every wait give up."""
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as orc
    emu.emu_set_spin_max.argtypes = [ctypes.c_uint32]
    emu.emu_set_spin_max(1)
    try:
        hangs = 0
        for name, data in corpus().items():
            c = zlib.compress(data, 4)
            r, out, st = run(emu, c, len(data), nwaves=nw)
            assert r == 0 and out == data, (name, r)
            hangs += st["hangs"]
        rng = np.random.default_rng(5)
        base = corpus()["smooth_f32"][:60000]
        good = zlib.compress(base, 4)
        for t in range(24):
            b = bytearray(good)
            i = int(rng.integers(0, len(b)))
            b[i] ^= 1 << int(rng.integers(0, 8))
            ref = orc.uncompress(bytes(b), "zlib", 0, 1, len(base))
            r, out, _ = run(emu, bytes(b), len(base), nwaves=nw)
            r1, _, _ = run(emu, bytes(b), len(base), nwaves=1)
            if isinstance(ref, int):
                assert r < 0 and r != -100 and r == r1, (t, ref, r, r1)
            else:
                assert r == 0 and out == ref, (t, r)
        assert hangs > 0, "the forced timeouts never fired"
    finally:
        emu.emu_set_spin_max(0)


@pytest.mark.parametrize("nw", [1, 2])
def test_long_literal_runs_before_matches(emu, nw):
    """Literal runs of 1..3000 random bytes, each followed by a repeat of earlier bytes, at
    several levels: runs that cross many lanes' segments before a match (the round-5
    4-byte-record experiment's escape path; kept as a regression case for any record
    format)."""
    rng = np.random.default_rng(21)
    parts = []
    for n in (1, 100, 509, 510, 511, 512, 513, 1000, 1023, 1024, 2047, 3000, 5, 511, 600):
        parts.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        parts.append(parts[-1][: max(1, min(n, 40))] * 3)          # a match (or several) after the run
    data = b"".join(parts) * 3
    for level in (1, 6, 9):
        c = zlib.compress(data, level)
        r, out, st = run(emu, c, len(data), nwaves=nw)
        assert r == 0 and out == data, (level, r)
        assert st["matches"] > 0


def _alphabet_cases():
    """streams whose dynamic headers exercise every code-length symbol: sparse alphabets
    (zero runs: symbols 17 and 18), skewed ones (repeats of the previous length: 16),
    dense ones (two literal lengths per lookup of the header's two-symbol LUT), long and
    short distance alphabets"""
    rng = np.random.default_rng(2026)
    out = []
    for k in range(48):
        nsym = int(rng.choice([2, 3, 5, 9, 17, 40, 90, 160, 256]))
        alpha = rng.choice(256, nsym, replace=False).astype(np.uint8)
        p = rng.dirichlet(np.full(nsym, float(rng.choice([0.05, 0.3, 1.0, 5.0]))))
        data = alpha[rng.choice(nsym, int(rng.integers(300, 40000)), p=p)]
        if k % 3 == 0:        # repeats at many distances
            reps = [data[i:i + 40] for i in rng.integers(0, max(1, data.size - 40), 200)]
            data = np.concatenate([data] + reps)
        out.append(data.tobytes())
    return out


def test_dynamic_headers_all_code_length_symbols(emu):
    for k, data in enumerate(_alphabet_cases()):
        for level in (1, 6, 9):
            c = zlib.compress(data, level)
            r, out, _ = run(emu, c, len(data))
            assert r == 0 and out == data, (k, level, r)


def test_dynamic_header_corruptions_match_zlib(emu):
    """bit flips inside the first dynamic header (HLIT / HDIST / HCLEN, the code-length code,
    the code lengths): the emulator must accept exactly what zlib accepts, bit-exact"""
    rng = np.random.default_rng(7)
    data = _alphabet_cases()[5]
    c = bytearray(zlib.compress(data, 6))
    for t in range(160):
        b = bytearray(c)
        bit = int(rng.integers(19, min(len(b) * 8, 19 + 600)))    # after the zlib header and BFINAL/BTYPE
        b[bit // 8] ^= 1 << (bit % 8)
        try:
            ref = zlib.decompress(bytes(b))
        except zlib.error:
            ref = None
        r, out, _ = run(emu, bytes(b), len(data))
        if ref is not None and len(ref) == len(data):
            assert r == 0 and out == ref, (t, bit, r)
        else:
            assert r != 0, (t, bit)
