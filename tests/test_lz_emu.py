"""CPU emulation of the GPU LZ4 / BloscLZ split decoder (hsds_amd/csrc/lz_wave.h compiled
with LANE_LOOP iterating the 64 lanes): every lz4 / lz4hc / blosclz golden object of the
reference (tests/golden/codec2_cases.*) and randomized streams that exercise window
splits, long literal runs past the 4 KiB stage, overlapping matches and extension bytes,
checked against the CPU oracle (oracle/oracle.c) and the reference's sha256."""
import ctypes
import hashlib
import os
import struct
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU = os.path.join(ROOT, "tests", "emu", "liblz_emu.so")
SRC = os.path.join(ROOT, "tests", "emu", "lz_emu.cpp")


@pytest.fixture(scope="module")
def emu():
    hdrs = [os.path.join(ROOT, "hsds_amd", "csrc", h) for h in ("lz_wave.h", "inflate_wave.h")]
    if not os.path.exists(EMU) or os.path.getmtime(EMU) < max(os.path.getmtime(p) for p in [SRC] + hdrs):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", EMU, SRC])
    L = ctypes.CDLL(EMU)
    L.emu_lz_stream.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
    return L


def split(L, comp, n, fmt):
    src = np.frombuffer(comp, np.uint8).copy() if len(comp) else np.zeros(1, np.uint8)
    dst = np.zeros(max(n, 1), np.uint8)
    r = L.emu_lz_stream(src.ctypes.data, len(comp), dst.ctypes.data, n, fmt)
    return r, dst[:n].tobytes()


def frame_decode(L, f):
    """Blosc1 frame walk (same rules as oracle.c orc_blosc_decode) with every lz4 /
    blosclz split decoded by the emulated wave decoder.  Returns bytes or a status."""
    if len(f) < 16:
        return -1
    flags, ts = f[2], f[3]
    nb, bs, cb = struct.unpack("<III", f[4:16])
    if cb > len(f):
        return -1
    if flags & 2:
        return f[16:16 + nb]
    codec = flags >> 5
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
                r, d = split(L, f[p:p + cs], ne, codec)
                if r != 0:
                    return r
                blk += d
            p += cs
        if flags & 1 and ts > 1:
            cnt = bsz // ts
            blk = np.frombuffer(bytes(blk[:cnt * ts]), np.uint8).reshape(ts, cnt).T.tobytes() + bytes(blk[cnt * ts:])
        out += blk
    return bytes(out)


def test_reference_goldens(emu, golden2):
    meta, arrs = golden2
    checked = 0
    for c in meta["cases"]:
        if c["codec"] not in (0, 1):
            continue                      # zstd: outside the engine
        blob = arrs[c["name"] + "__in"].tobytes()
        got = frame_decode(emu, blob)
        if c["status"] == "error" or c["name"].endswith("_trunc"):
            assert isinstance(got, int), c["name"]
            continue
        assert not isinstance(got, int), (c["name"], got)
        assert hashlib.sha256(got).hexdigest() == c["out_sha256"], c["name"]
        checked += 1
    assert checked >= 40


# ---- randomized streams (tiny writers of each format) ------------------------------

def lz4_write(rng, n_out):
    """A valid LZ4 block of about n_out bytes with random literal runs (some past 4 KiB),
    overlapping matches (distance < length) and long extension bytes."""
    out, seq = bytearray(), bytearray()

    def ext(v):
        b = bytearray()
        while v >= 255:
            b.append(255)
            v -= 255
        b.append(v)
        return b
    while len(out) < n_out:
        r = rng.random()
        lit = int(rng.integers(0, 16)) if r < 0.6 else int(rng.integers(16, 300)) if r < 0.95 else int(rng.integers(4000, 9000))
        ml = int(rng.integers(4, 19)) if rng.random() < 0.8 else int(rng.integers(19, 3000))
        lits = rng.integers(0, 256, lit, dtype=np.uint8).tobytes()
        if len(out) + lit == 0:
            lit, lits = 1, b"\x07"
        dist_max = min(len(out) + lit, 65535)
        d = int(rng.integers(1, dist_max + 1)) if rng.random() < 0.7 else int(rng.integers(1, min(8, dist_max) + 1))
        tok = (min(lit, 15) << 4) | min(ml - 4, 15)
        seq.append(tok)
        if lit >= 15:
            seq += ext(lit - 15)
        seq += lits
        seq += struct.pack("<H", d)
        if ml - 4 >= 15:
            seq += ext(ml - 4 - 15)
        out += lits
        for k in range(ml):
            out.append(out[len(out) - d])
    tail = rng.integers(0, 256, int(rng.integers(5, 40)), dtype=np.uint8).tobytes()
    lit = len(tail)
    seq.append(min(lit, 15) << 4)
    if lit >= 15:
        seq += ext(lit - 15)
    seq += tail
    out += tail
    return bytes(seq), bytes(out)


def blosclz_write(rng, n_out):
    out, s = bytearray(), bytearray()
    first = True
    while len(out) < n_out:
        if first or rng.random() < 0.5 or len(out) == 0:
            n = int(rng.integers(1, 33))
            lits = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            s.append(n - 1)
            s += lits
            out += lits
            first = False
            continue
        ln = int(rng.integers(3, 9)) if rng.random() < 0.7 else int(rng.integers(9, 2000))
        far = rng.random() < 0.2 and len(out) > 8192
        d = int(rng.integers(8192, min(len(out), 8192 + 65535) + 1)) if far else \
            int(rng.integers(1, min(len(out), 8191) + 1))
        c_len = min(ln - 2, 7)
        if far:
            ofs, code = 31 << 8, 255
        else:
            ofs, code = ((d - 1) >> 8) << 8, (d - 1) & 255
            if ofs == (31 << 8) and code == 255:
                continue                  # not encodable in the short form
        s.append((c_len << 5) | (ofs >> 8))
        if c_len == 7:
            v = ln - 9
            while v >= 255:
                s.append(255)
                v -= 255
            s.append(v)
        s.append(code)
        if far:
            s += struct.pack(">H", d - 8192)
        for k in range(ln):
            out.append(out[len(out) - d])
    return bytes(s), bytes(out)


@pytest.mark.parametrize("seed", range(12))
def test_random_lz4_streams(emu, oracle_lib, seed):
    rng = np.random.default_rng(seed)
    comp, raw = lz4_write(rng, int(rng.integers(1, 200000)))
    assert oracle_lib.lz4_decode(comp, len(raw)) == raw
    r, got = split(emu, comp, len(raw), 1)
    assert r == 0 and got == raw


@pytest.mark.parametrize("seed", range(12))
def test_random_blosclz_streams(emu, oracle_lib, seed):
    rng = np.random.default_rng(100 + seed)
    comp, raw = blosclz_write(rng, int(rng.integers(1, 150000)))
    assert oracle_lib.blosclz_decode(comp, len(raw)) == raw
    r, got = split(emu, comp, len(raw), 0)
    assert r == 0 and got == raw


def test_corrupt_streams_fail_like_the_oracle(emu, oracle_lib):
    rng = np.random.default_rng(5)
    for fmt, writer, dec in ((1, lz4_write, oracle_lib.lz4_decode), (0, blosclz_write, oracle_lib.blosclz_decode)):
        comp, raw = writer(rng, 20000)
        for k in range(60):
            bad = bytearray(comp)
            pos = int(rng.integers(0, len(bad)))
            bad[pos] ^= int(rng.integers(1, 256))
            bad = bytes(bad) if k % 7 else bytes(bad[:int(rng.integers(1, len(bad)))])
            want = dec(bad, len(raw))
            r, got = split(emu, bad, len(raw), fmt)
            if isinstance(want, int):
                assert r != 0, (fmt, k)
            else:
                assert r == 0 and got == want, (fmt, k)


def _ext(v):
    return bytes([255] * (v // 255) + [v % 255])


def test_headers_longer_than_the_stage(emu, oracle_lib):
    """LZ4 / BloscLZ items whose length-extension bytes exceed the 4 KiB LDS stage
    (runs of several MB): the parser falls back to global reads for that item."""
    rng = np.random.default_rng(9)
    # LZ4: 2 MB literal run, then a 3 MB overlapping match (distance 1), then 6 literals
    lits = rng.integers(0, 256, 2_000_000, dtype=np.uint8).tobytes()
    tail = b"abcdef"
    ml = 3_000_000
    comp = (bytes([0xFF]) + _ext(len(lits) - 15) + lits + struct.pack("<H", 1) + _ext(ml - 4 - 15)
            + bytes([len(tail) << 4]) + tail)
    raw = lits + lits[-1:] * ml + tail
    assert oracle_lib.lz4_decode(comp, len(raw)) == raw
    r, got = split(emu, comp, len(raw), 1)
    assert r == 0 and got == raw
    # BloscLZ: 3 literals, then a 2 MB match of distance 3
    ln = 2_000_000
    comp = bytes([2]) + b"xyz" + bytes([7 << 5]) + _ext(ln - 9) + bytes([2])
    raw = b"xyz" * ((ln + 3) // 3 + 1)
    raw = raw[:3 + ln]
    assert oracle_lib.blosclz_decode(comp, len(raw)) == raw
    r, got = split(emu, comp, len(raw), 0)
    assert r == 0 and got == raw


def test_group_of_splits_shares_the_resolve(emu, oracle_lib):
    """Up to 64 splits decoded together (mixed formats, sizes, corrupt ones): the
    resolve interleaves every split's 16-byte groups across the lanes."""
    emu.emu_lz_group.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    rng = np.random.default_rng(21)
    for n in (64, 37, 1):
        comps, raws, fmts = [], [], []
        for i in range(n):
            fmt = int(rng.integers(0, 2))
            comp, raw = (lz4_write if fmt else blosclz_write)(rng, int(rng.integers(1, 30000)))
            if i % 9 == 4:
                b = bytearray(comp)
                b[int(rng.integers(0, len(b)))] ^= 0x5A
                comp = bytes(b)
            comps.append(np.frombuffer(comp, np.uint8).copy())
            raws.append(raw)
            fmts.append(fmt)
        # destinations at odd offsets of one buffer: unaligned dword groups
        offs = np.cumsum([0] + [len(r) + 3 for r in raws])
        out = np.zeros(int(offs[-1]) + 16, np.uint8)
        src_p = (ctypes.c_void_p * n)(*[c.ctypes.data for c in comps])
        dst_p = (ctypes.c_void_p * n)(*[out.ctypes.data + int(offs[i]) + 1 for i in range(n)])
        slen = np.array([len(c) for c in comps], np.uint32)
        dlen = np.array([len(r) for r in raws], np.uint32)
        fm = np.array(fmts, np.uint32)
        st = np.zeros(n, np.int32)
        emu.emu_lz_group(src_p, slen.ctypes.data, dst_p, dlen.ctypes.data, fm.ctypes.data, n, st.ctypes.data)
        for i in range(n):
            dec = oracle_lib.lz4_decode if fmts[i] else oracle_lib.blosclz_decode
            want = dec(comps[i].tobytes(), len(raws[i]))
            if isinstance(want, int):
                assert st[i] != 0, (n, i)
            else:
                o = int(offs[i]) + 1
                assert st[i] == 0 and out[o:o + len(raws[i])].tobytes() == want, (n, i)
