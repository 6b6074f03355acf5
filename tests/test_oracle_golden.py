"""Pin the CPU oracle (oracle/oracle.c) against the reference's own outputs.

The fixtures under tests/golden/ were produced by the reference's storUtil._compress /
_uncompress (hsds/util/storUtil.py:182-281) running over libblosc 1.21.0 + zlib 1.2.11
(tests/golden/make_golden.py).  The oracle must reproduce every decoded byte and every
error, and its Blosc encoder must reproduce the reference's F1 objects byte-for-byte.
"""
import hashlib

import numpy as np
import pytest


def _sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def _cases(golden):
    meta, arrs = golden
    for c in meta["cases"]:
        yield c, arrs[c["name"] + "__in"].tobytes(), arrs.get(c["name"] + "__out")


def test_uncompress_matches_reference(golden, oracle_lib):
    orc = oracle_lib
    n = 0
    for c, blob, out_arr in _cases(golden):
        itemsize = np.dtype(c["dtype"]).itemsize if c["dtype"] else 1
        expected = int(np.prod(c["chunk_shape"])) * itemsize
        got = orc.uncompress(blob, c["compressor"], c["shuffle"], itemsize, expected)
        if c["status"] == "error":
            assert isinstance(got, int) and got < 0, c["name"]
            continue
        assert not isinstance(got, int), (c["name"], got)
        assert len(got) == c["out_len"] and _sha(got) == c["out_sha256"], c["name"]
        if out_arr is not None:
            assert got == out_arr.tobytes(), c["name"]
        n += 1
    assert n >= 25


def test_uncompress_other_blosc_codecs(golden2, oracle_lib):
    """lz4 / lz4hc / blosclz / zstd objects written by the reference's _compress (and
    typesize>1 frames, and corrupted ones): every decoded byte and every error.  A
    truncated object is rejected where the reference reads past its end (DESIGN.md
    deviations)."""
    orc = oracle_lib
    checked = 0
    for c, blob, out_arr in _cases(golden2):
        itemsize = np.dtype(c["dtype"]).itemsize
        expected = int(np.prod(c["chunk_shape"])) * itemsize
        got = orc.uncompress(blob, c["compressor"], c["shuffle"], itemsize, expected)
        if c["status"] == "error" or c["name"].endswith("_trunc"):
            assert isinstance(got, int) and got < 0, c["name"]
            continue
        assert not isinstance(got, int), (c["name"], got)
        assert len(got) == c["out_len"] and _sha(got) == c["out_sha256"], c["name"]
        if out_arr is not None:
            assert got == out_arr.tobytes(), c["name"]
        checked += 1
    assert checked >= 90


def test_blosc_encoder_is_byte_identical_to_reference(golden, oracle_lib):
    """storUtil._compress always builds Blosc(cname='zlib') over a bytes object, so
    typesize is 1; the oracle's frame writer must emit the
    same bytes as the reference for those cases."""
    orc = oracle_lib
    checked = 0
    for c, blob, _ in _cases(golden):
        if c["status"] != "ok" or not c["note"].startswith("reference _compress"):
            continue
        if not orc.is_blosc(blob):
            continue
        itemsize = np.dtype(c["dtype"]).itemsize
        raw = orc.uncompress(blob, c["compressor"], c["shuffle"], itemsize, c["out_len"])
        enc = orc.blosc_encode(raw, typesize=1, clevel=c["level"], shuffle=c["shuffle"])
        assert enc == blob, c["name"]
        checked += 1
    assert checked >= 8


def test_blosc_header_fields(golden, oracle_lib):
    orc = oracle_lib
    for c, blob, _ in _cases(golden):
        if c["status"] != "ok" or not orc.is_blosc(blob):
            continue
        hdr = np.frombuffer(blob[:16], np.uint8)
        nbytes, bs, cbytes = np.frombuffer(blob[4:16], "<u4")
        assert hdr[0] == 2 and hdr[1] == 1, c["name"]
        assert nbytes == c["out_len"] and cbytes == len(blob), c["name"]
        if not hdr[2] & 0x02 and c["note"].startswith("reference _compress") and c["level"]:
            assert bs == orc.blosc_blocksize(c["level"], hdr[3], nbytes), c["name"]


def test_shuffle_kat(golden, oracle_lib):
    orc = oracle_lib
    meta, _ = golden
    kat = meta["shuffle_kat"]          # hsds/tests/unit/shuffle_test.py:26-41
    data = bytes.fromhex(kat["in"])
    assert orc.shuffle(data, 2).hex() == kat["shuffled"]
    assert orc.unshuffle(bytes.fromhex(kat["shuffled"]), 2).hex() == kat["unshuffled"]
    for c in meta["shuffle_cases"]:
        n = np.dtype(c["dtype"]).itemsize
        data = bytes.fromhex(c["in"])
        assert orc.shuffle(data, n).hex() == c["shuffled"]
        assert orc.unshuffle(bytes.fromhex(c["shuffled"]), n) == data


def test_batch_matches_single(oracle_lib):
    orc = oracle_lib
    rng = np.random.default_rng(5)
    raw = [np.round(np.cumsum(rng.normal(size=16384)), 2).astype(np.float32).view(np.uint8)
           for _ in range(6)]
    blobs = orc.encode_batch(raw, op="blosc", typesize=1, clevel=4, shuffle=1, nthreads=3)
    for r, b in zip(raw, blobs):
        assert bytes(b) == orc.blosc_encode(r, 1, 4, 1)
    outs, st = orc.uncompress_batch(blobs, [r.size for r in raw], "zlib", 1, 4, nthreads=3)
    assert (st == raw[0].size).all()
    for r, o in zip(raw, outs):
        assert np.array_equal(np.asarray(o)[:r.size], r)


@pytest.mark.parametrize("level", [1, 4, 9])
def test_zlib_roundtrip(oracle_lib, level):
    import zlib
    data = np.random.default_rng(level).integers(0, 7, 50000, dtype=np.uint8).tobytes()
    c = oracle_lib.zlib_encode(data, level)
    assert zlib.decompress(c) == data
    assert oracle_lib.uncompress(c, "zlib", 0, 1, len(data)) == data
    assert oracle_lib.adler32(data) == zlib.adler32(data)


def test_blosc_header_rule_all_codecs(golden2, oracle_lib):
    """c-blosc 1.21 compute_blocksize and the dont-split flag for lz4 / lz4hc /
    blosclz / zlib frames: 960 headers written by libblosc 1.21.0."""
    meta, _ = golden2
    rows = meta["headers"]
    assert len(rows) >= 900
    for r in rows:
        bs = oracle_lib.blosc_blocksize_codec(r["clevel"], r["typesize"], r["nbytes"], r["cname"])
        assert bs == r["blocksize"], r
        ts = r["typesize"] if r["typesize"] <= 255 else 1
        split = ts <= 16 and bs // ts >= 128
        assert bool(r["flags"] & 0x10) == (not split), r
