"""The oracle's bitshuffle+LZ4 restatement (oracle.c orc_bitshuffle_decode / _encode,
storUtil.py:103-131,144-174) against the golden frames of
tests/golden/make_bitshuffle_golden.py (transposition from imagecodecs' bitshuffle
0.3.5 core, LZ4 blocks from liblz4 1.9.3)."""
import hashlib

import numpy as np


def test_bitshuffle_goldens(bshuf_golden, oracle_lib):
    meta, arrs = bshuf_golden
    n_ok = n_err = 0
    for c in meta["cases"]:
        blob = arrs[c["name"] + "__in"].tobytes()
        got = oracle_lib.bitshuffle_decode(blob, c["nbytes"], c["itemsize"])
        if c["status"] == "error":
            assert isinstance(got, int) and got < 0, c["name"]
            n_err += 1
            continue
        assert not isinstance(got, int), (c["name"], got)
        assert hashlib.sha256(got).hexdigest() == c["out_sha256"], c["name"]
        n_ok += 1
    assert n_ok >= 13 and n_err >= 6


def test_bitshuffle_transposition_golden(bshuf_golden, oracle_lib):
    """the 1 MiB f32 frame's first LZ4 block decodes to the oracle's transposition"""
    meta, arrs = bshuf_golden
    raw = arrs["f4_1MiB_b2048__raw"].tobytes()
    blob = arrs["f4_1MiB_b2048__in"].tobytes()
    nb = int.from_bytes(blob[12:16], "big")
    t = oracle_lib.lz4_decode(blob[16:16 + nb], 2048 * 4)
    assert t == oracle_lib.bshuf_trans(raw[:2048 * 4], 4)


def test_bitshuffle_encode_roundtrip(oracle_lib):
    rng = np.random.default_rng(5)
    for es, n, block in ((4, 262144, 2048), (2, 1003, 256), (8, 5, 2048), (3, 999, 128), (1, 70000, 0)):
        raw = (np.arange(n * es) // 5 % 251).astype(np.uint8).tobytes() if es != 3 else \
            rng.integers(0, 256, n * es, dtype=np.uint8).tobytes()
        blob = oracle_lib.bitshuffle_encode(raw, es, block)
        assert int.from_bytes(blob[:8], "big") == len(raw)
        assert int.from_bytes(blob[8:12], "big") == block * es
        assert oracle_lib.bitshuffle_decode(blob, len(raw), es) == raw
