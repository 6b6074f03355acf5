"""Blosc frames with the bitshuffle flag (0x04), as HDF5 Blosc-filter writers produce them,
decoded the way storUtil._uncompress does through numcodecs Blosc().decode
(storUtil.py:195-208; c-blosc 1.21 blosc_d + bitunshuffle, format version 2).

Fixtures: tests/golden/make_blosc_bitshuffle_golden.py (libblosc 1.21.0 writer frames and
hand-built stored-split frames, expected outputs from the reference's _uncompress).
CPU: the oracle's restatement against every fixture.  GPU: the engine, per object
(_uncompress) and as one mixed batch (hsds_decode_batch)."""
import hashlib

import numpy as np
import pytest


def _sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def _cases(golden):
    meta, arrs = golden
    for c in meta["cases"]:
        yield c, arrs[c["name"] + "__in"].tobytes()


def test_fixture_coverage(blosc_bit_golden):
    cases = [c for c, _ in _cases(blosc_bit_golden)]
    assert len(cases) >= 40
    assert {c["typesize"] for c in cases} >= {1, 2, 3, 4, 8, 16}
    assert {c["compressor"] for c in cases} >= {"zlib", "lz4", "blosclz", "zstd"}
    assert sum(1 for c in cases if c["flags"] & 0x04 and not c["flags"] & 0x02) >= 30


def test_oracle_matches_reference(blosc_bit_golden, oracle_lib):
    orc = oracle_lib
    for c, blob in _cases(blosc_bit_golden):
        assert c["status"] == "ok", c["name"]
        out = orc.blosc_decode(blob, c["out_len"])
        assert len(out) == c["out_len"] and _sha(out) == c["out_sha256"], c["name"]


@pytest.mark.gpu
def test_gpu_uncompress_matches_reference(blosc_bit_golden, torch_dev):
    from hsds_amd import codec
    n = 0
    for c, blob in _cases(blosc_bit_golden):
        out = codec._uncompress(blob, compressor=c["compressor"], shuffle=0, dtype=np.dtype(c["dtype"]),
                                chunk_shape=tuple(c["chunk_shape"]))
        assert len(out) == c["out_len"] and _sha(out) == c["out_sha256"], c["name"]
        n += 1
    assert n >= 40


@pytest.mark.gpu
def test_gpu_batch_mixed_with_plain_frames(blosc_bit_golden, oracle_lib, torch_dev):
    """zlib bitshuffled frames batched with ordinary F1 frames: every chunk bit-exact."""
    import torch
    from hsds_amd.engine import ChunkEngine, pack_chunks
    orc = oracle_lib
    blobs, sizes, want = [], [], []
    rng = np.random.default_rng(5)
    for c, blob in _cases(blosc_bit_golden):
        if c["compressor"] != "zlib":
            continue
        blobs.append(np.frombuffer(blob, np.uint8))
        sizes.append(c["out_len"])
        want.append(c["out_sha256"])
        raw = np.round(np.cumsum(rng.normal(size=c["out_len"] // 4 + 1)), 2).astype(np.float32).tobytes()[:c["out_len"]]
        blobs.append(np.frombuffer(orc.blosc_encode(raw, typesize=1, clevel=4, shuffle=1), np.uint8))
        sizes.append(len(raw))
        want.append(_sha(raw))
    src, descs, ext = pack_chunks(blobs, sizes)
    eng = ChunkEngine(0)
    d_src = torch.from_numpy(src).to(torch_dev)
    d_dst = torch.zeros(ext, dtype=torch.uint8, device=torch_dev)
    d_st = torch.full((len(blobs),), 77, dtype=torch.int32, device=torch_dev)
    eng.decode(d_src, descs, d_dst, d_st, compressor="zlib", shuffle=0, itemsize=1)
    torch.cuda.synchronize()
    st = d_st.cpu().numpy()
    out = d_dst.cpu().numpy()
    for k in range(len(blobs)):
        assert st[k] == 0, (k, st[k])
        o = int(descs[k]["dst_off"])
        assert _sha(out[o:o + sizes[k]].tobytes()) == want[k], k


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch.device("cuda", 0)
