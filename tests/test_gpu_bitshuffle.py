"""GPU parity for bitshuffle+LZ4 objects (shuffle = 2; storUtil._unshuffle codec 2,
storUtil.py:144-174): bshuf_kernel through the C ABI against the golden frames of
tests/golden/make_bitshuffle_golden.py (expected results from liblz4 1.9.3 and
imagecodecs' bitshuffle 0.3.5 core) and against the oracle (oracle.c
orc_bitshuffle_decode / _encode).  Bit-exact."""
import hashlib
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return torch.device("cuda", 0)


def _dtype(c):
    return np.dtype("S%d" % c["itemsize"]) if c["itemsize"] not in (1, 2, 4, 8, 16) else \
        np.dtype({1: "u1", 2: "<u2", 4: "<u4", 8: "<u8", 16: "<c16"}[c["itemsize"]])


def test_unshuffle_goldens(bshuf_golden, torch_dev):
    from hsds_amd import codec
    meta, arrs = bshuf_golden
    for c in meta["cases"]:
        blob = arrs[c["name"] + "__in"].tobytes()
        dt = _dtype(c)
        shape = (c["nbytes"] // c["itemsize"],)
        if c["status"] == "error":
            with pytest.raises(codec.HTTPInternalServerError):
                codec._unshuffle(2, blob, dtype=dt, chunk_shape=shape)
            continue
        out = codec._unshuffle(2, blob, dtype=dt, chunk_shape=shape)
        assert _sha(out) == c["out_sha256"], c["name"]
        # the same through _uncompress(compressor=None, shuffle=2)
        assert codec._uncompress(blob, None, 2, None, dt, shape) == out


def test_batch_mixed_goldens_and_oracle_frames(bshuf_golden, oracle_lib, torch_dev):
    """one hsds_decode_batch over golden frames of every itemsize is not possible (one
    itemsize per call, as per dataset); per itemsize, a batch of goldens + oracle frames
    at unaligned destination offsets"""
    import torch
    from hsds_amd.engine import ChunkEngine, CHUNK_DESC_DTYPE
    meta, arrs = bshuf_golden
    eng = ChunkEngine(0)
    rng = np.random.default_rng(9)
    by_es = {}
    for c in meta["cases"]:
        by_es.setdefault(c["itemsize"], []).append((arrs[c["name"] + "__in"].tobytes(), c["nbytes"],
                                                   c["out_sha256"] if c["status"] == "ok" else None))
    for es, items in by_es.items():
        for k in range(6):
            n = int(rng.integers(1, 40000))
            raw = (np.cumsum(rng.integers(-2, 3, n * es)) % 256).astype(np.uint8).tobytes()
            block = [2048, 256, 0, 8, 64, 1024][k]
            items.append((oracle_lib.bitshuffle_encode(raw, es, block), len(raw), _sha(raw)))
        src_off, dst_off, blob = 0, 0, bytearray()
        descs = np.zeros(len(items), CHUNK_DESC_DTYPE)
        for i, (b, nb, _) in enumerate(items):
            descs[i] = (src_off, len(b), dst_off, nb)
            blob += b + b"\0" * 3
            src_off += len(b) + 3
            dst_off += nb + 5                      # unaligned destinations
        src = torch.from_numpy(np.frombuffer(bytes(blob), np.uint8).copy()).to(torch_dev)
        dst = torch.zeros(dst_off + 8, dtype=torch.uint8, device=torch_dev)
        st = torch.full((len(items),), 99, dtype=torch.int32, device=torch_dev)
        eng.decode(src, descs, dst, st, compressor=None, shuffle=2, itemsize=es)
        torch.cuda.synchronize()
        st_h, dst_h = st.cpu().numpy(), dst.cpu().numpy()
        for i, (b, nb, want) in enumerate(items):
            if want is None:
                assert st_h[i] < 0, (es, i)
                continue
            assert st_h[i] == 0, (es, i, st_h[i])
            o = int(descs[i]["dst_off"])
            assert _sha(dst_h[o:o + nb].tobytes()) == want, (es, i)


def test_outer_codec_then_bitshuffle(oracle_lib, torch_dev):
    """_uncompress(compressor, shuffle=2): the outer codec's output is the bitshuffle
    object (storUtil.py:189-227)"""
    from hsds_amd import codec
    raw = (np.arange(300000, dtype="<f4") * 0.25).tobytes()
    frame = oracle_lib.bitshuffle_encode(raw, 4, 2048)
    shape, dt = (300000,), np.dtype("<f4")
    assert codec._uncompress(zlib.compress(frame), "deflate", 2, None, dt, shape) == raw
    blosc = oracle_lib.blosc_encode(frame, typesize=1, clevel=5, shuffle=0)
    assert codec._uncompress(blosc, "gzip", 2, None, dt, shape) == raw
    with pytest.raises(codec.HTTPInternalServerError):
        codec._uncompress(zlib.compress(frame[:-4]), "deflate", 2, None, dt, shape)


def test_full_size_chunks(oracle_lib, torch_dev):
    """64 x 1 MiB f32 chunks at the HSDS default block (2048 elements): bit-exact"""
    import torch
    from hsds_amd.engine import ChunkEngine, pack_chunks
    rng = np.random.default_rng(21)
    raws, blobs = [], []
    for i in range(64):
        a = (np.cumsum(rng.standard_normal(262144)) * 0.01).astype("<f4") if i % 2 else \
            rng.integers(0, 1000, 262144).astype("<f4")
        raws.append(a.tobytes())
        blobs.append(oracle_lib.bitshuffle_encode(a.tobytes(), 4, 2048))
    src, descs, ext = pack_chunks(blobs, [1 << 20] * 64)
    eng = ChunkEngine(0)
    d_src = torch.from_numpy(src).to(torch_dev)
    d_dst = torch.zeros(ext, dtype=torch.uint8, device=torch_dev)
    st = torch.full((64,), 99, dtype=torch.int32, device=torch_dev)
    eng.decode(d_src, descs, d_dst, st, compressor=None, shuffle=2, itemsize=4)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    h = d_dst.cpu().numpy()
    for i in range(64):
        o = int(descs[i]["dst_off"])
        assert h[o:o + (1 << 20)].tobytes() == raws[i], i
